"""Worker of tests/test_gpu_data.py (a fresh process in deterministic mode): batches of an on-disk
DDAD-layout dataset through `DevicePrefetcher` vs the same batches as host tensors, through the
fusion step; prints one JSON line listing every difference."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE, os.path.join(HERE, 'golden')]

import torch  # noqa: E402

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False


def main(tmp):
    import common as G
    import data_fake
    from vfdepth_amd import _lib
    from vfdepth_amd import data as D
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    _lib.load()
    dev = torch.device('cuda:0')
    cfg = G.step_cfg()                               # 96x160, reduced voxels
    path, _, _ = data_fake.write_ddad(tmp, h=192, w=320, n_samples=5)
    cfg['data']['data_path'] = path
    cfg['data']['mask_path'] = D.ALL_ONES_MASK
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
    algo.set_train()
    loader = torch.utils.data.DataLoader(D.construct_dataset(cfg, 'val', **D.augmentation(cfg, 'val')),
                                         batch_size=1, shuffle=False, pin_memory=True)
    host = [dict(b) for b in loader]
    noise = torch.zeros(6, 1, 2, 96, 160, device=dev)
    with torch.no_grad():
        algo.process_batch(dict(host[0]), 0, noise=noise)      # warm-up (MIOpen's first-use work)
    out = {'batches': 0, 'input_diff': [], 'loss_diff': {}, 'depth_diff': [], 'finite': True}
    for i, dev_batch in enumerate(D.DevicePrefetcher(loader, dev)):
        out['batches'] += 1
        assert dev_batch[('color', 0, 0)].is_cuda and dev_batch[('K', 0)].dtype == torch.float32
        for k, v in host[i].items():
            if torch.is_tensor(v) and v.is_floating_point() and not torch.equal(dev_batch[k].cpu(), v.float()):
                out['input_diff'].append(str(k))
        with torch.no_grad():
            # alternate which path runs first: any state carried between steps would show up
            if i % 2:
                out_h, loss_h = algo.process_batch(dict(host[i]), 0, noise=noise)
                out_d, loss_d = algo.process_batch(dev_batch, 0, noise=noise)
            else:
                out_d, loss_d = algo.process_batch(dev_batch, 0, noise=noise)
                out_h, loss_h = algo.process_batch(dict(host[i]), 0, noise=noise)
        for k in loss_h:
            if not torch.equal(loss_d[k], loss_h[k]):
                out['loss_diff'][f'{i}:{k}'] = (float(loss_d[k]), float(loss_h[k]))
        for c in range(6):
            if not torch.equal(out_d[('cam', c)][('depth', 0)], out_h[('cam', c)][('depth', 0)]):
                out['depth_diff'].append(f'{i}:{c}')
        out['finite'] &= bool(torch.isfinite(loss_d['total_loss']))
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main(sys.argv[1])
