"""Worker of test_deterministic_steps_bit_identical (tests/test_gpu_parity.py): a fresh process,
so MIOpen reads MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC before its first convolution.  Runs two
eager training steps of the reduced fusion config from the same state under
torch.backends.cudnn.deterministic and prints one JSON line comparing them bit for bit."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, 'golden')]

# MIOpen's deterministic switch selects among its deterministic solvers, but a find-db record (the
# committed tuned picks include split-K weight gradients with atomics) is used as it stands: this
# process gets an empty user db, whatever the parent (pytest's conftest copy) exported
import tempfile  # noqa: E402
os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='vfd_det_db_')

import torch  # noqa: E402

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False


def main():
    import common as G
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    dev = torch.device('cuda:0')
    cfg = G.step_cfg()
    N, frames = cfg['data']['num_cams'], cfg['training']['frame_ids']
    H, W = cfg['training']['height'], cfg['training']['width']
    batch = synth.make_batch(cfg, seed=99, device=dev)
    noise = 1e-5 * torch.randn(N, 1, len(frames) - 1, H, W, generator=torch.Generator().manual_seed(98)).to(dev)
    runs = []
    for i in range(3):
        algo = VFDepthAlgo(cfg, 0)
        algo.branch_streams = i < 2          # the third run: the pose branch on the main stream
        for m in algo.models.values():
            m.load_state_dict(seeded_state_dict(m, seed=G.STEP_SEED))
        algo.set_train()
        algo.optimizer.zero_grad(set_to_none=True)
        outputs, losses = algo.process_batch(dict(batch), 0, noise=noise)
        disp = outputs['_disp_all'][0]
        disp.retain_grad()
        losses['total_loss'].backward()
        torch.cuda.synchronize()
        runs.append(({k: v.detach().clone() for k, v in losses.items()}, outputs['_depth_all'][0].detach().clone(),
                     disp.grad.detach().clone(),
                     {f'{n}.{k}': p.grad.detach().clone() for n, m in algo.models.items()
                      for k, p in m.named_parameters() if p.grad is not None}))
    (l0, d0, gd0, g0), (l1, d1, gd1, g1), (l2, d2, gd2, g2) = runs
    out = {'single_stream_equal': bool(torch.equal(d0, d2) and all(torch.equal(l0[k], l2[k]) for k in l0)
                                       and torch.equal(gd0, gd2) and all(torch.equal(g0[k], g2[k]) for k in g0)),'env': os.environ.get('MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC'),
           'depth_equal': bool(torch.equal(d0, d1)),
           'loss_diff': [k for k in l0 if not torch.equal(l0[k], l1[k])],
           'd_disp_equal': bool(torch.equal(gd0, gd1)),
           'n_grads': len(g0),
           'grad_diff': {k: float((g0[k] - g1[k]).norm() / g1[k].norm().clamp_min(1e-30))
                         for k in g0 if not torch.equal(g0[k], g1[k])}}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
