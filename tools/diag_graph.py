"""Repeat the graph-replay vs eager comparison of tests/test_gpu_parity.py a few times in one
process and print every loss term and the auto-mask flip count (flake diagnosis)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
import torch  # noqa: E402

import common as G  # noqa: E402
from vfdepth_amd import synth  # noqa: E402
from vfdepth_amd.layers import seeded_state_dict  # noqa: E402
from vfdepth_amd.vfdepth import VFDepthAlgo  # noqa: E402

DEV = torch.device('cuda:0')


def once(rep):
    cfg = G.step_cfg()
    batch = synth.make_batch(cfg, seed=99, device=DEV)
    for f in cfg['training']['frame_ids'][1:]:
        for s in cfg['training']['scales']:
            for key in ('color', 'color_aug'):
                if (key, f, s) in batch:
                    batch[(key, f, s)] = batch[(key, 0, s)].clone()
    algos, init = [], {}
    for _ in range(2):
        a = VFDepthAlgo(cfg, 0)
        for name, m in a.models.items():
            init[name] = seeded_state_dict(m, seed=G.STEP_SEED)
            m.load_state_dict(init[name])
        a.set_train()
        a.set_optimizer(capturable=True)
        a.losses.device_seed = True
        algos.append(a)
    graphed = algos[0].graphed_train_step(batch, warmup=2)
    for name, m in algos[0].models.items():
        m.load_state_dict(init[name])
    for st in algos[0].optimizer.state.values():
        for t in st.values():
            if torch.is_tensor(t):
                t.zero_()
    algos[0].losses._counter.zero_()
    lg = {k: float(v) for k, v in graphed().items() if torch.is_tensor(v) and v.numel() == 1}
    algos[1].optimizer.zero_grad(set_to_none=True)
    out_e, le = algos[1].process_batch(dict(batch), 0)
    le = {k: float(v) for k, v in le.items() if torch.is_tensor(v) and v.numel() == 1}
    torch.cuda.synchronize()
    flips = [int((graphed.outputs[('cam', c)][('reproj_mask', 0)] != out_e[('cam', c)][('reproj_mask', 0)]).sum())
             for c in range(cfg['data']['num_cams'])]
    dd = [float((graphed.outputs[('cam', c)][('depth', 0)] - out_e[('cam', c)][('depth', 0)]).abs().max())
          for c in range(cfg['data']['num_cams'])]
    print(f'rep {rep}: flips {flips} max|d depth| {max(dd):.3g}', flush=True)
    for k in sorted(lg):
        if k in le:
            print(f'   {k:22s} graph {lg[k]: .8g}  eager {le[k]: .8g}  diff {lg[k] - le[k]: .3g}', flush=True)


for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    once(r)
