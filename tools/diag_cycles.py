"""Reference cycles that keep a training step's autograd graph alive after the step returns (they
survive until Python's cyclic collector happens to run — and an AccumulateGrad node kept alive that
way carries its stream into the next step, or into a HIP-graph capture).

    python tools/diag_cycles.py [--config -1] [--pairs 1]
"""
import argparse
import collections
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=-1)
    ap.add_argument('--pairs', type=int, default=1)
    a = ap.parse_args()
    os.environ['VFD_POSE_PAIRS'] = str(a.pairs)
    import bench
    from vfdepth_amd import _lib, synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    _lib.load()
    if a.config < 0:
        import common as G
        cfg = G.step_cfg()
    else:
        cfg, _ = bench.make_cfg(a.config)
    algo = VFDepthAlgo(cfg, 0)
    for m in algo.models.values():
        m.load_state_dict(seeded_state_dict(m, seed=7))
    algo.set_train()
    batch = synth.make_batch(cfg, seed=3, device='cuda:0')
    gc.disable()
    algo.train_step(dict(batch))
    torch.cuda.synchronize()
    gc.collect()
    algo.train_step(dict(batch))
    torch.cuda.synchronize()
    gc.set_debug(gc.DEBUG_SAVEALL)
    n = gc.collect()
    kinds = collections.Counter(type(o).__name__ for o in gc.garbage)
    print(f'unreachable objects after one step: {n}')
    for k, v in kinds.most_common(40):
        print(f'  {v:6d}  {k}')
    graphs = [o for o in gc.garbage if torch.is_tensor(o) and o.grad_fn is not None]
    print(f'tensors with grad_fn among them: {len(graphs)}')
    nodes = [o for o in gc.garbage if 'Backward' in type(o).__name__]
    print('autograd nodes:', collections.Counter(type(o).__name__ for o in nodes).most_common(20))
    # the cycles' entry points: dicts / frames / cells among the garbage that reference a node
    for o in gc.garbage:
        if isinstance(o, dict) and any('Backward' in type(v).__name__ for v in o.values()):
            print('dict with a node:', {k: type(v).__name__ for k, v in list(o.items())[:12]})
            break
    for o in gc.garbage:
        if type(o).__name__ in ('frame', 'cell', 'function', 'method'):
            print('  ', type(o).__name__, getattr(o, '__qualname__', None) or getattr(getattr(o, 'f_code', None), 'co_name', ''),
                  getattr(getattr(o, 'f_code', None), 'co_filename', ''))


if __name__ == '__main__':
    main()
