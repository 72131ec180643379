"""One eager training step of the reduced (or config-2) fusion step with MIOpen logging on (the
caller sets MIOPEN_LOG_LEVEL / MIOPEN_ENABLE_LOGGING): the log on stderr names the solver every
convolution runs.  Used to compare the solver picks of the pose net's stacked frame pairs (batch
12) with its per-pair calls (batch 6).

    MIOPEN_ENABLE_LOGGING=1 MIOPEN_LOG_LEVEL=5 python tools/diag_miopen_solvers.py [--config 0]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.path.isdir(os.path.join(ROOT, 'miopen_db')):
    sys.path.insert(0, ROOT)
    from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
    use_private_copy()

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', type=int, default=0)
    a = ap.parse_args()
    import bench
    from vfdepth_amd import _lib, synth
    from vfdepth_amd.vfdepth import VFDepthAlgo
    _lib.load()
    cfg, _ = bench.make_cfg(a.config)
    algo = VFDepthAlgo(cfg, 0)
    algo.set_train()
    batch = synth.make_batch(cfg, seed=3, device='cuda:0')
    algo.train_step(dict(batch))
    torch.cuda.synchronize()
    print('step done', flush=True)


if __name__ == '__main__':
    main()
