"""Two VFDepthAlgo twins from one seeded state: does an earlier eager step of one of them (then a
rewind to the initial state) change the gradients its next step computes?  Per-net relative
gradient differences, twin vs twin and twin vs itself.

    python tools/diag_twins.py [--branch 0|1] [--pre 0|1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests', 'golden')]
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--branch', type=int, default=1)
    ap.add_argument('--pre', type=int, default=1, help='an eager train_step of twin 0 before the comparison')
    a = ap.parse_args()
    import common as G
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    cfg = G.step_cfg()
    batch = synth.make_batch(cfg, seed=99, device='cuda:0')
    algos, init = [], {}
    for _ in range(2):
        al = VFDepthAlgo(cfg, 0)
        for n, m in al.models.items():
            init[n] = seeded_state_dict(m, seed=G.STEP_SEED)
            m.load_state_dict(init[n])
        al.set_train()
        al.set_optimizer(capturable=True)
        al.losses.device_seed = True
        al.branch_streams = bool(a.branch)
        algos.append(al)
    if a.pre:
        algos[0].train_step(dict(batch))

    def step(al):
        for n, m in al.models.items():
            m.load_state_dict(init[n])
        if getattr(al.losses, '_counter', None) is not None:
            al.losses._counter.zero_()
        al.optimizer.zero_grad(set_to_none=True)
        _, l = al.process_batch(dict(batch), 0)
        l['total_loss'].backward()
        torch.cuda.synchronize()
        return float(l['total_loss']), {n: {k: p.grad.detach().clone() for k, p in m.named_parameters()}
                                        for n, m in al.models.items()}

    def rel(ga, gb):
        num = sum(float((ga[k].double() - gb[k].double()).pow(2).sum()) for k in gb)
        den = sum(float(gb[k].double().pow(2).sum()) for k in gb)
        return (num / max(den, 1e-300)) ** 0.5
    r0a, r0b, r1a, r1b = step(algos[0]), step(algos[0]), step(algos[1]), step(algos[1])
    print(f'branch {a.branch} pre {a.pre}: losses {r0a[0]:.7f} {r0b[0]:.7f} {r1a[0]:.7f} {r1b[0]:.7f}')
    for net in r0a[1]:
        print(f'  {net}: twin0 vs twin0 {rel(r0b[1][net], r0a[1][net]):.3g}, twin1 vs twin1 '
              f'{rel(r1b[1][net], r1a[1][net]):.3g}, twin0 vs twin1 {rel(r0a[1][net], r1a[1][net]):.3g}')
        worst = sorted(((float((r0a[1][net][k] - r1a[1][net][k]).norm() / max(float(r1a[1][net][k].norm()), 1e-30)), k)
                        for k in r1a[1][net]), reverse=True)[:4]
        print('     worst:', ', '.join(f'{k} {v:.3g}' for v, k in worst))


if __name__ == '__main__':
    main()
