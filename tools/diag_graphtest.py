"""test_graph_replay_matches_eager's sequence (twin models, non-deterministic mode) with switches, to
find what makes the replay's pose-encoder gradients differ from the twin's eager step.

    python tools/diag_graphtest.py [--pre 0|1] [--sync 0|1] [--twin-first 0|1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests', 'golden')]
if os.environ.get('VFD_DIAG_MIOPEN_DET') == '1':      # MIOpen's deterministic solvers only (empty db)
    import tempfile
    os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='vfd_det_db_')
    os.environ['MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC'] = '1'
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--pre', type=int, default=1)
    ap.add_argument('--sync', type=int, default=0)
    ap.add_argument('--self', type=int, default=0, help='eager reference from the graphed model itself')
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
        algos.append(al)
    if a.pre:
        algos[0].train_step(dict(batch))
    graphed = algos[0].graphed_train_step(batch, warmup=2)

    def rewind(al):
        for n, m in al.models.items():
            m.load_state_dict(init[n])
        for st in al.optimizer.state.values():
            for t in st.values():
                if torch.is_tensor(t):
                    t.zero_()
        if getattr(al.losses, '_counter', None) is not None:
            al.losses._counter.zero_()
    rewind(algos[0])
    graphed()
    if a.sync:
        torch.cuda.synchronize()
    gg = {n: {k: p.grad.detach().clone() for k, p in m.named_parameters()} for n, m in algos[0].models.items()}
    ref = algos[0] if a.self else algos[1]
    runs = []
    for _ in range(2):
        rewind(ref)
        ref.optimizer.zero_grad(set_to_none=True)
        _, l = ref.process_batch(dict(batch), 0)
        l['total_loss'].backward()
        torch.cuda.synchronize()
        runs.append({n: {k: p.grad.detach().clone() for k, p in m.named_parameters()} for n, m in ref.models.items()})

    def rel(ga, gb):
        num = sum(float((ga[k].double() - gb[k].double()).pow(2).sum()) for k in gb)
        den = sum(float(gb[k].double().pow(2).sum()) for k in gb)
        return (num / max(den, 1e-300)) ** 0.5
    tag = f"miopen_det {os.environ.get('VFD_DIAG_MIOPEN_DET', '0')} vfd_det {os.environ.get('VFD_DETERMINISTIC', '0')}"
    print(f'pre {a.pre} sync {a.sync} self {a.self} {tag}: ' + ', '.join(
        f'{net} graph-vs-eager {rel(gg[net], runs[0][net]):.3g} (eager spread {rel(runs[1][net], runs[0][net]):.3g})'
        for net in gg), flush=True)


if __name__ == '__main__':
    main()
