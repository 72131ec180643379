"""Worker of test_graph_replay_bit_identical (tests/test_gpu_parity.py): a fresh process under the
deterministic flag (MIOpen reads MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC before its first
convolution; empty user db, as tests/det_worker.py), so two eager steps from one state are
bit-identical — and so must be a HIP-graph replay of the DEFAULT step (batched pose pairs, pose
branch on its own stream) against the eager step, and replays against each other.  Any difference
is a missing dependency in the captured graph (a race) or a capture that computes something else.
Prints one JSON line.

    python tests/graph_det_worker.py [--ddp]
"""
import json
import os
import socket
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, 'golden')]

import tempfile  # noqa: E402
os.environ['MIOPEN_USER_DB_PATH'] = tempfile.mkdtemp(prefix='vfd_det_db_')
os.environ['MIOPEN_DEBUG_CONVOLUTION_DETERMINISTIC'] = '1'
os.environ.setdefault('TORCH_NCCL_ASYNC_ERROR_HANDLING', '0')
# the process group's pooled events must not be re-recorded inside the capture while its
# watchdog still polls them (hipErrorCapturedEvent in the watchdog thread, round 6)
os.environ.setdefault('TORCH_NCCL_CUDA_EVENT_CACHE', '0')

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

torch.backends.cudnn.deterministic = True
torch.backends.cudnn.benchmark = False


def main():
    import common as G
    from vfdepth_amd import synth
    from vfdepth_amd.layers import seeded_state_dict
    from vfdepth_amd.vfdepth import VFDepthAlgo
    ddp = '--ddp' in sys.argv
    if ddp:
        with socket.socket() as s:
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    dev = torch.device('cuda:0')
    cfg = G.step_cfg()
    cfg['ddp'].update({'ddp_enable': ddp, 'world_size': 1, 'gpus': [0], 'graph_capture': ddp})
    batch = synth.make_batch(cfg, seed=99, device=dev)
    algo = VFDepthAlgo(cfg, 0)
    inner = {k: getattr(m, 'module', m) for k, m in algo.models.items()}
    init = {k: seeded_state_dict(m, seed=G.STEP_SEED) for k, m in inner.items()}
    for k, m in inner.items():
        m.load_state_dict(init[k])
    algo.set_train()
    algo.set_optimizer(capturable=True)
    algo.losses.device_seed = True
    algo.train_step(dict(batch))                 # an eager branch-stream step before the capture
    graphed = algo.graphed_train_step(batch, warmup=2)
    grads = [p.grad for m in inner.values() for p in m.parameters()]   # the tensors the replay writes

    def rewind():
        for k, m in inner.items():
            m.load_state_dict(init[k])
        for st in algo.optimizer.state.values():
            for t in st.values():
                if torch.is_tensor(t):
                    t.zero_()
        algo.losses._counter.zero_()

    def snap(losses, outputs, gl):
        torch.cuda.synchronize()
        return ({k: v.detach().clone() for k, v in losses.items() if torch.is_tensor(v)},
                [outputs[('cam', c)][('depth', 0)].detach().clone() for c in range(cfg['data']['num_cams'])],
                [g.detach().clone() if g is not None else None for g in gl])

    replays = []
    for _ in range(3):
        rewind()
        replays.append(snap(graphed(), graphed.outputs, grads))
    # back to back: two replays with no host synchronisation between them (the bench's loop),
    # against the same two replays with a device sync between: the graph launch must order the
    # second replay after ALL of the first one's work (its pose-branch nodes included)
    twice = []
    for sync in (True, False):
        rewind()
        graphed()
        if sync:
            torch.cuda.synchronize()
        twice.append(snap(graphed(), graphed.outputs, grads))
    eager = []
    for _ in range(2):
        rewind()
        algo.optimizer.zero_grad(set_to_none=True)
        out, losses = algo.process_batch(dict(batch), 0)
        losses['total_loss'].backward()
        eager.append(snap(losses, out, [p.grad for m in inner.values() for p in m.parameters()]))

    def same(a, b):
        la, da, ga = a
        lb, db, gb = b
        bad = [k for k in lb if not torch.equal(la[k], lb[k])]
        bad += [f'depth{c}' for c in range(len(db)) if not torch.equal(da[c], db[c])]
        names = [f'{k}.{n}' for k, m in inner.items() for n, _ in m.named_parameters()]
        bad += [names[i] for i in range(len(gb)) if (ga[i] is None) != (gb[i] is None)
                or (gb[i] is not None and not torch.equal(ga[i], gb[i]))]
        return bad
    res = {'eager_vs_eager': same(eager[1], eager[0])[:12],
           'replay_vs_replay': sorted(set(same(replays[1], replays[0]) + same(replays[2], replays[0])))[:12],
           'replay_vs_eager': same(replays[0], eager[0])[:12],
           'back_to_back_vs_synced': same(twice[1], twice[0])[:12],
           'branch_stream': getattr(algo, '_bstream', None) is not None, 'pairs_batched': algo.pose.batch_pairs,
           'ddp': ddp, 'total_loss': float(replays[0][0]['total_loss'])}
    print(json.dumps(res), flush=True)
    if ddp:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
