"""The bench's own multi-rank path at world size 2 on one MI355X: `bench.py --gpus 2` starts its
ranks itself (launch_ranks -> torch.distributed.run as a child process -> init_process_group ->
DDP + SyncBatchNorm -> barrier-bracketed timed steps -> max over ranks), exactly as the driver's
scaling run does, except for the test-only overrides VFD_BENCH_BACKEND=gloo and
VFD_BENCH_ONE_DEVICE=1 (RCCL does not run two ranks on one device).  Reference:
utils/ddp.py:10-29, train.py:59-61, models/vfdepth.py:61-70.

Named so that it runs before the pytest process touches the GPU (the ranks are child processes)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_bench_two_ranks_on_one_gpu():
    import torch
    if torch.cuda.device_count() < 1:          # counting devices does not initialise the GPU
        pytest.skip('no HIP device')
    steps = 3
    env = dict(os.environ, VFD_BENCH_BACKEND='gloo', VFD_BENCH_ONE_DEVICE='1', HSA_ENABLE_IPC_MODE_LEGACY='0',
               OMP_NUM_THREADS='4', PYTHONUNBUFFERED='1')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--config', '0', '--steps', str(steps),
           '--warmup', '1', '--no-cpu-baseline', '--no-parity']
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=840)
    assert p.returncode == 0, f'bench --gpus 2 exited {p.returncode}:\n{p.stderr[-4000:]}'
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, f'expected ONE JSON line (rank 0), got {len(lines)}:\n{p.stdout[-2000:]}'
    out = json.loads(lines[0])
    assert out['n_gpus'] == 2 and out['config']['parallelism'] == 'dp2' and out['steps'] == steps
    # whole-job throughput: both ranks' iterations over the slowest rank's time
    assert out['value'] == pytest.approx(2 * out['config']['batch_per_gpu'] * 1e3 / out['ms_per_step'], rel=1e-9)
    assert out['scaling'] == 'weak'
    sbn = out['syncbn']
    assert sbn is not None and sbn['backend'] == 'gloo' and sbn['allreduce_per_step'] > 0
    print(f"bench world 2 (gloo, one GPU): {out['value']:.2f} it/s, {out['ms_per_step']:.1f} ms/step, "
          f"{sbn['allreduce_per_step']:.0f} SyncBN all-reduces/step ({sbn['host_ms_per_step']:.1f} ms host)")
