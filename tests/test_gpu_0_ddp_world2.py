"""World size 2 on the MI355X: the SyncBatchNorm branch of the fused BatchNorm kernels and the
fusion step under DDP + SyncBatchNorm (reference models/vfdepth.py:56-71, utils/ddp.py:10-29).

Two ranks share cuda:0 over a gloo group (tests/ddp_world2_worker.py has the checks).  The file is
named so that it runs first in a `-m gpu` session: the ranks are started as child processes
before this pytest process has touched the GPU."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.timeout(600)
def test_syncbn_and_ddp_world2_on_one_gpu():
    import torch
    if torch.cuda.device_count() < 1:          # counting devices does not initialise the GPU
        pytest.skip('no HIP device')
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE='2', LOCAL_RANK=str(rank), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY='0', OMP_NUM_THREADS='4')
        procs.append(subprocess.Popen([sys.executable, '-u', os.path.join(ROOT, 'tests', 'ddp_world2_worker.py')],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=540)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for rank, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f'rank {rank} exited {p.returncode}:\n{out[-4000:]}'
        assert f'OK rank {rank}' in out, out[-2000:]
        print(out.strip().splitlines()[-1])
