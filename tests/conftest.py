import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'tests', 'golden')):
    if p not in sys.path:
        sys.path.insert(0, p)

# the tests' MIOpen runs work on a private copy of the committed find-db (they would otherwise
# write their immediate-mode records into it, vfdepth_amd/miopen_db.py)
from vfdepth_amd.miopen_db import use_private_copy  # noqa: E402
use_private_copy()


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) device')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


def golden(name):
    import numpy as np
    return np.load(os.path.join(ROOT, 'tests', 'golden', name))


# ---- long GPU sessions: say which test is running every minute (a silent minute looks like a hang
# to the GPU runner), and print a failure's traceback at once (a session cut short still shows it)
_CURRENT = {'name': None, 't0': 0.0}


def pytest_sessionstart(session):
    import threading
    import time
    tr = session.config.pluginmanager.get_plugin('terminalreporter')
    beat_dir = os.path.join(ROOT, 'gpurun_out')

    def beat():
        while True:
            time.sleep(60)
            if not _CURRENT['name']:
                continue
            msg = f'[heartbeat] {_CURRENT["name"]} running for {time.time() - _CURRENT["t0"]:.0f} s'
            if tr is not None:          # the terminal writer bypasses pytest's output capture
                tr.write_line(msg)
            if os.path.isdir(beat_dir):
                with open(os.path.join(beat_dir, 'pytest_heartbeat.txt'), 'a') as f:
                    f.write(msg + '\n')
    threading.Thread(target=beat, daemon=True).start()


def pytest_runtest_logstart(nodeid, location):
    import time
    _CURRENT['name'], _CURRENT['t0'] = nodeid, time.time()


def pytest_runtest_logreport(report):
    if report.failed:
        print(f'\n[failure] {report.nodeid} ({report.when}):\n{report.longreprtext[-6000:]}\n', flush=True)
