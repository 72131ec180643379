"""Build the gfx950 hot-path library `vfdepth_amd/libvfd_hip.so` with hipcc (in-tree).

    python -m vfdepth_amd.build            # incremental
    python -m vfdepth_amd.build --force

No CMake: one hipcc invocation per translation unit, then a shared link.  `-ffp-contract=off`
keeps every multiply and add separately rounded, the same operation sequence as the reference's
CPU ATen path, so boundary decisions (OOB / mask / argmin) agree with it.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, 'csrc')
INCLUDE = os.path.join(ROOT, 'include')
LIB = os.path.join(HERE, 'libvfd_hip.so')
SOURCES = ['capi.hip', 'fusion.hip', 'view.hip', 'photo.hip', 'aggregate.hip', 'projconv.hip', 'depthsyn.hip', 'padconv.hip', 'bnact.hip', 'reflectpad.hip', 'geometry.hip', 'maxpool.hip', 'weights.hip', 'dispconv.hip', 'decconv.hip']
ARCH = os.environ.get('VFD_OFFLOAD_ARCH', 'gfx950')
FLAGS = ['-O3', f'--offload-arch={ARCH}', '-std=c++17', '-fPIC', '-ffp-contract=off',
         '-Wno-unused-result', '-I', INCLUDE, '-I', CSRC]


def _hipcc():
    for cand in (os.environ.get('HIPCC'), '/opt/rocm/bin/hipcc', 'hipcc'):
        if cand and (os.path.sep not in cand or os.path.exists(cand)):
            return cand
    raise RuntimeError('hipcc not found')


def _digest(paths, extra=()):
    """sha256 over the CONTENT of `paths` (and the compile command): what a target was built from.
    Content, not mtimes — a checkout, a copy or a snapshot to the GPU box resets mtimes."""
    h = hashlib.sha256()
    for x in extra:
        h.update(str(x).encode())
    for p in paths:
        with open(p, 'rb') as fh:
            h.update(fh.read())
    return h.hexdigest()


def _stale(out, digest):
    """out is missing, or was built from different content (its .sha record differs)."""
    rec = out + '.sha'
    if not (os.path.exists(out) and os.path.exists(rec)):
        return True
    with open(rec) as fh:
        return fh.read().strip() != digest


def _record(out, digest):
    with open(out + '.sha', 'w') as fh:
        fh.write(digest + '\n')


def build(force=False, verbose=True):
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, 'vfd_common.h'), os.path.join(INCLUDE, 'vfd_capi.h')]
    objs, jobs = [], []
    os.makedirs(os.path.join(HERE, 'build'), exist_ok=True)
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(HERE, 'build', src.replace('.hip', '.o'))
        objs.append(o)
        dg = _digest([s] + headers, extra=FLAGS)
        if force or _stale(o, dg):
            jobs.append(([hipcc] + FLAGS + ['-c', s, '-o', o], o, dg))
    # translation units compile in parallel (at most 8 hipcc processes)
    from concurrent.futures import ThreadPoolExecutor

    def run(job):
        cmd, out, dg = job
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
        _record(out, dg)
    with ThreadPoolExecutor(max_workers=max(1, min(8, os.cpu_count() or 1))) as ex:
        list(ex.map(run, jobs))
    dg = _digest(objs, extra=[ARCH])
    if force or _stale(LIB, dg):
        cmd = [hipcc, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB] + objs
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
        _record(LIB, dg)
    return LIB


if __name__ == '__main__':
    build(force='--force' in sys.argv)
