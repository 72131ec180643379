"""Build the gfx950 hot-path library `vfdepth_amd/libvfd_hip.so` with hipcc (in-tree).

    python -m vfdepth_amd.build            # incremental
    python -m vfdepth_amd.build --force

No CMake: one hipcc invocation per translation unit, then a shared link.  `-ffp-contract=off`
keeps every multiply and add separately rounded, the same operation sequence as the reference's
CPU ATen path, so boundary decisions (OOB / mask / argmin) agree with it.
"""
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


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True):
    hipcc = _hipcc()
    headers = [os.path.join(CSRC, 'vfd_common.h'), os.path.join(INCLUDE, 'vfd_capi.h')]
    objs, cmds = [], []
    os.makedirs(os.path.join(HERE, 'build'), exist_ok=True)
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(HERE, 'build', src.replace('.hip', '.o'))
        objs.append(o)
        if force or _stale(o, [s] + headers):
            cmds.append([hipcc] + FLAGS + ['-c', s, '-o', o])
    # translation units compile in parallel (at most 8 hipcc processes)
    from concurrent.futures import ThreadPoolExecutor

    def run(cmd):
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    with ThreadPoolExecutor(max_workers=max(1, min(8, os.cpu_count() or 1))) as ex:
        list(ex.map(run, cmds))
    if force or _stale(LIB, objs):
        cmd = [hipcc, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB] + objs
        if verbose:
            print(' '.join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


if __name__ == '__main__':
    build(force='--force' in sys.argv)
