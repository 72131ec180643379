"""Build an experiment variant of the library with extra -D flags (kernel tuning sweeps).

    python tools/build_variant.py NAME -DVFD_PBW_U=4 [...]   -> variants/libvfd_NAME.so
Run with VFD_LIB=variants/libvfd_NAME.so (vfdepth_amd/_lib.py honours it)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vfdepth_amd import build as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    B.build(force=False, verbose=False)
    out_dir = os.path.join('/tmp', 'vfd_variants', name)
    os.makedirs(out_dir, exist_ok=True)
    objs = []
    only = os.environ.get('VFD_VARIANT_SRCS')      # e.g. "fusion.hip": the rest from the main build
    for src in B.SOURCES:
        if only and src not in only.split(','):
            objs.append(os.path.join(B.HERE, 'build', src.replace('.hip', '.o')))
            continue
        o = os.path.join(out_dir, src.replace('.hip', '.o'))
        subprocess.check_call([B._hipcc()] + B.FLAGS + defs + ['-c', os.path.join(B.CSRC, src), '-o', o])
        objs.append(o)
    lib = os.path.join(ROOT, 'variants', f'libvfd_{name}.so')
    subprocess.check_call([B._hipcc(), f'--offload-arch={B.ARCH}', '-shared', '-fPIC', '-o', lib] + objs)
    print(lib)


if __name__ == '__main__':
    main()
