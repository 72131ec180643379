"""FETCH_SIZE calibration on a known-byte probe: reads a 512 MiB buffer once with 4-, 8- and 16-B
lanes (tools/probe/fetch_probe.hip, prebuilt by `python tools/probe_fetch.py --build`).  Run under
`rocprofv3 --pmc FETCH_SIZE` and compare each kernel's FETCH_SIZE with 512 MiB.

    rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python tools/probe_fetch.py
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, 'probe', 'libfetchprobe.so')


def build():
    subprocess.check_call(['/opt/rocm/bin/hipcc', '-O3', '--offload-arch=gfx950', '-shared', '-fPIC',
                           os.path.join(HERE, 'probe', 'fetch_probe.hip'), '-o', SO])


def main():
    if '--build' in sys.argv:
        build()
        return
    import torch
    lib = ctypes.CDLL(SO)
    n = (512 << 20) // 4
    src = torch.rand(n, device='cuda')
    out = torch.empty(4096, device='cuda')
    st = torch.cuda.current_stream().cuda_stream
    for width in (4, 8, 16):
        for _ in range(2):               # the second dispatch of each width is the measured one
            assert lib.probe_read(ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(n), width,
                                  ctypes.c_void_p(out.data_ptr()), 4096, ctypes.c_void_p(st)) == 0
        torch.cuda.synchronize()
    print('probe bytes per dispatch', n * 4, flush=True)


if __name__ == '__main__':
    main()
