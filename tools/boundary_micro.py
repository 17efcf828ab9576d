"""What a kernel boundary costs behind a kernel that writes B bytes (default-policy vs non-temporal stores): time per
(streaming write kernel + one-workgroup kernel) pair minus the write kernel alone, for B from 4 to 256 MB
(tools/boundary_micro.hip; the guide's boundary row: ≈1.5–1.9 µs + dirty bytes ÷ 6 TB/s).
usage: python tools/boundary_micro.py   (builds tools/_boundary_micro.so with hipcc if missing)"""
import ctypes
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, '_boundary_micro.so')


def main():
    if not os.path.exists(SO):
        subprocess.run(['hipcc', '-O3', '--offload-arch=gfx950', '-shared', '-fPIC',
                        os.path.join(HERE, 'boundary_micro.hip'), '-o', SO], check=True)
    lib = ctypes.CDLL(SO)
    lib.boundary_run.restype = ctypes.c_float
    lib.boundary_run.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_void_p]
    scratch = torch.zeros(16, device='cuda')
    for mb in (4, 16, 32, 64, 128, 256):
        n = mb * (1 << 20) // 4
        x = torch.randn(n, device='cuda')
        y = torch.empty(n, device='cuda')
        torch.cuda.synchronize()
        r = {}
        for nt in (0, 1):
            for tiny in (0, 1):
                r[nt, tiny] = min(lib.boundary_run(x.data_ptr(), y.data_ptr(), n, nt, 50, tiny, scratch.data_ptr())
                                  for _ in range(3))
        print(f'{mb:4d} MB written: default stores {r[0, 0]:7.1f} us/launch, + tiny kernel {r[0, 1] - r[0, 0]:5.1f} us; '
              f'nt stores {r[1, 0]:7.1f} us/launch, + tiny kernel {r[1, 1] - r[1, 0]:5.1f} us', flush=True)


if __name__ == '__main__':
    main()
