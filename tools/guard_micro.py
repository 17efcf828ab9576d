"""linear1 of the fp32 mode at bench shapes: the exact fp32 GEMM (c2dsr_gemm, the default) vs the guarded split
producer (c2dsr_rgemm_x3_relu_guard on the fragment-ordered image) vs the plain split product (no guard), each with
the relu·dropout epilogue.  usage: python tools/guard_micro.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib  # noqa: E402
from c2dsr_amd.ops import FP32, gemm, rgemm, rgemm_relu_guard, to_split_bf16  # noqa: E402


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    lib.load()
    dev = torch.device('cuda')
    N = K = 256
    W = torch.randn(N, K, device=dev) / 16
    b = torch.randn(N, device=dev) / 16
    Wf = to_split_bf16(W, frag=True)
    rd = ((11, 22), 0.2, 0)
    for M in (20000, 38000, 57000):
        A = torch.randn(M, K, device=dev)
        C = torch.empty(M, N, device=dev)
        t_x = timeit(lambda: gemm(A, W, C, M=M, N=N, K=K, transB=1, bias=b, relu_drop=rd, precision=FP32))
        t_g = timeit(lambda: rgemm_relu_guard(A, Wf, W, C, M=M, N=N, K=K, bias=b, relu_drop=rd, frag=True))
        t_s = timeit(lambda: rgemm(A, Wf, C, M=M, N=N, K=K, bias=b, relu_drop=rd, x3=True, frag=True))
        print(f'linear1 M {M}: exact {t_x:6.1f} us, guarded split {t_g:6.1f} us, split (no guard) {t_s:6.1f} us',
              flush=True)


if __name__ == '__main__':
    main()
