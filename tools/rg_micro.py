"""Micro-benchmark of the K3 row-streaming projection GEMM (c2dsr_rgemm) at the encoder's shapes: time vs M
for K = 256 (N = 256, 512) and the achieved HBM rate of its A read + C write (HIP events).
usage: python tools/rg_micro.py [epi | wg | x3]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd.ops import rgemm, to_bf16, to_split_bf16, weight_img  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def epilogue_costs():
    """The drop(relu) epilogue (linear1) with and without a row map, against the plain product."""
    dev = torch.device('cuda')
    K = N = 256
    M = 57000
    Wb = to_bf16(torch.randn(N, K, device=dev))
    A = torch.randn(M, K, device=dev)
    C = torch.empty(M, N, device=dev)
    rowmap = torch.sort(torch.randperm(102400, device=dev)[:M])[0].to(torch.int32)
    lib_ = os.path.basename(os.environ.get("C2DSR_LIB", "default"))
    for name, kw in (('plain', {}), ('relu_drop', dict(relu_drop=((1, 2), 0.2, 0))),
                     ('relu_drop+map', dict(relu_drop=((1, 2), 0.2, 0, rowmap))),
                     ('relu p=0', dict(relu_drop=((1, 2), 0.0, 0)))):
        t = timeit(lambda: rgemm(A, Wb, C, M=M, N=N, K=K, **kw))
        print(f'{lib_}: epilogue {name:14s} M {M}: {t:6.1f} us', flush=True)


def wg_costs():
    """The weight-gradient product (c2dsr_wgemm: split partials + fixed-order sum) at the encoder's shapes."""
    from c2dsr_amd.ops import wgemm
    dev = torch.device('cuda')
    lib_ = os.path.basename(os.environ.get("C2DSR_LIB", "default"))
    for T, N, kind in ((38000, 256, 'fp32'), (57000, 256, 'fp32'), (38000, 256, 'bf16'), (57000, 512, 'bf16'),
                       (38000, 256, 'x3'), (57000, 256, 'x3'), (57000, 512, 'x3')):
        dY = torch.randn(T, N, device=dev)
        if kind == 'bf16':
            dY = dY.to(torch.bfloat16)
        X = torch.randn(T, 256, device=dev)
        dW = torch.zeros(N, 256, device=dev)
        db = torch.zeros(N, device=dev)
        t = timeit(lambda: wgemm(dY, X, dW, T=T, N=N, D=256, db=db, x3=kind == 'x3'))
        gb = (T * N * (2 if kind == 'bf16' else 4) + T * 256 * 4) / t / 1e3
        print(f'{lib_}: wgemm T {T} N {N} {kind} dY: {t:6.1f} us {gb:6.0f} GB/s', flush=True)


def main(x3=False):
    dev = torch.device('cuda')
    K = 256
    for N in (256, 512):
        W = torch.randn(N, K, device=dev)
        # x3: the row image (c2dsr_rgemm_x3) and the fragment-ordered image the fp32 step uses (c2dsr_rgemm_x3f)
        forms = ((('x3', False, to_split_bf16(W)), ('x3f', True, to_split_bf16(W, frag=True))) if x3 else
                 (('b16', False, to_bf16(W)), ('b16f', True, weight_img(W, 'b16'))))
        for M in (8192, 20000, 38000, 57000, 102400):
            A = torch.randn(M, K, device=dev)
            C = torch.empty(M, N, device=dev)
            for name, fr, Wb in forms:
                t = timeit(lambda: rgemm(A, Wb, C, M=M, N=N, K=K, x3=x3, frag=fr))
                gb = 4.0 * M * (K + N) / t / 1e3
                print(f'{os.path.basename(os.environ.get("C2DSR_LIB", "default"))}: {name} N {N} M {M:6d}: '
                      f'{t:6.1f} us {gb:6.0f} GB/s', flush=True)
                if x3:
                    rg3_stamps(lambda: rgemm(A, Wb, C, M=M, N=N, K=K, x3=x3, frag=fr))


def rg3_stamps(f):
    """Diagnostic build (-DRG3_STAMP): cycles per chunk per wave of the rg3 loop's phases."""
    import ctypes
    from c2dsr_amd import _lib
    so = ctypes.CDLL(os.path.join(_lib._DIR, 'libc2dsr_hip.so'))  # the stamp entry exists in the diagnostic build only
    if not hasattr(so, 'c2dsr_rg3_stamps'):
        return
    fn = so.c2dsr_rg3_stamps
    buf = (ctypes.c_ulonglong * 8)()
    torch.cuda.synchronize()
    fn(buf, 1)
    f()
    torch.cuda.synchronize()
    fn(buf, 1)
    ch, waves = max(1, buf[6]), max(1, buf[7])
    print(f'  stamps: prologue {buf[0] / waves:.0f} per wave; per chunk: mfma+stage {buf[1] / ch:.0f}, '
          f'epilogue {buf[2] / ch:.0f}, barrier {buf[3] / ch:.0f} cycles ({ch // waves} chunks per wave)', flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'epi':
        epilogue_costs()
    elif len(sys.argv) > 1 and sys.argv[1] == 'wg':
        wg_costs()
    elif len(sys.argv) > 1 and sys.argv[1] == 'x3':
        main(x3=True)
    else:
        main()
