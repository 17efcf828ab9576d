"""Micro-benchmark of K6 (c2dsr_adamw) at the MB parameter count (105.8 M): direct-accumulation (KEEP,
36 B/param) and fold (48 B/param) modes, HIP-event timed; C2DSR_LIB selects a variant library."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from c2dsr_amd._lib import lib, stream  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


n = 105_800_000
b = [torch.zeros(n, device='cuda') for _ in range(6)]
p, fresh, acc, m, v, vx = b
s = stream()
keep = timeit(lambda: lib('c2dsr_adamw', p, acc, acc, m, v, vx, n, 1e-3, 5e-4, 0.9, 0.999, 1e-8, 1, None, s))
fold = timeit(lambda: lib('c2dsr_adamw', p, fresh, acc, m, v, vx, n, 1e-3, 5e-4, 0.9, 0.999, 1e-8, 1, None, s))
print(f'{os.path.basename(os.environ.get("C2DSR_LIB", "default"))}: keep {keep:.1f} us ({36 * n / keep / 1e3:.0f} GB/s), '
      f'fold {fold:.1f} us ({48 * n / fold / 1e3:.0f} GB/s)', flush=True)
