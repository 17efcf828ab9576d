"""Micro-benchmark of K1 (c2dsr_gcn_spmm: pieces + split-row combine) on the bench's Movie-Book graph
(d=256, dropout 0.2), forward (mask on the gathered rows) and backward (Aᵀ, mask on the output rows)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from c2dsr_amd import ops  # noqa: E402
from c2dsr_amd.graph import DeviceGraph  # noqa: E402


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


def main():
    cfg = dict(bench.CONFIGS['mb'])
    _, gs, _ = bench.make_workload(cfg, 20 * cfg['B'])
    dev = torch.device('cuda')
    g = DeviceGraph(gs, dev)
    d = cfg['d']
    X = torch.randn(g.n, d, device=dev)
    Y = torch.empty_like(X)
    keys = (1, 2)
    f = lambda: ops.spmm(g, False, X, keys, 0.2, False, 1.0, None, 0.0, 0.0, -1, 0.0, Y)  # noqa: E731
    b = lambda: ops.spmm(g, True, X, keys, 0.2, True, 1.0, None, 0.0, 0.0, -1, 0.0, Y)  # noqa: E731
    tf, tb = timeit(f), timeit(b)
    f()
    torch.cuda.synchronize()
    print(f'{os.path.basename(os.environ.get("C2DSR_LIB", "default"))}: spmm fwd {tf:.1f} us, bwd {tb:.1f} us '
          f'(splits {g.n_split}/{g.n_split_t}); checksum {float(Y.double().sum()):.6e}', flush=True)


if __name__ == '__main__':
    main()
