"""Host-side cost of one training step at the bench workload (MB, fp32 mode): per-step enqueue time (the host
returns before the device finishes unless it waits on a count), wall time with the device synchronised, and a
cProfile of the Python functions that issue the launches.
usage: python tools/host_time.py [precision] [config] [batch] [n_top]   (defaults: fp32 mb <config's B> 30)"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    precision = sys.argv[1] if len(sys.argv) > 1 else 'fp32'
    name = sys.argv[2] if len(sys.argv) > 2 else 'mb'
    cfg = dict(bench.CONFIGS[name])
    if len(sys.argv) > 3 and int(sys.argv[3]):
        cfg['B'] = int(sys.argv[3])
    n_top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    rows, gs, gp = bench.workload(cfg, name)
    from c2dsr_amd.trainer import Trainer
    args = bench.make_args(cfg, torch.device('cuda'), precision)
    torch.manual_seed(3407)
    tr = Trainer(args, None, data=(None, None, None), graphs=(gs, gp))
    B = cfg['B']
    batches = [tuple(torch.from_numpy(r[i * B:(i + 1) * B].copy()).cuda() for r in rows) for i in range(12)]
    tr.model.train()
    tr.optimizer.zero_grad()
    counts = {id(b): tr.launch_counts(tuple(r[i * B:(i + 1) * B] for r in rows), global_rows=B)
              for i, b in enumerate(batches)}  # as bench.py: the launch sizes come with the batch

    def step(b):
        tr.model.convolve_graph()
        return tr.train_batch(b, global_rows=B, counts=counts[id(b)])

    for i in range(3):
        step(batches[i])
    torch.cuda.synchronize()
    enq, wall = [], []
    for i in range(3, 9):
        t0 = time.perf_counter()
        step(batches[i])
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e3)
        wall.append((t2 - t0) * 1e3)
    print('enqueue ms/step', [round(x, 2) for x in enq])
    print('wall    ms/step', [round(x, 2) for x in wall])
    pr = cProfile.Profile()
    pr.enable()
    for i in range(9, 12):
        step(batches[i])
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(n_top)


if __name__ == '__main__':
    main()
