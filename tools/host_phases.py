"""Host wall time per phase of a training step (bench workload, fp32 / bf16): where the host waits for the device.
Wraps Trainer.prepare, the model forward, LossHeadFn.apply, Trainer._backward and optimizer.step with perf_counter.
usage: python tools/host_phases.py [precision] [config]"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    precision = sys.argv[1] if len(sys.argv) > 1 else 'fp32'
    name = sys.argv[2] if len(sys.argv) > 2 else 'mb'
    cfg = dict(bench.CONFIGS[name])
    rows, gs, gp = bench.workload(cfg, name)
    from c2dsr_amd import trainer as T
    from c2dsr_amd.losshead import LossHeadFn
    args = bench.make_args(cfg, torch.device('cuda'), precision)
    torch.manual_seed(3407)
    tr = T.Trainer(args, None, data=(None, None, None), graphs=(gs, gp))
    B = cfg['B']
    host = [tuple(r[i * B:(i + 1) * B] for r in rows) for i in range(12)]
    batches = [tuple(torch.from_numpy(x.copy()).cuda() for x in h) for h in host]
    counts = [tr.launch_counts(h, global_rows=B) for h in host]
    acc = collections.defaultdict(list)

    def wrap(obj, attr, label):
        f = getattr(obj, attr)

        def g(*a, **k):
            t0 = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                acc[label].append((time.perf_counter() - t0) * 1e3)
        setattr(obj, attr, g)

    wrap(tr, 'prepare', 'prepare')
    wrap(tr.model, 'launch_graph', 'launch_graph')
    wrap(tr.model, 'convolve_graph', 'convolve_graph')
    wrap(tr, '_backward', 'backward')
    wrap(tr.optimizer, 'step', 'optimizer.step')
    wrap(LossHeadFn, 'apply', 'losshead.forward')
    mfwd = tr.model.forward
    wrap(tr.model, 'forward', 'model.forward')
    tr.model.train()
    tr.optimizer.zero_grad()
    for i in range(12):
        t0 = time.perf_counter()
        tr.model.convolve_graph()
        tr.train_batch(batches[i], global_rows=B, counts=counts[i])
        acc['step (enqueue)'].append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    for k, v in acc.items():
        v = v[-8:] if len(v) >= 8 else v
        print(f'{k:20s} ms per call (last {len(v)}): ' + ' '.join(f'{x:6.2f}' for x in v))
    del mfwd


if __name__ == '__main__':
    main()
