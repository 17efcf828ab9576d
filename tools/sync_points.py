"""Where a training step synchronises the host with the device: one bench-workload step (MB, fp32 mode, counts
from the data pipeline as bench.py hands them in) under torch.cuda.set_sync_debug_mode('warn'), printing the Python
stack of every synchronising operation torch reports (blocking copies, .item(), …).
usage: python tools/sync_points.py [config] [batch]"""
import collections
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else 'mb'
    cfg = dict(bench.CONFIGS[name])
    if len(sys.argv) > 2:
        cfg['B'] = int(sys.argv[2])
    rows, gs, gp = bench.workload(cfg, name)
    from c2dsr_amd.trainer import Trainer
    args = bench.make_args(cfg, torch.device('cuda'), 'fp32')
    torch.manual_seed(3407)
    tr = Trainer(args, None, data=(None, None, None), graphs=(gs, gp))
    B = cfg['B']
    host = [tuple(r[i * B:(i + 1) * B] for r in rows) for i in range(5)]
    batches = [tuple(torch.from_numpy(x.copy()).cuda() for x in h) for h in host]
    counts = [tr.launch_counts(h, global_rows=B) for h in host]
    tr.model.train()
    tr.optimizer.zero_grad()
    for i in range(3):
        tr.model.convolve_graph()
        tr.train_batch(batches[i], global_rows=B, counts=counts[i])
    torch.cuda.synchronize()
    seen = collections.Counter()
    stacks = {}

    def show(message, category, filename, lineno, file=None, line=None):
        st = ''.join(traceback.format_stack(limit=12)[:-2])
        key = str(message)[:80] + ' @ ' + ' <- '.join(
            f'{os.path.basename(f.filename)}:{f.lineno}' for f in traceback.extract_stack(limit=12)[-6:-2])
        seen[key] += 1
        stacks.setdefault(key, st)

    warnings.showwarning = show
    warnings.simplefilter('always')
    torch.cuda.set_sync_debug_mode('warn')
    tr.model.convolve_graph()
    tr.train_batch(batches[3], global_rows=B, counts=counts[3])
    torch.cuda.set_sync_debug_mode('default')
    torch.cuda.synchronize()
    print(f'{sum(seen.values())} synchronising operations in one step')
    for k, c in seen.most_common():
        print(f'{c:4d}  {k}')
    for k, st in list(stacks.items())[:6]:
        print('-----', k, '\n', st)


if __name__ == '__main__':
    main()
