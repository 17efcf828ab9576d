#!/bin/bash
# two-rank rehearsal of bench.py's N>1 path on one GPU (gloo: the ranks share the device), as the driver launches it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r06_dp2.log 2>&1 || { tail -30 gpurun_out/r06_dp2.log; exit 1; }
grep "\[bench\] rank\|data parallel\|WARNING" gpurun_out/r06_dp2.log | head
tail -1 gpurun_out/r06_dp2.log | cut -c1-600
