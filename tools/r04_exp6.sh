#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp6.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
run ./tools/peak/s_phase 20000 || { cat $O; exit 1; }
run python -u -m pytest tests/test_gpu_kernels.py -q -x -k embed --timeout 200 --timeout-method thread || { cat $O; exit 1; }
run python -u tools/embed_micro.py || { cat $O; exit 1; }
cat $O
