#!/bin/bash
# fragment-ordered split weight images (c2dsr_rgemm_x3f): the rgemm tests, the torch-op test, timing row vs frag
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp11.log
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ce3.py tests/test_gpu_torch_ops.py -q -x -k "rgemm or split or torch_ops" --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
timeout -k 10 150 python -u tools/rg_micro.py x3 2>&1 | grep -v amdgpu.ids >> $O || { cat $O; exit 1; }
cat $O
