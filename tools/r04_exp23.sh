#!/bin/bash
# K5 S phase with the row-fragment reads inside the asm triples (variants/lib_sasm.so, CE3_SASM) vs the default:
# the ce3 tests on the variant first, then an interleaved A/B at MB head-b shapes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp23.log
: > $O
C2DSR_LIB=variants/lib_sasm.so timeout -k 10 200 python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 200 --timeout-method thread >> $O 2>&1 || { cat $O; exit 1; }
for r in 1 2 3; do for v in base sasm; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/ce3_micro.py 2>&1 | grep -v amdgpu.ids >> $O || { cat $O; exit 1; }; done; done
grep -E "passed|failed|^==|ce3 Mv" $O | sed 's/split.*us; //; s/ (.*executed, ns 12)//; s/checksum.*//'
