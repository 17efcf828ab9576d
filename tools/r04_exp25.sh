#!/bin/bash
# K5 (builtin second product): DMA spacing DQ=1, S-read distance DS=3 / 1 against the default, A/B ×3
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp25.log
: > $O
for r in 1 2 3; do for v in base dq1 ds3 ds1; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/ce3_micro.py 2>&1 | grep -v amdgpu.ids >> $O || { cat $O; exit 1; }; done; done
grep -E "^==|ce3 Mv" $O | sed 's/split.*us; //; s/ (.*executed, ns 12)//; s/checksum.*//' | paste - -
