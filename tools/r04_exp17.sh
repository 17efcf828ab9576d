#!/bin/bash
# K5 with the builtin second product (default now): step-pattern VALU share (VN), transposed-read distance (DT),
# DMA spacing (DQ) variants against the default, at MB head-b shapes
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp17.log
: > $O
for r in 1 2; do for v in base vn3 vn8 dt3 dq4; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/ce3_micro.py 2>&1 | grep -v amdgpu.ids >> $O || { cat $O; exit 1; }; done; done
cat $O
