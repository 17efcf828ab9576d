#!/bin/bash
# K5: the S phase on builtin MFMAs as well (bis0: fwd_u, bis1: dw) on top of the builtin second product, A/B ×3
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp19.log
: > $O
for r in 1 2 3; do for v in base bis0 bis1; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/ce3_micro.py 2>&1 | grep -v amdgpu.ids >> $O || { cat $O; exit 1; }; done; done
cat $O
