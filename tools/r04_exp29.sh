#!/bin/bash
# K1 on fp32 tables at d = 256 (MB) with GCN_PF_F32 work items per wave vs the default kernel (tools/gcn_micro.py:
# per-launch time + checksum), then the round's evidence part a at HEAD
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp29.log
: > $O
for r in 1 2; do for v in default pff2 pff4; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != default ] && L=variants/lib_$v.so
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/gcn_micro.py 2>&1 | grep -v amdgpu.ids >> $O || { tail -20 $O; exit 1; }; done; done
cat $O
bash tools/r04_final_a.sh ${1:-r04h}
