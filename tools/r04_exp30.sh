#!/bin/bash
# K1 on bf16 tables with split-row combine variants (COMBINE_HI: all slices in flight; COMBINE_U=32): bit-identity and
# per-launch time vs the default kernel (tools/gcn_pf_check.py), then the C5 bf16-table line, interleaved
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp30.log
: > $O
for v in default hi u32; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != default ] && L=variants/lib_$v.so
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/gcn_pf_check.py 2>&1 | grep -v amdgpu.ids >> $O || { tail -20 $O; exit 1; }; done
cat $O
for r in 1 2; do for v in default hi u32; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != default ] && L=variants/lib_$v.so
  C2DSR_LIB=$L timeout -k 10 300 python -u bench.py --config c5 --c5-tables bf16 --steps 3 --warmup 1 > gpurun_out/exp30_c5_$v$r.log 2>&1 || { tail -20 gpurun_out/exp30_c5_$v$r.log; exit 1; }
  echo "$v $r $(tail -1 gpurun_out/exp30_c5_$v$r.log | cut -c1-260)" | tee -a $O; done; done
