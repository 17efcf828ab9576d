#!/bin/bash
# Round-4 micro-benchmarks (each step under its own limit; one log): K5 phase stamps, embedding backward variants,
# x3 projections with rg3 phase stamps, weight gradients, host enqueue time, a bench line + kernel trace + gaps.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp2.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
C2DSR_LIB=variants/lib_stamp.so run python -u tools/ce3_micro.py || exit 1
C2DSR_LIB=variants/lib_stamp.so run python -u tools/ce3_micro.py 18944 36845 || exit 1
for v in base pref2 pref4 pref8 pref4c32; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; C2DSR_LIB=$L run python -u tools/embed_micro.py || exit 1; done
run python -u tools/rg_micro.py x3 || exit 1
C2DSR_LIB=variants/lib_rgstamp.so run python -u tools/rg_micro.py x3 || exit 1
run python -u tools/rg_micro.py wg || exit 1
run python -u tools/host_time.py fp32 || exit 1
cat $O
