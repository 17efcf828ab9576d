#!/bin/bash
# K5 MODE 0 (fwd_u) on compiler-visible MFMAs, MODE 1 (dw) on asm triples (variants/lib_bi0.so) vs the default,
# interleaved A/B at MB head-b shapes, then the ce3 tests on the variant
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp10.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for r in 1 2; do for v in base bi0; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L run python -u tools/ce3_micro.py || { cat $O; exit 1; }; done; done
C2DSR_LIB=variants/lib_bi0.so run python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 200 --timeout-method thread
cat $O
O2=gpurun_out/exp10b.log
: > $O2
for v in base rgco base rgco; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O2
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/rg_micro.py x3 2>&1 | grep -v amdgpu.ids >> $O2 || exit 1; done
cat $O2
