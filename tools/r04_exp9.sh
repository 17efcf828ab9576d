#!/bin/bash
# K5 at two waves per SIMD (variants/lib_ce8.so) vs the default: timing, the ce3 tests on the variant, and one PMC
# pass per library on the micro (LDS bank conflicts / LDS-array cycles / waits / MFMA busy)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/exp9.log
: > $O
run() { echo "== $*" >> $O; timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids >> $O; }
for v in base ce8; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O
  C2DSR_LIB=$L run python -u tools/ce3_micro.py || { cat $O; exit 1; }; done
C2DSR_LIB=variants/lib_ce8.so run python -u -m pytest tests/test_gpu_ce3.py -q -x --timeout 200 --timeout-method thread || { cat $O; exit 1; }
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"
for v in base ce8; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so
  C2DSR_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/exp9_$v -o run --output-format csv -- python3 tools/ce3_micro.py > gpurun_out/exp9_$v.log 2>&1 || { echo "pmc $v failed" >> $O; cat $O; exit 1; }
  python tools/pmc_kernels.py gpurun_out/exp9_$v ce3_kernel >> $O 2>&1; done
cat $O
O2=gpurun_out/exp9b.log
: > $O2
for v in base rgnow; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== $v" >> $O2
  C2DSR_LIB=$L timeout -k 10 150 python -u tools/rg_micro.py x3 2>&1 | grep -v amdgpu.ids >> $O2 || exit 1; done
cat $O2
