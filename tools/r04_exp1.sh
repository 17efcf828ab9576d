#!/bin/bash
# Round-4 micro-benchmarks: K5 (ce3) with phase stamps, embedding backward pieces, x3 projections.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/exp1.log
: > $O
timeout -k 10 120 python -u tools/ce3_micro.py >> $O 2>&1 || { tail -20 $O; exit 1; }
C2DSR_LIB=variants/lib_stamp.so timeout -k 10 120 python -u tools/ce3_micro.py >> $O 2>&1 || { tail -20 $O; exit 1; }
C2DSR_LIB=variants/lib_stamp.so timeout -k 10 120 python -u tools/ce3_micro.py 18944 36845 >> $O 2>&1 || { tail -20 $O; exit 1; }
for v in base pref2 pref4 pref8 pref4c32 pref8c32; do L=c2dsr_amd/libc2dsr_hip.so; [ $v != base ] && L=variants/lib_$v.so; echo "== embed $v" >> $O; C2DSR_LIB=$L timeout -k 10 120 python -u tools/embed_micro.py >> $O 2>&1 || { tail -20 $O; exit 1; }; done
timeout -k 10 120 python -u tools/rg_micro.py x3 >> $O 2>&1 || { tail -20 $O; exit 1; }
C2DSR_LIB=variants/lib_rgstamp.so timeout -k 10 120 python -u tools/rg_micro.py x3 >> $O 2>&1 || { tail -20 $O; exit 1; }
timeout -k 10 120 python -u tools/rg_micro.py wg >> $O 2>&1 || { tail -20 $O; exit 1; }
cat $O
