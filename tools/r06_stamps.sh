#!/bin/bash
# per-phase cycle stamps of the K5 tile loop (diagnostic builds variants/st_*): usage bash tools/r06_stamps.sh V1 V2 ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/r06_stamps.txt
: > $out
for v in "$@"; do
  C2DSR_LIB_DIR=variants/$v timeout -k 5 60 python -u tools/ce3b_micro.py 18944 63937 5 1 2>&1 | grep -E "ce3b|stamps" | sed "s|^|$v |" >> $out || { echo "fail $v" >> $out; exit 1; }
  C2DSR_LIB_DIR=variants/$v timeout -k 5 60 python -u tools/ce3_micro.py 18944 63937 12 1 2>&1 | grep -E "ce3 |stamps" | sed "s|^|$v |" >> $out || { echo "fail $v" >> $out; exit 1; }
done
cat $out
