#!/bin/bash
# run a micro-benchmark once per variant library directory:  bash tools/run_variants.sh SCRIPT.py "ARGS" NAME...
set -o pipefail
script=$1; args=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for n in "$@"; do
  C2DSR_LIB_DIR=variants/$n timeout -k 5 90 python -u $script $args 2>&1 | grep -v Warning | tail -2 | sed "s/^/$n /" || exit 1
done
