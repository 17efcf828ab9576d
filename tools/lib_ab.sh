#!/bin/bash
# Same-box A/B of library builds on a bench line: bash tools/lib_ab.sh ROUNDS VARIANT... [-- BENCH ARGS]
# ("default" = the in-tree libraries; others: variants/NAME from tools/lib_variant.sh), alternating per round.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
R=$1; shift
V=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done; [ "$1" = "--" ] && shift
for r in $(seq 1 $R); do for v in "${V[@]}"; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  line=$(timeout -k 10 300 env C2DSR_LIB_DIR=$D python3 bench.py --no-cpu-baseline --no-extra "$@" 2>/dev/null | tail -1) || exit 1
  echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done; done
