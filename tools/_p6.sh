#!/bin/bash
# one-off: attention backward with the dP loop's loads pipelined (ATTN_BPF) vs default
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do for v in default bpf; do
  if [ $v = default ]; then D=""; else D="variants/$v"; fi
  echo "== $v $rep"; timeout -k 5 90 env C2DSR_LIB_DIR=$D python -u tools/attn_micro.py 2>&1 | tail -1 || exit 1
done; done > gpurun_out/bpf.log
cut -c1-250 gpurun_out/bpf.log
timeout -k 10 200 env C2DSR_LIB_DIR=variants/bpf python3 -u -m pytest tests -m gpu -q --timeout 100 -k "attn" > gpurun_out/bpf_test.log 2>&1; tail -1 gpurun_out/bpf_test.log
