set -o pipefail
bash tools/evidence_a.sh r06j || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r06j_gputest.log 2>&1; echo "gputest rc=$?"
tail -2 gpurun_out/r06j_gputest.log
