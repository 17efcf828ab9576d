set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r06s_gputest.log 2>&1; echo "gputest rc=$?"
tail -4 gpurun_out/r06s_gputest.log
