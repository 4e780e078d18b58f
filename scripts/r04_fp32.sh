#!/bin/bash
# Round-4 session: the full-precision path (tests/test_gpu_full_precision.py),
# with a heartbeat file so the long phases (fp32 7B oracle, 8 rank processes)
# stay visibly alive.  FP32_K: a pytest -k filter.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
(while true; do date >> gpurun_out/heartbeat_fp32.log; sleep 30; done) &
HB=$!
timeout -k 10 1000 python -u -m pytest -v -x --timeout 900 --timeout-method thread \
  tests/test_gpu_full_precision.py ${FP32_K:+-k "$FP32_K"} > gpurun_out/fp32.log 2>&1
rc=$?
kill $HB
echo "[fp32] rc=$rc"; tail -30 gpurun_out/fp32.log
exit $rc
