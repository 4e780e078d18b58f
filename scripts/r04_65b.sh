#!/bin/bash
# Round-4 session: configs D/E at full size (tests/test_gpu_llama65b_tp.py),
# with a heartbeat file so the long phases stay visibly alive.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
(while true; do date >> gpurun_out/heartbeat_65b.log; sleep 30; done) &
HB=$!
timeout -k 10 1050 python -u -m pytest -v -x --timeout 1040 --timeout-method thread \
  tests/test_gpu_llama65b_tp.py ${K65:+-k "$K65"} > gpurun_out/parity_65b.log 2>&1
rc=$?
kill $HB
echo "[parity_65b] rc=$rc"; tail -30 gpurun_out/parity_65b.log
exit $rc
