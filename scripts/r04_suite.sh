#!/bin/bash
# Round-4 session: the whole -m gpu suite (minus the 65B test) and smoke(),
# with a heartbeat file for the long phases.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
(while true; do date >> gpurun_out/heartbeat_suite.log; sleep 30; done) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 620 --timeout-method thread \
  --deselect tests/test_gpu_llama65b_tp.py > gpurun_out/suite.log 2>&1
rc=$?
echo "[suite] rc=$rc"; tail -15 gpurun_out/suite.log
if [ $rc -eq 0 ]; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "[smoke] rc=$rc"; tail -3 gpurun_out/smoke.log
fi
kill $HB
exit $rc
