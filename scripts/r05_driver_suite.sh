#!/bin/bash
# The driver's round-end GPU check as it runs it (round 5): the whole -m gpu
# suite under the driver's 900-s step limit, then smoke(), with a heartbeat.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
rm -f gpurun_out/*_progress.log gpurun_out/parity_report.jsonl
(while true; do date >> gpurun_out/heartbeat_suite.log; sleep 30; done) &
HB=$!
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu --durations=25 > gpurun_out/suite.log 2>&1
rc=$?
echo "[suite] rc=$rc"; tail -30 gpurun_out/suite.log
if [ $rc -eq 0 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "[smoke] rc=$rc"; tail -2 gpurun_out/smoke.log
fi
kill $HB
exit $rc
