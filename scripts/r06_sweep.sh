#!/bin/bash
# Round 6: one-off randomised parity sweep at fresh seeds over the paths this
# round added (chained SSM beam steps, split-row top-k, the all-reduce with the
# residual norm folded in -- two-shot forced so small TP shapes take it).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export FFMI_RANDOM_SEED_OFFSET=${OFF:-70000}
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
(while true; do date >> gpurun_out/heartbeat_sweep.log; sleep 30; done) &
HB=$!
rc=0
FFMI_RANDOM_SCALE=${KS:-5} timeout -k 10 400 $PT tests/test_gpu_kernels.py -k "random" > gpurun_out/sweep_kernels.log 2>&1 || rc=1
tail -2 gpurun_out/sweep_kernels.log
[ $rc -eq 0 ] && { FFMI_RANDOM_SCALE=${PS:-3} FFMI_PEER_TWO_SHOT_MIN=0 timeout -k 10 400 $PT tests/test_gpu_peer.py -k "random" > gpurun_out/sweep_peer.log 2>&1 || rc=1; tail -2 gpurun_out/sweep_peer.log; }
[ $rc -eq 0 ] && { FFMI_RANDOM_SEEDS=${MS:-60} timeout -k 10 500 $PT tests/test_gpu_random_models.py > gpurun_out/sweep_models.log 2>&1 || rc=1; tail -2 gpurun_out/sweep_models.log; }
kill $HB
[ $rc -eq 0 ] || { for f in gpurun_out/sweep_*.log; do grep -m3 -A30 "FAILED\|Error" $f | head -60; done; }
exit $rc
