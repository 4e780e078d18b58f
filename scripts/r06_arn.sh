#!/bin/bash
# Round 6: the all-reduce with the residual norm folded in -- op-level and
# model-level equality with the unfused pair, then the whole transport suite.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_peer.py -k "rmsnorm or fused_norm" > gpurun_out/arn_new.log 2>&1 || { tail -40 gpurun_out/arn_new.log; exit 1; }
tail -3 gpurun_out/arn_new.log
timeout -k 10 900 $PT tests/test_gpu_peer.py tests/test_gpu_tp_local.py -k "not rmsnorm and not fused_norm" > gpurun_out/arn_suite.log 2>&1 || { tail -40 gpurun_out/arn_suite.log; exit 1; }
tail -3 gpurun_out/arn_suite.log
[ -n "$NO_GAPS" ] || bash scripts/r06_ssm_gaps.sh
