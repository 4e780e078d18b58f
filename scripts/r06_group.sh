#!/bin/bash
# Round 6: chained SSM slots launched several per graph (FFMI_CHAIN_GROUP):
# equality with the stepwise loop, then same-box A/B on the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_e2e.py -k chained > gpurun_out/group_tests.log 2>&1 || { tail -30 gpurun_out/group_tests.log; exit 1; }
tail -2 gpurun_out/group_tests.log
bash scripts/gpu_ab.sh -r 3 "" "FFMI_CHAIN_GROUP=3" "FFMI_CHAIN_GROUP=6"
