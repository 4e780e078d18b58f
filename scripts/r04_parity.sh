#!/bin/bash
# Round-4 session: the parity tests added this round (bench workload at full
# depth, negative control, token-chain literal bars), then the 65B TP test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
rm -f gpurun_out/*_progress.log
S=scripts/gpu_step.sh
$S parity_bw 640 python -u -m pytest -v --timeout 620 --timeout-method thread \
  tests/test_gpu_bench_workload.py tests/test_gpu_token_chain.py || exit 1
if [ "${WITH_65B:-0}" = 1 ]; then
  $S parity_65b 1000 python -u -m pytest -v --timeout 980 --timeout-method thread \
    tests/test_gpu_llama65b_tp.py || exit 1
fi
