#!/bin/bash
# Round 6: decode qkv (fused-norm consumer, T = 8, one row tile) with two
# weight tiles per workgroup (FFMI_FZ_NT2=1) vs one, incremental decoding,
# same box, alternating; then the fused-norm equality tests with it forced.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash scripts/gpu_ab.sh -r 3 -b "--mode incr --no-legs" "" "FFMI_FZ_NT2=1" || exit 1
FFMI_FZ_NT2=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "fused" > gpurun_out/fz_tests.log 2>&1 && tail -2 gpurun_out/fz_tests.log
