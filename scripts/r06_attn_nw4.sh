#!/bin/bash
# Round 6: decode attention with 4 waves per workgroup (FFMI_ATTN_NW4=1) --
# the attention tests with it forced, then incremental decoding, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
FFMI_ATTN_NW4=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "attention or attn" > gpurun_out/nw4_tests.log 2>&1 || { tail -30 gpurun_out/nw4_tests.log; exit 1; }
tail -1 gpurun_out/nw4_tests.log
bash scripts/gpu_ab.sh -r 3 -b "--mode incr --no-legs" "" "FFMI_ATTN_NW4=1"
