#!/bin/bash
# Round 6: split-row softmax top-k -- microbenchmark (split factors forced
# by FFMI_TOPK_SPLIT), the top-k GPU tests, and the headline with per-step
# timing (FFMI_STEP_TIMING) for the SSM step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r06_topk}
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 30 "gpurun_out/$n.log"; return $rc; }
run ${TAG}_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "softmax or topk or argmax" && \
run ${TAG}_bench_topk 120 python scripts/topk_bench.py && \
for g in 1 2 4 16; do FFMI_TOPK_SPLIT=$g run ${TAG}_bench_topk_g$g 120 python scripts/topk_bench.py || exit 1; grep "T=24 V=32000 k=3\|T=8 V=32000" gpurun_out/${TAG}_bench_topk_g$g.log; done && \
FFMI_STEP_TIMING=1 run ${TAG}_bench 300 python bench.py --no-cpu-baseline --no-legs --no-incr --steps 3 --warmup 1 --profile 0 && \
grep "step timing" gpurun_out/${TAG}_bench.log | sort -t= -k3 -n | head -40
