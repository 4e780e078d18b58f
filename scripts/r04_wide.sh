#!/bin/bash
# Round-4 session: the wide GEMM (FFMI_WIDE) -- kernel parity at the model's
# shapes, the T = 168 microbenchmark, then the bench with it off / on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
S=scripts/gpu_step.sh
FFMI_WIDE=1 $S wide_parity 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread \
  tests/test_gpu_llama_shapes.py tests/test_gpu_kernels.py -k "baseline_shapes or fused or linear" || exit 1
grep -q "passed" gpurun_out/wide_parity.log && ! grep -q "failed" gpurun_out/wide_parity.log || exit 1
for w in 0 1 0 1; do
  FFMI_WIDE=$w timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b --T 168 --xpacked \
    --wstream --iters 40 > gpurun_out/wide_gemm_$w.log 2>&1 || exit 1
  echo "== FFMI_WIDE=$w"; tail -6 gpurun_out/wide_gemm_$w.log
done
timeout -k 10 700 bash scripts/gpu_ab.sh -r 2 "FFMI_WIDE=0" "FFMI_WIDE=1" || exit 1
