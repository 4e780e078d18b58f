#!/bin/bash
# Same-box A/B of environment knobs on a C-ABI microbenchmark.
#   scripts/gpu_kernel_ab.sh "BENCH CMD" ARM [ARM ...]
# e.g. scripts/gpu_kernel_ab.sh "scripts/gemm_bench.py --shapes llama7b --T 168 --xpacked --wstream" \
#        "" "FFMI_GEMM_PLAN=12,2" "FFMI_MID_ULD=0"
#      scripts/gpu_kernel_ab.sh "scripts/attn_bench.py --iters 20" "" "FFMI_ATTN_QSPLIT=2"
# (the GEMM plan sweeps of DESIGN.md §5 -- FFMI_GEMM_PLAN="NTW,S" or
# "N:K:NTW,S;..." -- and FFMI_PREFILL_PLAN / FFMI_SKINNY arms run this way).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
CMD=$1; shift
for ARM in "$@"; do
  echo "== arm '$ARM'" | tee -a gpurun_out/kernel_ab.log
  env $ARM timeout -k 10 200 python3 $CMD 2>&1 | tee -a gpurun_out/kernel_ab.log || exit 1
done
