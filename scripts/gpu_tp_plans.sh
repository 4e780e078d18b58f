#!/bin/bash
# Sweep forced M-split plans (FFMI_GEMM_PLAN="NTW,S") on the TP = 8 per-rank
# GEMM shards at T = 168, cold weights (scripts/gemm_bench.py).
set -o pipefail
mkdir -p gpurun_out
for sh in llama7b_tp8 llama65b_tp8; do
  echo "== $sh planner"
  timeout -k 10 120 python scripts/gemm_bench.py --shapes $sh --T 168 --xpacked --wstream || exit 1
  for p in 2,1 2,2 2,4 2,8 4,2 4,4 4,8 6,2 6,4 6,8 8,4 8,8; do
    echo "== $sh plan $p"
    FFMI_GEMM_PLAN=$p timeout -k 10 120 python scripts/gemm_bench.py --shapes $sh --T 168 --xpacked --wstream || exit 1
  done
done
