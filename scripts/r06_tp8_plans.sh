#!/bin/bash
# Round 6: forced M-split plans (FFMI_GEMM_PLAN="NTW,S") on the LLaMA-7B TP = 8
# per-rank shapes at T = 168 (packed X, streamed weights, as the verify step),
# against the default plan; then the residual norm at the rows one rank owns
# under a reduce-scatter (T / 8 = 21) vs all 168.  One JSON line per shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-r06_tp8_plans}.log
: > $OUT
SH=${SHAPES:-llama7b_tp8}
OPS=${OPS:-}
gb() { for sh in $SH; do timeout -k 10 120 python scripts/gemm_bench.py --shapes $sh --T ${TS:-168} --xpacked --wstream --ops "$OPS" "$@" || return 1; done; }
echo "plan default" >> $OUT
gb >> $OUT 2>gpurun_out/plans.err || { tail -5 gpurun_out/plans.err; exit 1; }
for ntw in 2 4 6 8 12 16; do
  for s in 1 2 3 4 6 8; do
    echo "plan $ntw,$s" >> $OUT
    FFMI_GEMM_PLAN="$ntw,$s" gb >> $OUT 2>gpurun_out/plans.err || { tail -5 gpurun_out/plans.err; exit 1; }
  done
done
[ -n "$NO_NORM" ] || timeout -k 10 120 python scripts/norm_bench.py --rows 21,168 >> $OUT 2>gpurun_out/plans.err || { tail -5 gpurun_out/plans.err; exit 1; }
echo done
