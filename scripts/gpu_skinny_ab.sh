#!/bin/bash
# A/B of forced skinny GEMM shapes (FFMI_SKINNY="NT,KW") on decode / SSM shapes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; : > gpurun_out/skinny_ab.log
for V in "" "1,4" "1,8" "2,4" "2,8" "4,4" "4,2" "2,2"; do
  for C in 0 768; do
    echo "== FFMI_SKINNY='$V' cold_mb=$C" >> gpurun_out/skinny_ab.log
    FFMI_SKINNY="$V" timeout -k 10 120 python scripts/gemm_bench.py --shapes ssm --T 8,24 --cold-mb $C --iters 30 >> gpurun_out/skinny_ab.log 2>&1 || exit 1
  done
  echo "== FFMI_SKINNY='$V' llama7b cold" >> gpurun_out/skinny_ab.log
  FFMI_SKINNY="$V" timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b --T 8 --cold-mb 768 --iters 20 --ops qkv,o,down,lm_head >> gpurun_out/skinny_ab.log 2>&1 || exit 1
done
grep -v Warn gpurun_out/skinny_ab.log | tail -3
