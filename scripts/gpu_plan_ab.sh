set -o pipefail
mkdir -p gpurun_out
for plan in none 12,2 16,2 16,3 6,1 12,1; do
  if [ "$plan" = none ]; then unset FFMI_GEMM_PLAN; else export FFMI_GEMM_PLAN=$plan; fi
  echo "plan $plan"
  timeout -k 10 120 python -u scripts/gemm_bench.py --shapes llama7b --ops gate_up,qkv --T 168 --xpacked --wstream --iters 40 || exit 1
done
