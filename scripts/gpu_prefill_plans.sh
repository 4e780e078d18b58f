# forced M-split plans at the prefill size (T = 1024) for the LLaMA-7B shapes
set -o pipefail
mkdir -p gpurun_out
echo "== planner"
timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b --T 1024 --xpacked --wstream --iters 10 || exit 1
for p in 4,1 6,1 8,1 12,1 16,1 8,2 16,2; do
  echo "== plan $p"
  FFMI_GEMM_PLAN=$p timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b --T 1024 --xpacked --wstream --iters 10 || exit 1
done
