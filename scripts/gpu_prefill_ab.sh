# in-model A/B of the prefill-block plan (FFMI_PREFILL_PLAN) + the T = 1024 sweep
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do FFMI_PREFILL_PLAN=$v timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b --T 1024 --xpacked --wstream --iters 10 || exit 1; done
BENCH_ARGS="--no-incr" timeout -k 10 900 bash scripts/gpu_env_bench_ab.sh FFMI_PREFILL_PLAN=1 FFMI_PREFILL_PLAN=0 FFMI_PREFILL_PLAN=1 FFMI_PREFILL_PLAN=0 > gpurun_out/prefill_ab.log 2>&1 || { tail -20 gpurun_out/prefill_ab.log; exit 1; }
cut -c1-150 gpurun_out/prefill_ab.log
