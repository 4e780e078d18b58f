# In-model A/B of per-shape GEMM plans (FFMI_GEMM_PLAN="N:K:NTW,S;...").
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/model_plans.log
for plan in "" "4096:4096:8,4" "4096:11008:8,4" "4096:4096:16,8;4096:11008:16,8" "4096:11008:12,8" "12288:4096:12,4"; do
  echo "== plan '$plan'" >> gpurun_out/model_plans.log
  FFMI_GEMM_PLAN="$plan" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-incr > gpurun_out/mp.json 2>> gpurun_out/model_plans.log || exit 1
  python - >> gpurun_out/model_plans.log <<'PY'
import json
d = json.loads(open("gpurun_out/mp.json").read().strip().splitlines()[-1])
ob = d.get("op_breakdown_sampled", {})
print(d["value"], d["time_split_ms_per_generate"], {k: v["avg_us"] for k, v in ob.items()})
PY
done
cat gpurun_out/model_plans.log
