# In-model A/B: one-launch attention vs KV-update + attention (FFMI_ATTN_NO_FUSE).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/attn_ab.log
for env in "" "FFMI_ATTN_NO_FUSE=1"; do
  echo "== $env" >> gpurun_out/attn_ab.log
  env $env timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-incr > gpurun_out/ab.json 2>> gpurun_out/attn_ab.log || exit 1
  python - >> gpurun_out/attn_ab.log <<'PY'
import json
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
ob = d.get("op_breakdown_sampled", {})
print(d["value"], d["time_split_ms_per_generate"], {k: v["avg_us"] for k, v in ob.items()})
PY
done
cat gpurun_out/attn_ab.log
