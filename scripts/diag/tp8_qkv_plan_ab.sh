#!/bin/bash
# TP = 8 shard bench: the qkv GEMM's split-K plan against the verify
# attention that consumes its slabs (per-rank compute, one box)
set -o pipefail
mkdir -p gpurun_out; : > gpurun_out/tp8_qkv_ab.log
for rep in 1 2; do
for ARM in "" "FFMI_GEMM_PLAN=1536:4096:2,1" "FFMI_GEMM_PLAN=1536:4096:2,2" "FFMI_GEMM_PLAN=1536:4096:4,2" "FFMI_GEMM_PLAN=1536:4096:2,4" "FFMI_GEMM_PLAN=1536:4096:4,4"; do
  env $ARM timeout -k 10 200 python scripts/tp_shard_bench.py --tp 8 --steps 2 > gpurun_out/tp8_run.json 2> gpurun_out/tp8_run.err || { echo "arm '$ARM' failed"; tail -5 gpurun_out/tp8_run.err; exit 1; }
  python3 - "$ARM" <<'PY' | tee -a gpurun_out/tp8_qkv_ab.log
import json, sys
d = json.loads([l for l in open("gpurun_out/tp8_run.json") if l.startswith("{")][-1])
o = d["ops_avg_us"]
print(f"arm '{sys.argv[1]}': {d['s_per_generate']} s/gen, qkv {o.get('gemm_qkv')} attn {o.get('attention')} sum {round(o.get('gemm_qkv',0)+o.get('attention',0),2)}")
PY
done
done
