#!/bin/bash
# In-model A/B of forced M-split plans (FFMI_GEMM_PLAN), bench only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for P in "" "$@"; do
  echo "== plan '$P'"
  FFMI_GEMM_PLAN="$P" timeout -k 10 300 python bench.py --no-cpu-baseline --no-incr --steps 2 > gpurun_out/pm.json 2>gpurun_out/pm.err || { tail -3 gpurun_out/pm.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/pm.json'):
    if l.startswith('{'):
        d=json.loads(l); o=d['op_breakdown_sampled']; print(d['value'], d['time_split_ms_per_generate']['llm_steps'], {k:o[k]['avg_us'] for k in o})"
done
