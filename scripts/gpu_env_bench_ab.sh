#!/bin/bash
# Bench-only A/B of environment settings: scripts/gpu_env_bench_ab.sh "VAR=a" "VAR=b" ...
# (extra bench.py flags via BENCH_ARGS, e.g. BENCH_ARGS="--profile 0")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for P in "$@"; do
  echo "== $P"
  env $P timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 $BENCH_ARGS > gpurun_out/eb.json 2>gpurun_out/eb.err || { tail -3 gpurun_out/eb.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/eb.json'):
    if l.startswith('{'):
        d=json.loads(l); o=d.get('op_breakdown_sampled', {}); print(d['value'], d['time_split_ms_per_generate'], d.get('incr_decoding', {}).get('value'), {k: v['avg_us'] for k, v in o.items()})"
done
