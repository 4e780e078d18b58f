#!/bin/bash
# In-model A/B of environment settings: bench line per setting (SpecInfer,
# no incr side run), op breakdown and SSM step cost.
#   scripts/gpu_env_ab2.sh "" "FFMI_X=1" "FFMI_Y=0 FFMI_Z=2"
set -o pipefail
mkdir -p gpurun_out
for E in "$@"; do
  echo "== env '$E'"
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-incr --steps 2 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -3 gpurun_out/ab.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/ab.json'):
    if l.startswith('{'):
        d=json.loads(l); o=d['op_breakdown_sampled']; print(d['value'], 'verify_ms', d['verify_step_ms'], 'ssm_us', d['ssm_step_us'], {k:o[k]['avg_us'] for k in o})"
done
