#!/bin/bash
# Bench A/B of library build variants: scripts/gpu_lib_ab.sh "" v2 ...
# ("" = libffmi.so; "v2" = flexflow_amd/libffmi_v2.so, built beforehand with
#  make -C flexflow_amd/csrc BUILD=build_v2 OUT=../libffmi_v2.so EXTRA=-D...;
#  the round-1 weight-cache-policy trial was run this way before it became
#  the FFMI_W_STREAM flag).
# Each variant runs SpecInfer (with the incr side run) twice, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rep in 1 2; do
for V in "$@"; do
  echo "== variant '${V}' rep $rep"
  FFMI_LIB_VARIANT=$V timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/lab.json 2>gpurun_out/lab.err || { tail -3 gpurun_out/lab.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/lab.json'):
    if l.startswith('{'):
        d=json.loads(l); o=d['op_breakdown_sampled']
        print(d['value'], d['time_split_ms_per_generate'], 'incr', d['incr_decoding']['value'],
              {k: v['avg_us'] for k, v in o.items()})"
done
done
