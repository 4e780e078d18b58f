#!/bin/bash
# Generic A/B of an environment toggle: scripts/gpu_env_ab.sh VAR VALUE
# runs the T=168 GEMM bench, the GPU tests and the bench with VAR unset and set.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
VAR=$1; VAL=$2
for P in 0 1; do
  if [ $P = 1 ]; then export $VAR=$VAL; fi
  echo "== $VAR set=$P"
  timeout -k 10 120 python scripts/gemm_bench.py --T 168 --xpacked --iters 20 > gpurun_out/ab$P.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab$P.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['op'], d['T'], d['us'], d['GBps'])"
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_e2e.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_t$P.log 2>&1; echo "tests rc=$?"; tail -1 gpurun_out/ab_t$P.log
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-incr --steps 2 > gpurun_out/ab_b$P.json 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/ab_b$P.json'):
    if l.startswith('{'):
        d=json.loads(l); o=d['op_breakdown_sampled']; print(d['value'], d['time_split_ms_per_generate'], {k:o[k]['avg_us'] for k in o})"
done
