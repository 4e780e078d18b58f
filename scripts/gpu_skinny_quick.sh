#!/bin/bash
# Decode / SSM skinny GEMM shapes (cold and warm weights) + the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; : > gpurun_out/skq.log
timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b --T 8 --cold-mb 768 --iters 20 >> gpurun_out/skq.log 2>&1 && \
timeout -k 10 120 python scripts/gemm_bench.py --shapes ssm --T 8,24 --cold-mb 0 --iters 30 >> gpurun_out/skq.log 2>&1 && \
grep '^{' gpurun_out/skq.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['op'], d['T'], d['N'], d['K'], 'cold' if d['copies']>1 else 'warm', d['us'], d['GBps'])"
