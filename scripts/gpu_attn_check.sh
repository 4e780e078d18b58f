#!/bin/bash
# Attention change check: GPU parity (kernels, e2e, TP), in-model timeline,
# bench.  Stops at the first failing step (no GPU work after a failure).
set -o pipefail
mkdir -p gpurun_out
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; tail -n 30 "gpurun_out/$n.log"; return $rc; }
run gputests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
run diag 200 python scripts/diag_attn_model.py && \
run bench 300 python bench.py --no-cpu-baseline
