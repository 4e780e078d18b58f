#!/bin/bash
# Attention + o-projection fusion (OprojArgs): GPU tests, then an alternating
# same-box A/B of the SpecInfer bench (FFMI_FUSE_AO=0 / 1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --no-incr --steps 3 --warmup 1"
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 30 "gpurun_out/$n.log"; return $rc; }
j() { grep '^{' "gpurun_out/$1.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ssm_step_us'], d['verify_step_ms'])"; }
run t_ao 400 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread && \
run ao0_a 200 env FFMI_FUSE_AO=0 $B && j ao0_a && \
run ao1_a 200 env FFMI_FUSE_AO=1 $B && j ao1_a && \
run ao0_b 200 env FFMI_FUSE_AO=0 $B && j ao0_b && \
run ao1_b 200 env FFMI_FUSE_AO=1 $B && j ao1_b
