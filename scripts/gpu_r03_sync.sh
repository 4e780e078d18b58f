#!/bin/bash
# Host wait mode A/B (FFMI_SYNC: HIP default / spin / yield / blocking) on the
# SpecInfer bench, alternating on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
B="python bench.py --no-cpu-baseline --steps 3 --warmup 1"
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 30 "gpurun_out/$n.log"; return $rc; }
j() { grep -h "FFMI_SYNC" "gpurun_out/$1.log"; grep '^{' "gpurun_out/$1.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ssm_step_us'], d['verify_step_ms'], d['time_split_ms_per_generate'], d['incr_decoding']['value'])"; }
run s_def_a 200 $B && j s_def_a && \
run s_spin_a 200 env FFMI_SYNC=spin $B && j s_spin_a && \
run s_yield_a 200 env FFMI_SYNC=yield $B && j s_yield_a && \
run s_block_a 200 env FFMI_SYNC=block $B && j s_block_a && \
run s_def_b 200 $B && j s_def_b && \
run s_spin_b 200 env FFMI_SYNC=spin $B && j s_spin_b
