#!/bin/bash
# Same-box A/B of environment knobs on the bench (one gpurun session).
#   scripts/gpu_ab.sh [-r REPS] [-b "BENCH ARGS"] ARM [ARM ...]
# An ARM is a space-separated list of VAR=VALUE settings ("" = defaults), e.g.
#   scripts/gpu_ab.sh -r 2 "" "FFMI_FUSE_NORM=0" "FFMI_GEMM_PLAN=4096:11008:8,4"
#   scripts/gpu_ab.sh -b "--mode incr" "" "FFMI_W_TILE_MAJOR=1"
#   scripts/gpu_ab.sh "" "FFMI_LIB_VARIANT=nopipe"   (a library build variant)
# The arms alternate REPS times; each run is bounded; one summary line per run
# (tokens/s, verify step, SSM step, dominant GEMM) goes to stdout and
# gpurun_out/ab.log.  Stops at the first failing run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
REPS=1; BARGS="--no-cpu-baseline --no-incr --steps 3 --warmup 1"
while getopts "r:b:" o; do case $o in r) REPS=$OPTARG;; b) BARGS="--no-cpu-baseline --steps 3 --warmup 1 $OPTARG";; *) exit 2;; esac; done
shift $((OPTIND - 1))
: > gpurun_out/ab.log
for rep in $(seq "$REPS"); do
  for ARM in "$@"; do
    env $ARM timeout -k 10 400 python bench.py $BARGS > gpurun_out/ab_run.json 2> gpurun_out/ab_run.err || {
      echo "arm '$ARM' failed"; tail -5 gpurun_out/ab_run.err; exit 1; }
    python3 - "$ARM" "$rep" <<'PY' | tee -a gpurun_out/ab.log
import json, sys
d = json.loads([l for l in open("gpurun_out/ab_run.json") if l.startswith("{")][-1])
rf = d.get("roofline", {})
print(f"rep {sys.argv[2]} arm '{sys.argv[1]}': {d['value']} tok/s, verify {d.get('verify_step_ms')} ms, "
      f"ssm {d.get('ssm_step_us')} us, {rf.get('kernel')} {rf.get('avg_launch_us')} us "
      f"(frac {rf.get('frac')}); ops " +
      " ".join(f"{k}={v['avg_us']}" for k, v in d.get("op_breakdown_sampled", {}).items()))
PY
  done
done
