#!/bin/bash
# Same-box A/B of environment knobs on the bench's side legs (tree width 4,
# four SSMs, token chain) and the headline: one line per run.
#   scripts/legs_ab.sh [-r REPS] ARM [ARM ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
REPS=1
while getopts "r:" o; do case $o in r) REPS=$OPTARG;; *) exit 2;; esac; done
shift $((OPTIND - 1))
: > gpurun_out/legs_ab.log
for rep in $(seq "$REPS"); do
  for ARM in "$@"; do
    env $ARM timeout -k 10 400 python bench.py --no-cpu-baseline --no-incr --steps 2 --warmup 1 \
      > gpurun_out/legs_run.json 2> gpurun_out/legs_run.err || {
      echo "arm '$ARM' failed"; tail -5 gpurun_out/legs_run.err; exit 1; }
    python3 - "$ARM" "$rep" <<'PY' | tee -a gpurun_out/legs_ab.log
import json, sys
d = json.loads([l for l in open("gpurun_out/legs_run.json") if l.startswith("{")][-1])
legs = " ".join(f"{k}={d[k]['value']} (verify {d[k].get('verify_step_ms')} ms, ssm {d[k].get('ssm_step_us')} us)"
                for k in ("spec_width4", "spec_4ssm", "spec_token_chain") if k in d)
print(f"rep {sys.argv[2]} arm '{sys.argv[1]}': headline {d['value']} (ssm {d.get('ssm_step_us')} us); {legs}")
PY
  done
done
