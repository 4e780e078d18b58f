#!/bin/bash
# Round 6: chained SSM beam steps -- GPU tests (chained == stepwise, e2e),
# then the headline with per-step timing, chained and stepwise (same box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r06_chain}
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 40 "gpurun_out/$n.log"; return $rc; }
run ${TAG}_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_kernels.py -k "e2e or softmax or topk or argmax or chained or spec or graph" && \
run ${TAG}_bench1 300 python bench.py --no-cpu-baseline --no-legs --no-incr --steps 5 --warmup 2 --profile 0 && \
FFMI_SSM_CHAIN=0 run ${TAG}_bench0 300 python bench.py --no-cpu-baseline --no-legs --no-incr --steps 5 --warmup 2 --profile 0 && \
run ${TAG}_bench1b 300 python bench.py --no-cpu-baseline --no-incr --steps 5 --warmup 2 --profile 0 && \
for f in bench1 bench0 bench1b; do python3 - "gpurun_out/${TAG}_$f.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[1], d["value"], "verify", d.get("verify_step_ms"), "ssm", d.get("ssm_step_us"), d.get("time_split_ms_per_generate"),
      {k: (v.get("value"), v.get("ssm_step_us")) for k, v in d.items() if k.startswith("spec_")})
PY
done
