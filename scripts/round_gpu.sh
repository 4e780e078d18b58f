#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats (csv).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
S=scripts/gpu_step.sh
TAG=${TAG:-r01}
$S kernels 600 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q && \
$S e2e 600 python -m pytest tests/test_gpu_e2e.py -m gpu -x -q && \
$S bench 900 python bench.py --steps 3 --warmup 1 && \
(export TMPDIR=/tmp; cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/prof.log" 2>&1; echo "[prof] rc=$?")
