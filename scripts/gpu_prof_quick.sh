#!/bin/bash
# Kernel stats of one SpecInfer generate (no graphs: rocprofv3 tracing crashes
# inside HIP graph capture); TAG names the output directory.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-quick}
export TMPDIR=/tmp FFMI_NO_GRAPHS=1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-incr --profile 0 "$@" > "$R/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "[prof_$TAG] rc=$rc"; exit $rc
