#!/bin/bash
# Round-6 baseline session (one gpurun call): the top-k microbenchmark, a
# kernel trace of one headline generate (SSM / verify step timelines, the
# trace csv copied back for offline analysis) and the headline with op
# profiling off and on (same box).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r06_base}
run() { local n=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "gpurun_out/$n.log" 2>&1; local rc=$?; echo "[$n] rc=$rc"; [ $rc -eq 0 ] || tail -n 20 "gpurun_out/$n.log"; return $rc; }
run ${TAG}_topk 120 python scripts/topk_bench.py && \
(export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; cd /tmp && \
 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/${TAG}_tl -o bench -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-incr --no-legs --profile 0 > "$R/gpurun_out/${TAG}_tl.log" 2>&1) && \
cp /tmp/${TAG}_tl/bench_kernel_trace.csv gpurun_out/${TAG}_trace.csv && \
python3 scripts/step_timeline.py gpurun_out/${TAG}_trace.csv --gap 6 --skip 40 > gpurun_out/${TAG}_timeline.txt && \
run ${TAG}_bench_p0 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 2 --profile 0 && \
run ${TAG}_bench_p1 300 python bench.py --no-cpu-baseline --no-legs --steps 5 --warmup 2 --profile 1 && \
run ${TAG}_bench_p0b 300 python bench.py --no-cpu-baseline --no-legs --no-incr --steps 5 --warmup 2 --profile 0
