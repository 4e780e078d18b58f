# kernel timeline of the graphed bench steps (graph packets submitted one by
# one: DEBUG_CLR_GRAPH_PACKET_CAPTURE=0) -> step summary
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/ffmi_tl -o bench -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/timeline.log" 2>&1 && \
python3 "$R/scripts/step_timeline.py" /tmp/ffmi_tl/bench_kernel_trace.csv --skip 0 > "$R/gpurun_out/${TAG:-r03}_step_timeline.txt" && echo "[timeline] ok"
