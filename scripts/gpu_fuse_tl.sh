# step timelines (span, busy, idle per step class) with fused norms on / off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for v in 1 0; do
  (cd /tmp && FFMI_FUSE_NORM=$v timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl$v -o b -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/fuse_tl_$v.log" 2>&1) || exit 1
  python3 "$R/scripts/step_timeline.py" /tmp/tl$v/b_kernel_trace.csv > "$R/gpurun_out/fuse_tl_$v.txt" || exit 1
  echo "== fuse $v"; grep -A22 "^ssm" "$R/gpurun_out/fuse_tl_$v.txt" | head -24
done
