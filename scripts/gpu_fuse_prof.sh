# rocprof kernel stats of the bench with fused norms on / off
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
for v in 1 0; do
  (cd /tmp && FFMI_FUSE_NORM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fp$v -o b -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/fuse_prof_$v.log" 2>&1) || exit 1
  cp /tmp/fp$v/b_kernel_stats.csv "$R/gpurun_out/fuse_stats_$v.csv"
done
