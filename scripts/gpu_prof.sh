#!/bin/bash
# rocprofv3 kernel trace + stats of one bench step per arm (graph packets
# submitted one by one so the tracer can follow hipGraphLaunch).
#   scripts/gpu_prof.sh TAG [-b "BENCH ARGS"] [ARM ...]   (ARM as in gpu_ab.sh)
# Writes gpurun_out/TAG_<n>_kernel_stats.csv and a per-kernel summary
# (scripts/trace_groups.py) per arm.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=$1; shift
BARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0"
if [ "$1" = "-b" ]; then BARGS="$BARGS $2"; shift 2; fi
[ $# -eq 0 ] && set -- ""
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
n=0
for ARM in "$@"; do
  D=/tmp/ffmi_prof_${TAG}_$n
  (cd /tmp && env $ARM timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$D" -o b -- python3 "$R/bench.py" $BARGS > "$R/gpurun_out/${TAG}_$n.log" 2>&1) || {
    echo "arm '$ARM' failed"; tail -5 "gpurun_out/${TAG}_$n.log"; exit 1; }
  cp "$D/b_kernel_stats.csv" "gpurun_out/${TAG}_${n}_kernel_stats.csv"
  echo "== arm '$ARM' -> gpurun_out/${TAG}_${n}_kernel_stats.csv"
  python3 scripts/trace_groups.py "$D/b_kernel_trace.csv" 2>/dev/null | head -40
  n=$((n + 1))
done
