#!/bin/bash
# rocprofv3 kernel stats of the SpecInfer bench with and without the
# attention + o-projection fusion (FFMI_FUSE_AO), graphed steps traced one
# packet at a time
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp
B="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0"
FFMI_FUSE_AO=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_ao0 -o k -- python3 $B > "$R/gpurun_out/prof_ao0.log" 2>&1 && \
cp /tmp/p_ao0/k_kernel_stats.csv "$R/gpurun_out/ao0_kernel_stats.csv" && echo "[ao0] ok" && \
FFMI_FUSE_AO=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_ao1 -o k -- python3 $B > "$R/gpurun_out/prof_ao1.log" 2>&1 && \
cp /tmp/p_ao1/k_kernel_stats.csv "$R/gpurun_out/ao1_kernel_stats.csv" && echo "[ao1] ok"
