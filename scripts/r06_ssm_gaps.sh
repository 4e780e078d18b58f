#!/bin/bash
# Round 6: kernel trace of the headline bench (one timed generate, no side
# runs) -> idle time inside and between the chained SSM beam steps
# (scripts/ssm_gaps.py); then gate/up plans with 4-6 tiles x 3-8 slices on the
# LLaMA-7B TP = 8 shard (repeated pairs: the first launch of a sweep runs slow).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/tl
export TMPDIR=/tmp
# (graph packets one by one: the tracer faults in hipGraphLaunch otherwise,
# DESIGN.md §6 -- so the boundaries are those of packet-by-packet submission)
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o bench -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-incr --no-legs --profile 0 \
  > gpurun_out/tl/bench.log 2>&1 || { tail -5 gpurun_out/tl/bench.log; exit 1; }
f=$(ls gpurun_out/tl/*kernel_trace.csv | head -1)
python3 scripts/ssm_gaps.py "$f" | tee gpurun_out/r06_ssm_gaps.log
rm -f gpurun_out/tl/*.csv
OUT=gpurun_out/r06_tp8_gateup2.log
: > $OUT
for rep in 1 2; do
  for p in 6,8 4,4 4,5 4,7 6,5 4,3 2,4; do
    echo "plan $p" >> $OUT
    FFMI_GEMM_PLAN="$p" timeout -k 10 120 python scripts/gemm_bench.py --shapes llama7b_tp8 \
      --T 168 --xpacked --wstream --ops gate_up >> $OUT 2>gpurun_out/plans.err || { tail -5 gpurun_out/plans.err; exit 1; }
  done
done
echo done
