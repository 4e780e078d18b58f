#!/bin/bash
# Auxiliary round profiles: per-rank TP shard compute (scripts/tp_shard_bench.py,
# TP = 1/2/4/8, LLaMA-7B SpecInfer and incr; LLaMA-65B TP = 8) and the rocprofv3
# kernel stats of incremental decoding (config B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r01}
: > gpurun_out/tp_shards.jsonl
for a in "--tp 1" "--tp 2" "--tp 4" "--tp 8" "--tp 8 --mode incr" "--tp 8 --model 65b" "--tp 8 --model 65b --mode incr"; do
  timeout -k 10 300 python scripts/tp_shard_bench.py $a >> gpurun_out/tp_shards.jsonl 2> gpurun_out/tp_err.log || { tail -5 gpurun_out/tp_err.log; exit 1; }
  tail -1 gpurun_out/tp_shards.jsonl | cut -c1-200
done
(export TMPDIR=/tmp FFMI_NO_GRAPHS=1; cd /tmp && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ffmi_incr -o incr -- python3 "$R/bench.py" --mode incr --steps 1 --warmup 1 --no-cpu-baseline --profile 0 > "$R/gpurun_out/incr_prof.log" 2>&1 && \
 cp /tmp/ffmi_incr/incr_kernel_stats.csv "$R/gpurun_out/${TAG}_incr_kernel_stats.csv" && echo "[incr prof] ok")
