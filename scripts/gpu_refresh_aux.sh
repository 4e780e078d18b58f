#!/bin/bash
# Auxiliary round profiles: per-rank TP shard compute (scripts/tp_shard_bench.py,
# TP = 1/2/4/8, LLaMA-7B SpecInfer and incr; LLaMA-65B TP = 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r02}
: > gpurun_out/tp_shards.jsonl
for a in "--tp 1" "--tp 2" "--tp 4" "--tp 8" "--tp 8 --mode incr" "--tp 8 --model 65b" "--tp 8 --model 65b --mode incr"; do
  timeout -k 10 300 python scripts/tp_shard_bench.py $a >> gpurun_out/tp_shards.jsonl 2> gpurun_out/tp_err.log || { tail -5 gpurun_out/tp_err.log; exit 1; }
  tail -1 gpurun_out/tp_shards.jsonl | cut -c1-200
done
cp gpurun_out/tp_shards.jsonl "gpurun_out/${TAG}_tp_shards.jsonl"
