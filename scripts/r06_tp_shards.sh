#!/bin/bash
# Round 6 per-rank TP table (scripts/tp_shard_bench.py): 7B SpecInfer at TP
# 1/2/4/8, 65B TP 8, incr decoding TP 8, and config E's four SSMs replicated
# on the rank vs its one-SSM share when distributed.  One JSON line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/r06_tp_shards.jsonl
: > $OUT
run() { timeout -k 10 300 python scripts/tp_shard_bench.py --steps 2 "$@" 2> gpurun_out/tp_shard.err | grep '^{' >> $OUT || { echo "failed: $*"; tail -5 gpurun_out/tp_shard.err; exit 1; }; }
for tp in 1 2 4 8; do run --tp $tp; done
run --tp 8 --model 65b
run --tp 8 --mode incr
run --tp 8 --ssms 4
run --tp 1 --ssms 4
cat $OUT | cut -c1-220
