#!/bin/bash
# Round 6: split-row top-k workgroups per row forced (FFMI_TOPK_SPLIT=G) at
# the SSM's T = 8 / 24 shapes, standalone (scripts/topk_bench.py), twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/r06_topk_g.log
: > $OUT
for rep in 1 2; do
  for g in 4 8 16; do
    echo "G=$g" >> $OUT
    FFMI_TOPK_SPLIT=$g timeout -k 10 120 python scripts/topk_bench.py 2>&1 | grep -E "T=(8|24) V=32000 " >> $OUT || { tail -5 $OUT; exit 1; }
  done
done
cat $OUT
