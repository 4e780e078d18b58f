#!/bin/bash
# MFMA-utilisation PMC pass over the bench, config-B (incr decoding) kernel
# stats, and per-rank TP=8 shards of LLaMA-7B / LLaMA-65B (configs C/D/E).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
S=scripts/gpu_step.sh
TAG=${TAG:-r01}
(export TMPDIR=/tmp FFMI_NO_GRAPHS=1; cd /tmp && \
 timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_mfma_$TAG" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/pmc_mfma.log" 2>&1 && echo "[pmc_mfma] ok" && \
 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_incr_$TAG" -o bench -- python3 "$R/bench.py" --mode incr --steps 1 --warmup 1 --no-cpu-baseline --profile 0 > "$R/gpurun_out/prof_incr.log" 2>&1 && echo "[prof_incr] ok") && \
$S tp8_7b 300 python scripts/tp_shard_bench.py --tp 8 && \
$S tp8_65b 600 python scripts/tp_shard_bench.py --tp 8 --model 65b && \
$S tp8_65b_incr 600 python scripts/tp_shard_bench.py --tp 8 --model 65b --mode incr
