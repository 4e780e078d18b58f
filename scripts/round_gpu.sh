#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats (csv), PMC fetch,
# PMC MFMA utilisation (each counter pass in its own run).  Raw rocprofv3
# output stays in /tmp on the box (tens of MB); the summaries land in
# gpurun_out/ (gpurun copies back at most 64 MiB).
# rocprofv3 runs with FFMI_NO_GRAPHS=1: its tracing crashed inside HIP graph
# capture on this image (the LLM verify steps profiled here are never graphed).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
S=scripts/gpu_step.sh
TAG=${TAG:-r01}
P=/tmp/ffmi_prof_$TAG
B="$R/bench.py --steps 1 --no-cpu-baseline --no-incr --profile 0"
$S kernels 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_tp_local.py -m gpu -q && \
$S e2e 600 python -m pytest tests/test_gpu_e2e.py tests/test_gpu_checkpoint.py -m gpu -q && \
$S bench 900 python bench.py && \
(export TMPDIR=/tmp FFMI_NO_GRAPHS=1; cd /tmp && \
 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/prof" -o bench -- python3 $B --warmup 1 > "$R/gpurun_out/prof.log" 2>&1 && \
 cp "$P/prof/bench_kernel_stats.csv" "$R/gpurun_out/${TAG}_bench_kernel_stats.csv" && echo "[prof] ok" && \
 timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/pmc" -o bench -- python3 $B --warmup 0 > "$R/gpurun_out/pmc.log" 2>&1 && \
 python3 "$R/scripts/pmc_summary.py" "$P/pmc/bench_counter_collection.csv" > "$R/gpurun_out/${TAG}_pmc_fetch.json" && echo "[pmc] ok" && \
 timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$P/mfma" -o bench -- python3 $B --warmup 0 > "$R/gpurun_out/pmc_mfma.log" 2>&1 && \
 python3 "$R/scripts/mfma_summary.py" "$P/mfma/bench_counter_collection.csv" > "$R/gpurun_out/${TAG}_pmc_mfma.json" && echo "[pmc_mfma] ok")
