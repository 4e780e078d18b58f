#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel stats (csv), PMC fetch,
# PMC MFMA utilisation (each counter pass in its own run).
# rocprofv3 runs with FFMI_NO_GRAPHS=1: its tracing crashed inside HIP graph
# capture on this image (the LLM verify steps profiled here are never graphed).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
S=scripts/gpu_step.sh
TAG=${TAG:-r01}
$S kernels 600 python -m pytest tests/test_gpu_kernels.py -m gpu -q && \
$S e2e 600 python -m pytest tests/test_gpu_e2e.py -m gpu -q && \
$S bench 900 python bench.py && \
(export TMPDIR=/tmp FFMI_NO_GRAPHS=1; cd /tmp && \
 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$TAG" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/prof.log" 2>&1 && echo "[prof] ok" && \
 timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_$TAG" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/pmc.log" 2>&1 && echo "[pmc] ok" && \
 timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/gpurun_out/pmc_mfma_$TAG" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/pmc_mfma.log" 2>&1 && echo "[pmc_mfma] ok")
