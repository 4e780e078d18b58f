#!/bin/bash
# Weight layout A/B: k-major (default) vs tile-major (FFMI_W_TILE_MAJOR=1):
# GEMM parity tests, cold GEMM microbench at decode / verify sizes, bench.
set -o pipefail
S=scripts/gpu_step.sh
$S gemmtests 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_llama_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread && \
$S gemm_km 200 python scripts/gemm_bench.py --T 8,168 --xpacked --wstream && \
FFMI_W_TILE_MAJOR=1 $S gemm_tm 200 python scripts/gemm_bench.py --T 8,168 --xpacked --wstream && \
$S bench_km 300 python bench.py --no-cpu-baseline && \
FFMI_W_TILE_MAJOR=1 $S bench_tm 300 python bench.py --no-cpu-baseline
