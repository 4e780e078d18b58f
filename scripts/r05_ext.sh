#!/bin/bash
# Round-5 session: the SpecInfer extensions (tree width 4, 4 SSMs) on the GPU.
#   STAGE=tests: token chain + full precision spec tests + TP2 queue test, then the bench-
#   workload spec tests; STAGE=65b: the 80-layer TP test (ssm4 case); STAGE=bench: bench.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
rm -f gpurun_out/*_progress.log
S=scripts/gpu_step.sh
PT="python -u -m pytest -v --timeout-method thread"
case "${STAGE:-tests}" in
tests)
  $S ext_chain 600 $PT --timeout 580 tests/test_gpu_token_chain.py || exit 1
  $S ext_fp32 600 $PT --timeout 580 tests/test_gpu_full_precision.py -k "spec_equals_incr or negative_control" || exit 1
  $S ext_tp2 300 $PT --timeout 280 tests/test_gpu_peer.py -k "tp2_spec" || exit 1
  $S ext_bw 900 $PT --timeout 880 tests/test_gpu_bench_workload.py -k "spec_infer" || exit 1
  ;;
65b)
  $S ext_65b 1000 $PT --timeout 980 tests/test_gpu_llama65b_tp.py -k "ssm4" || exit 1
  ;;
bench)
  $S ext_bench 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  ;;
neg)
  $S ext_neg 600 $PT --timeout 580 tests/test_gpu_bench_workload.py -k "negative" || exit 1
  ;;
65all)
  $S ext_65all 1000 $PT --timeout 980 tests/test_gpu_llama65b_tp.py || exit 1
  ;;
tile)
  $S ext_tile 600 $PT --timeout 580 tests/test_gpu_llama_shapes.py -k "tile or 577 or 1024" || exit 1
  bash scripts/gpu_kernel_ab.sh "scripts/gemm_bench.py --shapes llama7b --T 577,1024 --xpacked --wstream --iters 20" "" "FFMI_TILE_GEMM=0" "" || exit 1
  ;;
gemm)
  $S ext_gemm 600 $PT --timeout 580 tests/test_gpu_llama_shapes.py tests/test_gpu_kernels.py -k "gemm or linear or shapes" || exit 1
  ;;
esac
