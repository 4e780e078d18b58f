set -o pipefail
S=scripts/gpu_step.sh
$S kern_sk4 300 env FFMI_GEMM_IMPL=skinny4 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "linear" && \
$S gb_reg 300 python scripts/gemm_bench.py --T 100,168,256 && \
$S gb_sk4 300 env FFMI_GEMM_IMPL=skinny4 python scripts/gemm_bench.py --T 100,168,256 && \
$S gb_sk8 300 env FFMI_GEMM_IMPL=skinny8 python scripts/gemm_bench.py --T 100,168,256 && \
$S gb_sk2 300 env FFMI_GEMM_IMPL=skinny2 python scripts/gemm_bench.py --T 64,100,168
