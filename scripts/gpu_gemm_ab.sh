set -o pipefail
S=scripts/gpu_step.sh
$S kern 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attention" && \
$S e2e 300 python -m pytest tests/test_gpu_e2e.py -m gpu -x -q && \
bash scripts/gpu_trace.sh
