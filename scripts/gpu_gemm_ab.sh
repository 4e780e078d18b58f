set -o pipefail
S=scripts/gpu_step.sh
$S kern 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q && \
$S e2e 300 python -m pytest tests/test_gpu_e2e.py -m gpu -x -q && \
$S bench 900 python bench.py --steps 2 --warmup 1 --no-cpu-baseline && \
bash scripts/gpu_trace.sh
