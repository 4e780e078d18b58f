# wave-parallel wide GEMM: kernel tests, SSM lm_head timing, same-box bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/wave_test.log 2>&1 || { echo kernel tests failed; tail -20 gpurun_out/wave_test.log; exit 1; }
for v in 1 0; do FFMI_WAVE_GEMM=$v timeout -k 10 120 python -u scripts/gemm_bench.py --shapes ssm --T 8,24 --ops lm_head --cold-mb 0 >> gpurun_out/wave_lm.log 2>&1 || exit 1; done
BENCH_ARGS="--no-incr" timeout -k 10 900 bash scripts/gpu_env_bench_ab.sh FFMI_WAVE_GEMM=1 FFMI_WAVE_GEMM=0 FFMI_WAVE_GEMM=1 FFMI_WAVE_GEMM=0 > gpurun_out/wave_ab.log 2>&1
