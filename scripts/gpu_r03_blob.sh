# blob fetch (first kernel reads the step's staging blob from mapped host
# memory): e2e + model tests, same-box bench A/B, per-rank TP shard table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_tp_local.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/blob_test.log 2>&1 || { echo tests failed; tail -20 gpurun_out/blob_test.log; exit 1; }
tail -2 gpurun_out/blob_test.log
BENCH_ARGS="--no-incr" timeout -k 10 900 bash scripts/gpu_env_bench_ab.sh FFMI_BLOB_FETCH=1 FFMI_BLOB_FETCH=0 FFMI_BLOB_FETCH=1 FFMI_BLOB_FETCH=0 > gpurun_out/blob_ab.log 2>&1 || { tail -20 gpurun_out/blob_ab.log; exit 1; }
cat gpurun_out/blob_ab.log | cut -c1-300
TAG=r03 bash scripts/gpu_refresh_aux.sh
