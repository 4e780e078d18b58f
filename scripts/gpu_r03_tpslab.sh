# split-K slabs folded into the xGMI all-reduce's copy-in; 1-rank shards defer
# to the norm: TP tests, per-rank shard table, boundary diagnostic
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_tp_local.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tpslab_test.log 2>&1 || { echo TP tests failed; tail -30 gpurun_out/tpslab_test.log; exit 1; }
tail -2 gpurun_out/tpslab_test.log
TAG=r03 bash scripts/gpu_refresh_aux.sh || exit 1
timeout -k 10 300 python -u scripts/diag_boundaries.py > gpurun_out/boundaries.log 2>&1; tail -12 gpurun_out/boundaries.log
