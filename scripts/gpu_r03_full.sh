# round 3: the whole -m gpu suite, then the bench line
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fulldepth_progress.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 420 --timeout-method thread > gpurun_out/r03_gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/r03_gputest.log; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench.log 2>&1
