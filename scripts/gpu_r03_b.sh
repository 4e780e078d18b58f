# round 3: parity tests touched this round (full depth, alignment, e2e, peer incl. config E)
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fulldepth_progress.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fulldepth.py tests/test_gpu_alignment.py tests/test_gpu_e2e.py tests/test_gpu_peer.py -v -m gpu --timeout 420 --timeout-method thread > gpurun_out/r03_parity.log 2>&1
