set -o pipefail
timeout -k 10 200 python scripts/diag_stamps.py > gpurun_out/stamps.log 2>&1; echo "stamps rc=$?"
TAG=r01b bash scripts/round_gpu.sh
