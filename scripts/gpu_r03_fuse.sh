# residual norms folded into the skinny GEMMs: full GPU suite, then bench A/B
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/fulldepth_progress.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 420 --timeout-method thread > gpurun_out/fuse_test.log 2>&1 || { echo tests failed; tail -40 gpurun_out/fuse_test.log; exit 1; }
tail -2 gpurun_out/fuse_test.log
timeout -k 10 900 bash scripts/gpu_env_bench_ab.sh FFMI_FUSE_NORM=1 FFMI_FUSE_NORM=0 FFMI_FUSE_NORM=1 FFMI_FUSE_NORM=0 > gpurun_out/fuse_ab.log 2>&1 || { tail -20 gpurun_out/fuse_ab.log; exit 1; }
cut -c1-170 gpurun_out/fuse_ab.log
