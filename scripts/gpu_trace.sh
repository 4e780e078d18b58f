set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
export FFMI_NO_GRAPHS=1  # rocprofv3 tracing crashes inside HIP graph capture
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/trace" -o bench -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline --no-incr --profile 0 > "$R/gpurun_out/trace.log" 2>&1; echo "[trace] rc=$?"
