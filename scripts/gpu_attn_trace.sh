# Attention microbenchmark under a kernel trace; per-launch-group durations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/atr" -o attn -- python3 "$R/scripts/attn_bench.py" --iters 20 "$@" > "$R/gpurun_out/attn.log" 2>&1
rc=$?
cd "$R" && cat gpurun_out/attn.log | grep ctx && python3 scripts/trace_groups.py gpurun_out/atr/attn_kernel_trace.csv
exit $rc
