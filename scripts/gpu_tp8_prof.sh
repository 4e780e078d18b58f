# rocprof kernel stats of the per-rank TP = 8 shard (7B SpecInfer), graphed
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
export TMPDIR=/tmp DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/tp8prof -o tp8 -- python3 "$R/scripts/tp_shard_bench.py" --tp 8 > "$R/gpurun_out/tp8_prof.log" 2>&1 && \
cp /tmp/tp8prof/tp8_kernel_stats.csv "$R/gpurun_out/tp8_kernel_stats.csv" && \
python3 - "$R/gpurun_out/tp8_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f}ms {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:7.2f}us {r["Name"][:100]}')
PY
