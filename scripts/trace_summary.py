"""Per-(kernel, grid) duration summary of a rocprofv3 --kernel-trace csv.

    python scripts/trace_summary.py gpurun_out/trace/bench_kernel_trace.csv [N]
"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
d = collections.defaultdict(list)
for r in rows:
    k = (r["Kernel_Name"][:72], r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"])
    d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(v) / 1000:8.2f} ms n={len(v):6d} avg={sum(v) / len(v):7.2f} us  {k}")
