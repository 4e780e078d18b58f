"""Launch groups of a rocprofv3 kernel trace, split at each runtime copy/fill
kernel (one group per uploaded batch): avg / min us per kernel name."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
groups = [collections.OrderedDict()]
for r in rows:
    n = r["Kernel_Name"][:48]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    if n.startswith("__amd_rocclr"):
        if any(groups[-1].values()):
            groups.append(collections.OrderedDict())
        continue
    groups[-1].setdefault(n, []).append(d)
for i, g in enumerate(groups):
    for n, v in g.items():
        print(f"group {i}: {n:50s} n={len(v):3d} avg={sum(v) / len(v):7.2f} min={min(v):7.2f}")
