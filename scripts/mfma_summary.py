"""MFMA utilisation per kernel from a rocprofv3 --pmc run of the bench
(counters SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES, csv).

  util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x kernel cycles)
  kernel cycles = GRBM_GUI_ACTIVE / 8   (rocprofv3 sums GRBM over the 8 XCDs,
                                         MI355X_MICROARCH.md, DVFS give-back)
  SIMDs = 256 CUs x 4

A cross-check is printed for the gate/up GEMM: the MFMA count the launch
issues by construction (m-tiles x n-tiles x k-steps of v_mfma_f32_16x16x32_f16,
16 busy cycles each) against the counter.

    python scripts/mfma_summary.py gpurun_out/pmc_mfma/bench_counter_collection.csv \
        > profiles/r01_pmc_mfma.json
"""
import collections
import csv
import json
import sys

SIMDS = 256 * 4


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n


def main(path):
    disp = collections.defaultdict(dict)  # dispatch -> {counter: value, "k": name}
    for r in csv.DictReader(open(path)):
        d = disp[r.get("Dispatch_Id") or r.get("Correlation_Id")]
        d["k"] = short(r["Kernel_Name"])
        d["grid"] = r.get("Grid_Size")
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for d in disp.values():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            continue
        p = per[d["k"]]
        p[0] += 1
        p[1] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
        p[2] += d["GRBM_GUI_ACTIVE"] / 8.0
        p[3] += d.get("SQ_BUSY_CYCLES", 0.0)
    rows = []
    for k, (n, busy, cyc, sqb) in per.items():
        rows.append({"kernel": k, "launches": n, "kernel_cycles_avg": round(cyc / n),
                     "mfma_busy_cycles_avg": round(busy / n),
                     "mfma_util": round(busy / (SIMDS * cyc), 4) if cyc else None})
    rows.sort(key=lambda r: -r["kernel_cycles_avg"] * r["launches"])
    total_busy = sum(p[1] for p in per.values())
    total_cyc = sum(p[2] for p in per.values())
    out = {"counters": "SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE/8 (kernel cycles), 1024 SIMDs",
           "all_kernels_mfma_util": round(total_busy / (SIMDS * total_cyc), 4) if total_cyc else None,
           "kernels": rows[:16]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
