"""Average rocprofv3 --pmc counters per kernel over one or more passes (csv).

    python scripts/pmc_counters.py OUT.json PREFIX DIR [DIR ...]

Every DIR holds one pass's `*_counter_collection.csv`; rows whose kernel name
starts with PREFIX (after stripping 'void ') are grouped by (name, grid size),
each counter averaged over the launches.  Derived figures use the SQ units of
MI355X_MICROARCH.md (SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_BUSY_CYCLES count
quad-cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs).
"""
import collections
import csv
import glob
import json
import os
import sys


def main(out, prefix, dirs):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = r["Kernel_Name"]
                if k.startswith("void "):
                    k = k[5:]
                if not k.startswith(prefix):
                    continue
                key = (k.split("(")[0], int(r["Grid_Size"]))
                per[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = []
    for (name, grid), cs in sorted(per.items(), key=lambda kv: -max(len(v) for v in kv[1].values())):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        row = {"kernel": name, "grid_size": grid,
               "launches": max(len(v) for v in cs.values()),
               "counters": {c: round(v, 1) for c, v in sorted(avg.items())}}
        g = avg.get("GRBM_GUI_ACTIVE")
        if g:
            cyc = g / 8.0  # per XCD
            row["gui_active_cycles_per_xcd"] = round(cyc)
            for c in ("TA_BUSY_avr", "TA_BUSY_max"):
                if c in avg:
                    row[c + "_frac"] = round(avg[c] / cyc, 3)
            # TA/TD instances: 16 per XCD... report busy per instance from the sums
            for c, n in (("TA_TA_BUSY_sum", 256), ("TD_TD_BUSY_sum", 256),
                         ("TD_TC_STALL_sum", 256), ("TA_DATA_STALLED_BY_TC_CYCLES_sum", 256),
                         ("TA_ADDR_STALLED_BY_TC_CYCLES_sum", 256),
                         ("TA_ADDR_STALLED_BY_TD_CYCLES_sum", 256),
                         ("TCP_PENDING_STALL_CYCLES_sum", 256),
                         ("TCP_TCP_TA_DATA_STALL_CYCLES_sum", 256)):
                if c in avg:
                    row[c.replace("_sum", "") + "_per_cu_frac"] = round(avg[c] / n / cyc, 3)
        if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            w = avg["SQ_WAVE_CYCLES"]
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in avg:
                    row[c + "_of_wave_cycles"] = round(avg[c] / w, 3)
        res.append(row)
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res[:4], indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
