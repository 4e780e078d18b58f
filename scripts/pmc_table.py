"""Per-kernel PMC table of the verify step from a rocprofv3 --pmc csv:
average counter value per launch for each (kernel, grid) with >= --min-launches
launches, labelled with the verify-step op it belongs to at T = 168.  FETCH_SIZE
is reported x 2 x 1024 bytes (gfx950: half the bytes of 16-B streaming reads,
MI355X_MICROARCH.md § HBM), WRITE_SIZE x 1024 (exact for 16-B stores).

    python scripts/pmc_table.py <counter_collection.csv> > profiles/rNN_pmc_<counter>.json
"""
import collections
import csv
import json
import sys

# verify-step kernels of the LLaMA-7B bench (T = 168), by template prefix
LABELS = [
    ("gemm_mid_kernel<3, 6, 4, 1,", "gate_up_silu"),
    ("gemm_mid_kernel<3, 6, 4, 0,", "qkv"),
    ("gemm_mid_kernel<3, 8, 4, 0,", "down (and lm_head)"),
    ("gemm_mid_kernel<3, 4, 4, 0,", "o_proj"),
    ("attention_kernel<128, 2, 8, true", "verify attention (fused KV update)"),
    ("rmsnorm_kernel<512, 1, 8, 2>", "residual norm after down (8 slabs)"),
    ("rmsnorm_kernel<512, 1, 4, 2>", "residual norm after o_proj (4 slabs)"),
    ("softmax_topk_reg_kernel", "softmax top-k / argmax"),
]
SCALE = {"FETCH_SIZE": 2 * 1024, "WRITE_SIZE": 1024}


def main(path, min_launches=64):
    per = collections.defaultdict(list)
    counters = set()
    for r in csv.DictReader(open(path)):
        c = r["Counter_Name"]
        counters.add(c)
        name = r["Kernel_Name"].split("(")[0].replace("void ffmi::", "")
        per[(c, name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    out = []
    for (c, name, grid), vals in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        if len(vals) < min_launches:
            continue
        label = next((lb for p, lb in LABELS if name.startswith(p)), None)
        out.append({"counter": c, "kernel": name, "op": label, "grid_size": grid,
                    "launches": len(vals),
                    "bytes_per_launch": round(sum(vals) / len(vals) * SCALE.get(c, 1))})
    json.dump({"counters": sorted(counters), "correction": {k: f"x {v}" for k, v in SCALE.items()},
               "kernels": out}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
