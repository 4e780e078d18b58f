"""Idle GPU time inside and between chained SSM beam steps, from a rocprofv3
--kernel-trace csv: an SSM step ends with its softmax top-k (T = 24 rows);
for every step that follows another without a host gap (> --gap us), the gap
from that top-k's end to the next kernel's start is the inter-graph boundary,
compared with the median boundary between kernels inside the steps.

    python scripts/ssm_gaps.py gpurun_out/tl/bench_kernel_trace.csv
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gap", type=float, default=20.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, r["Kernel_Name"])
          for r in rows]
    inter, intra, spans, kern = [], [], [], []
    i = 0
    while i < len(ks):
        # an SSM step: the kernels up to and including a top-k, after a
        # D = 64 attention (the 68M SSM's heads)
        j = i
        while j < len(ks) and "softmax_topk" not in ks[j][2]:
            j += 1
        if j >= len(ks):
            break
        step = ks[i:j + 1]
        if any("attention_kernel<64" in k[2] for k in step) and len(step) <= 20:
            gaps = [step[q + 1][0] - step[q][1] for q in range(len(step) - 1)]
            if all(g < a.gap for g in gaps):
                intra.extend(gaps)
                spans.append(step[-1][1] - step[0][0])
                kern.append(sum(k[1] - k[0] for k in step))
                if j + 1 < len(ks):
                    g = ks[j + 1][0] - ks[j][1]
                    if g < a.gap:
                        inter.append(g)
        i = j + 1
    if not spans:
        print("no SSM steps found")
        return
    print(f"SSM steps: {len(spans)}; span median {statistics.median(spans):.2f} us, kernel sum "
          f"median {statistics.median(kern):.2f} us")
    print(f"boundary inside a step: median {statistics.median(intra):.2f} us "
          f"(n {len(intra)})")
    if inter:
        print(f"top-k end -> next step's first kernel (no host gap): median "
              f"{statistics.median(inter):.2f} us, mean {statistics.mean(inter):.2f} (n {len(inter)})")


if __name__ == "__main__":
    main()
