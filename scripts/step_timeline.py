"""Step timeline of a rocprofv3 --kernel-trace csv: splits the kernel stream
into model steps (a host gap > --gap us ends a step), classifies each step
(verify: M-split GEMMs at T > 64; ssm: D = 64 attention; decode: the rest)
and prints, per class, the median step's span, the sum of its kernel
durations and the idle time between kernels (launch / dependency gaps), plus
the median kernel-by-kernel breakdown of one step.

    python scripts/step_timeline.py gpurun_out/tl/bench_kernel_trace.csv [--gap 20]
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--gap", type=float, default=20.0, help="us of idle GPU that ends a step")
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N steps (warmup)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    steps, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and (s - last_end) / 1000 > a.gap and cur:
            steps.append(cur)
            cur = []
        cur.append((r["Kernel_Name"], s, e))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        steps.append(cur)
    steps = steps[a.skip:]
    cls = collections.defaultdict(list)
    for st in steps:
        names = " ".join(k[0] for k in st)
        if "gemm_mid_kernel" in names and "attention_kernel<128" in names:
            c = "verify"
        elif "attention_kernel<64" in names:
            c = "ssm"
        elif "attention_kernel<128" in names:
            c = "decode"
        else:
            c = "other"
        cls[c].append(st)
    for c, sts in sorted(cls.items()):
        spans = [(st[-1][2] - st[0][1]) / 1000 for st in sts]
        busy = [sum(e - s for _, s, e in st) / 1000 for st in sts]
        nk = [len(st) for st in sts]
        print(f"{c:7s} steps={len(sts):5d} kernels/step={statistics.median(nk):5.0f} "
              f"span={statistics.median(spans):8.1f}us busy={statistics.median(busy):8.1f}us "
              f"idle={statistics.median(spans) - statistics.median(busy):7.1f}us")
        # kernel-position breakdown over the steps with the median kernel count
        n = int(statistics.median(nk))
        same = [st for st in sts if len(st) == n]
        if not same:
            continue
        print(f"  per-kernel (median over {len(same)} steps of {n} kernels): dur / gap before")
        agg = collections.defaultdict(lambda: [0.0, 0.0, ""])
        for i in range(n):
            durs = [(st[i][2] - st[i][1]) / 1000 for st in same]
            gaps = [((st[i][1] - st[i - 1][2]) / 1000 if i else 0.0) for st in same]
            nm = same[0][i][0]
            short = nm.split("(")[0].replace("void ", "").replace("ffmi::", "")[:60]
            if n <= 40:
                print(f"    {i:3d} {statistics.median(durs):7.2f} {statistics.median(gaps):6.2f}  {short}")
            g = agg[short]
            g[0] += statistics.median(durs)
            g[1] += statistics.median(gaps)
        if n > 40:
            for k, (d, g, _) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:20]:
                print(f"    {d:8.1f} {g:7.1f}  {k}")


if __name__ == "__main__":
    main()
