"""Kernel statistics from a rocprofv3 rocpd SQLite database (the default
output format of `rocprofv3 --kernel-trace --stats -d DIR -o NAME`).

    python scripts/rocpd_summary.py gpurun_out/prof/r01_results.db > profiles/x.csv
"""
import sqlite3
import sys


def main(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name order by sum(duration) desc"
                     ).fetchall()
    tot = sum(r[2] for r in rows)
    print('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"')
    for n, cnt, s, a, mn, mx in rows:
        print(f'"{n}",{cnt},{s},{a:.1f},{100.0 * s / tot:.4f},{mn},{mx}')


if __name__ == "__main__":
    main(sys.argv[1])
