#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 SQLite results DB (rocpd schema).

python tools/prof_db_summary.py gpurun_out/prof/run_results.db [--top 30] [--csv out.csv]
"""
import argparse
import collections
import csv
import re
import sqlite3


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name)
    return n[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--csv", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    q = ("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    agg = collections.defaultdict(lambda: [0, 0.0])
    for name, ns in con.execute(q):
        e = agg[short(name)]
        e[0] += 1
        e[1] += ns
    total = sum(v[1] for v in agg.values())
    rows = sorted(((k, c, t) for k, (c, t) in agg.items()), key=lambda r: -r[2])
    print(f"total kernel time {total / 1e6:.2f} ms over {sum(v[0] for v in agg.values())} dispatches")
    for k, c, t in rows[:a.top]:
        print(f"{t / 1e6:9.3f} ms {100 * t / total:5.1f}% {c:6d}x {t / c / 1e3:9.2f} us  {k}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for k, c, t in rows:
                w.writerow([k, c, int(t), t / c, 100 * t / total])


if __name__ == "__main__":
    main()
