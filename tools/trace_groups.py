#!/usr/bin/env python3
"""Group a rocprofv3 kernel trace (…_kernel_trace.csv) by (kernel template, workgroups,
LDS bytes) and print the groups by total time, per `--div` (e.g. per training step) —
the per-shape view the --stats summary (one row per symbol) does not give.
usage: python tools/trace_groups.py trace.csv --div 5 [--top 40]"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)
    name = name.replace("void ", "").replace("isr::", "")
    return name[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--div", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    g = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for r in csv.DictReader(open(args.trace)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        wg = int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1) or 1) // max(1, int(r["Workgroup_Size_X"]))
        key = (short(r["Kernel_Name"]), wg, int(r.get("LDS_Block_Size", 0) or 0))
        g[key][0] += 1
        g[key][1] += dur
        total += dur
    rows = sorted(g.items(), key=lambda kv: -kv[1][1])
    print(json.dumps({"total_us_per_div": round(total / args.div, 1), "groups": len(rows)}))
    for (k, wg, lds), (n, us) in rows[: args.top]:
        print(json.dumps({"kernel": k, "wgs": wg, "lds": lds, "calls_per_div": round(n / args.div, 2),
                          "us_per_div": round(us / args.div, 1), "avg_us": round(us / n, 1),
                          "share": round(us / total, 4)}))


if __name__ == "__main__":
    main()
