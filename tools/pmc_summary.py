#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc CSVs (tools/profile_pmc.sh) per (kernel, grid).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reads 1/2 of the bytes of wide (16 B/lane) coalesced
streaming reads — the glds / dwordx4 loads these kernels use — so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.
usage: tools/pmc_summary.py <outdir> [--json out.json] [--match substr]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import statistics
from collections import defaultdict
from pathlib import Path


def load(outdir: Path):
    data = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [values per dispatch]
    for f in glob.glob(str(outdir / "pass*" / "**" / "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "?")
            grid = r.get("Grid_Size", "?")
            key = (name, grid)
            disp = r.get("Dispatch_Id", "0")
            data[key][(r["Counter_Name"], disp)].append(float(r["Counter_Value"]))
    out = {}
    for key, cv in data.items():
        per = defaultdict(list)
        for (cname, disp), vals in cv.items():
            per[cname].append(sum(vals))  # sum over dimensions (XCD / SE instances) of one dispatch
        out[key] = {c: statistics.mean(v) for c, v in per.items()}
        out[key]["dispatches"] = max(len(v) for v in per.values())
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--json")
    ap.add_argument("--match", default="")
    args = ap.parse_args()
    res = load(Path(args.outdir))
    rows = []
    for (name, grid), c in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        if args.match and args.match not in name:
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        row = {"kernel": name[:90], "grid": grid, "dispatches": c["dispatches"],
               "wait_any": round(c.get("SQ_WAIT_ANY", 0) / wc, 3),
               "wait_inst": round(c.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
               "active_inst": round(c.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
               "mfma_busy_per_cu_cycle": None,
               "lds_bank_conflict_frac": round(c.get("SQ_LDS_BANK_CONFLICT", 0) / (c.get("SQ_LDS_IDX_ACTIVE", 0) or 1), 3),
               "lds_unaligned": c.get("SQ_LDS_UNALIGNED_STALL", 0),
               "hbm_read_bytes": 2 * c.get("FETCH_SIZE", 0) * 1024,
               "hbm_write_bytes": c.get("WRITE_SIZE", 0) * 1024,
               "l2_hit": round(c.get("TCC_HIT", 0) / ((c.get("TCC_HIT", 0) + c.get("TCC_MISS", 0)) or 1), 3),
               "gui_active": c.get("GRBM_GUI_ACTIVE", 0)}
        if c.get("GRBM_GUI_ACTIVE"):
            # SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; 1024 SIMDs on the chip
            row["mfma_busy_per_cu_cycle"] = round(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 3)
        row["hbm_bytes"] = row["hbm_read_bytes"] + row["hbm_write_bytes"]
        rows.append(row)
        print(json.dumps(row))
    if args.json:
        Path(args.json).write_text(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
