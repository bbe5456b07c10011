#!/usr/bin/env python3
"""Per-kernel-shape time breakdown of one generator forward (HIP events around
every launch, summed per tag, median over rounds).

usage: python tools/breakdown.py [--batch 16] [--lr-size 128] [--rounds 5] [--u8]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from collections import defaultdict
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr-size", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--u8", action="store_true", help="uint8 in / uint8 out (Model wrapper path)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
    lr, _ = synth_lr_batch(args.batch, args.lr_size, args.lr_size, seed=1234)
    x = lr.to(dev).contiguous() if args.u8 else normalize(lr).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, args.batch, args.lr_size, args.lr_size, dev, args.u8, args.u8,
                                (0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
    out = torch.empty(plan.out_shape, dtype=plan.out_dtype, device=dev)
    for _ in range(3):
        plan.run(x, out)
    torch.cuda.synchronize()
    per = defaultdict(list)
    totals = []
    for _ in range(args.rounds):
        evs = []

        def around(tag):
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            evs.append((tag, e))
            return e

        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        plan.run(x, out, around=around)
        t1.record()
        torch.cuda.synchronize()
        totals.append(t0.elapsed_time(t1))
        acc = defaultdict(float)
        cnt = defaultdict(int)
        for tag, (a, b) in evs:
            acc[tag] += a.elapsed_time(b)
            cnt[tag] += 1
        for tag in acc:
            per[tag].append((acc[tag], cnt[tag]))
    total = statistics.median(totals)
    rows = []
    for tag, v in per.items():
        ms = statistics.median([a for a, _ in v])
        rows.append({"tag": "x".join(map(str, tag)), "launches": v[0][1], "ms": round(ms, 4),
                     "us_per_launch": round(ms * 1e3 / v[0][1], 2), "frac": round(ms / total, 4)})
    rows.sort(key=lambda r: -r["ms"])
    for r in rows:
        print(json.dumps(r))
    print(json.dumps({"total_ms": round(total, 4), "sum_ms": round(sum(r["ms"] for r in rows), 4)}))


if __name__ == "__main__":
    main()
