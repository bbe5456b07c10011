#!/usr/bin/env python3
"""Whole-generator A/B: batch split over S HIP streams, eager vs HIP-graph replay.

S sub-batches on S streams (engine.SplitGeneratorPlan) issue S x 245 launches per
forward; a HIP graph removes the host enqueue cost so more streams can be tried.
Interleaved rounds in one process; every config's output must equal the first's.
usage: python tools/ab_graph.py --splits 1,2,4,8 [--rounds 7]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr-size", type=int, default=128)
    args = ap.parse_args()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
    lr, _ = synth_lr_batch(args.batch, args.lr_size, args.lr_size, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    runs = {}
    for s in [int(v) for v in args.splits.split(",")]:
        plan = engine.make_plan(gw, args.batch, args.lr_size, args.lr_size, dev, False, False, mean, std, streams=s)
        out = torch.empty(plan.out_shape, device=dev)
        runs[f"eager{s}"] = (lambda p=plan, o=out: p.run(x, o), out)
        gout = torch.empty(plan.out_shape, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            plan.run(x, gout)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            plan.run(x, gout)
        runs[f"graph{s}"] = (g.replay, gout)
    names = list(runs)
    ref = None
    for c in names:
        fn, o = runs[c]
        fn()
        torch.cuda.synchronize()
        ref = o.clone() if ref is None else ref
        assert torch.equal(o, ref), f"config {c} output differs"
    t = {c: [] for c in names}
    for _ in range(args.rounds):
        for c in names:
            fn, _ = runs[c]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.steps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t[c].append(e0.elapsed_time(e1) / args.steps)
    px = args.batch * (args.lr_size * 4) ** 2
    for c in names:
        print(json.dumps({"config": c, "ms_median": round(statistics.median(t[c]), 4),
                          "ms_min": round(min(t[c]), 4), "mpix_s": round(px / statistics.median(t[c]) / 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
