#!/usr/bin/env python3
"""Whole-generator A/B of batch splitting across HIP streams (engine.SplitGeneratorPlan):
S sub-batches on S streams, later sub-batches staggered by a spin kernel, vs the
single-stream plan.  Interleaved rounds in one process; outputs must be identical.

usage: python tools/ab_split.py --configs "1,2:0,2:10,2:20,4:0" [--rounds 7]
  "S:stagger_us[:GxWy]"; "1" = the single-stream GeneratorPlan; GxWy = isr_conv3x3_fwd_variant
  ids for the growth (cout 32) and wide (cout 64/256) convs under the split plan.
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
    ap.add_argument("--configs", default="1,2:0,2:10,2:20,4:0")
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
    names = args.configs.split(",")
    plans = {}
    for c in names:
        if c == "1":
            plans[c] = engine.GeneratorPlan(gw, args.batch, args.lr_size, args.lr_size, dev, False, False, mean, std)
        else:
            parts = c.split(":")
            s, st = parts[0], parts[1]
            var = None
            if len(parts) > 2:  # conv variants "GxWy": x for the cout-32 growth convs, y for cout-64/256
                g = int(parts[2][1:parts[2].index("W")])
                w = int(parts[2][parts[2].index("W") + 1:])
                var = {("conv3x3", "*", 32): g, ("conv3x3", "*", 64): w, ("conv3x3", "*", 256): w}
            plans[c] = engine.SplitGeneratorPlan(gw, args.batch, args.lr_size, args.lr_size, dev, False, False,
                                                 mean, std, splits=int(s), stagger_us=float(st), variants=var)
    out = torch.empty(plans[names[0]].out_shape, device=dev)
    ref = None
    for c in names:
        for _ in range(2):
            plans[c].run(x, out)
        torch.cuda.synchronize()
        ref = out.clone() if ref is None else ref
        assert torch.equal(out, ref), f"config {c} output differs"
    t = {c: [] for c in names}
    for _ in range(args.rounds):
        for c in names:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                plans[c].run(x, out)
            e1.record()
            torch.cuda.synchronize()
            t[c].append(e0.elapsed_time(e1) / args.steps)
    px = args.batch * (args.lr_size * 4) ** 2
    for c in names:
        print(json.dumps({"config": c, "ms_median": round(statistics.median(t[c]), 4),
                          "ms_min": round(min(t[c]), 4), "mpix_s": round(px / statistics.median(t[c]) / 1e3, 1)}))


if __name__ == "__main__":
    main()
