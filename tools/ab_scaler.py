#!/usr/bin/env python3
"""A/B the conv3x3 kernel variant of the non-trunk convs (Scalers 64->256 with the PixelShuffle
epilogue, conv1 64->64) inside the production forward (trunk on the chain kernel), HIP-graph
replays, interleaved rounds; outputs must stay bit-identical.
usage: python tools/ab_scaler.py --variants 0,1,3,8,9"""
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
    ap.add_argument("--variants", default="0,1,3,8,9")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    lr, _ = synth_lr_batch(16, 128, 128, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    runs = {}
    for v in (int(q) for q in args.variants.split(",")):
        var = {("conv3x3", 64, 256): v} if v else None
        plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, mean, std, variants=var, chain=True)
        assert plan.chain is not None
        out = torch.empty(plan.out_shape, device=dev)
        runs[v] = (engine.GraphedPlan(plan, x, out), out)
    ref = None
    for v, (g, o) in runs.items():
        g.run()
        torch.cuda.synchronize()
        ref = o.clone() if ref is None else ref
    t = {v: [] for v in runs}
    for _ in range(args.rounds):
        for v, (g, o) in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                g.run()
            e1.record()
            torch.cuda.synchronize()
            t[v].append(e0.elapsed_time(e1) / args.steps)
    for v, (g, o) in runs.items():
        print(json.dumps({"scaler_variant": v, "ms_median": round(statistics.median(t[v]), 4),
                          "identical": bool(torch.equal(o, ref))}), flush=True)


if __name__ == "__main__":
    main()
