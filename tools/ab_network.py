#!/usr/bin/env python3
"""Whole-generator A/B of conv3x3 variant choices, interleaved rounds in one
process on one device (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/ab_network.py --configs "G0W0,G1W1,G0W1" [--rounds 7]
  Gx = variant for the cout-32 growth convs, Wy = variant for cout-64/256 convs.
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


def parse_cfg(s: str) -> dict:
    g = int(s[s.index("G") + 1:s.index("W")])
    w = int(s[s.index("W") + 1:])
    return {("conv3x3", "*", 32): g, ("conv3x3", "*", 64): w, ("conv3x3", "*", 256): w}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="G0W0,G1W1")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr-size", type=int, default=128)
    args = ap.parse_args()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    lr, _ = synth_lr_batch(args.batch, args.lr_size, args.lr_size, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    names = args.configs.split(",")
    plans = {c: engine.GeneratorPlan(gw, args.batch, args.lr_size, args.lr_size, dev, False, False,
                                     (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), variants=parse_cfg(c))
             for c in names}
    out = torch.empty(plans[names[0]].out_shape, device=dev)
    ref = None
    for c in names:  # warm-up + cross-check outputs (variants must agree bit-for-bit)
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
    for c in names:
        px = args.batch * (args.lr_size * 4) ** 2
        print(json.dumps({"config": c, "ms_median": round(statistics.median(t[c]), 4),
                          "ms_min": round(min(t[c]), 4), "mpix_s": round(px / statistics.median(t[c]) / 1e3, 1)}))


if __name__ == "__main__":
    main()
