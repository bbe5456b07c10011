#!/usr/bin/env python3
"""Whole-generator A/B of the persistent RRDB-trunk kernel (isr_conv_chain) against
per-conv launches, every config HIP-graph captured, interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24).  Configs "S:C:A[:V]" = streams S, chain C (0/1),
acquire A (0/1), chain kernel variant V (isr_conv_chain_variant: 0 trunk.hip, 1 round-2).  Outputs must be bit-identical.
usage: python tools/ab_chain.py --configs 2:0:0,1:0:0,1:1:0,1:1:1,2:1:0
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
    ap.add_argument("--configs", default="2:0:0,1:0:0,1:1:0,1:1:1,2:1:0")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr-size", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(args.blocks, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    lr, _ = synth_lr_batch(args.batch, args.lr_size, args.lr_size, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    runs = {}
    for c in args.configs.split(","):
        f = [int(v) for v in c.split(":")]
        s_, ch, acq = f[:3]
        engine.CHAIN_VARIANT = f[3] if len(f) > 3 else 0
        n, hw = args.batch, args.lr_size
        if s_ > 1:
            plan = engine.SplitGeneratorPlan(gw, n, hw, hw, dev, False, False, mean, std, splits=s_, chain=bool(ch))
            chains = [p.chain for p in plan.subs]
        else:
            plan = engine.GeneratorPlan(gw, n, hw, hw, dev, False, False, mean, std, chain=bool(ch),
                                        chain_acquire=bool(acq))
            chains = [plan.chain]
        out = torch.empty(plan.out_shape, device=dev)
        runs[c] = (engine.GraphedPlan(plan, x, out), out, [q for q in chains if q is not None])
    ref = None
    for c, (g, o, chains) in runs.items():
        g.run()
        torch.cuda.synchronize()
        assert not any(q.failed() for q in chains), c
        ref = o.clone() if ref is None else ref
        assert torch.equal(o, ref), f"config {c} output differs"
    t = {c: [] for c in runs}
    for _ in range(args.rounds):
        for c, (g, _, _) in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(args.steps):
                g.run()
            e1.record()
            torch.cuda.synchronize()
            t[c].append(e0.elapsed_time(e1) / args.steps)
    for c, (_, _, chains) in runs.items():
        assert not any(q.failed() for q in chains), c
    px = args.batch * (args.lr_size * 4) ** 2
    for c in runs:
        print(json.dumps({"config": c, "ms_median": round(statistics.median(t[c]), 4), "ms_min": round(min(t[c]), 4),
                          "mpix_s": round(px / statistics.median(t[c]) / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
