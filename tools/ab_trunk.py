#!/usr/bin/env python3
"""Time the RRDB-trunk chain launch alone (isr_conv_chain, bench geometry) under tuning
knobs (tuning build: ISR_LIB=.../libisr_tuning.so): ablations (timing only, outputs wrong)
and the resident workgroups per CU; interleaved rounds in one process.
Configs "A:P" = ablation bits A (1 no halo DMA, 2 no MFMA, 4 no stores), per-CU cap P (0 = 2).
usage: python tools/ab_trunk.py --configs 0:0,1:0,2:0,4:0,0:1"""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, engine, models, ops  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="0:0,1:0,2:0,4:0,0:1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr-size", type=int, default=128)
    args = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    lr, _ = synth_lr_batch(args.batch, args.lr_size, args.lr_size, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, args.batch, args.lr_size, args.lr_size, dev, False, False, (0.485, 0.456, 0.406),
                                (0.229, 0.224, 0.225), chain=True)
    out = torch.empty(plan.out_shape, device=dev)
    plan.run(x, out)
    torch.cuda.synchronize()
    ch = plan.chain
    stream = ops._stream()
    cfgs = [tuple(int(v) for v in c.split(":")) for c in args.configs.split(",")]
    t = {c: [] for c in cfgs}
    for _ in range(args.rounds):
        for c in cfgs:
            _lib.check(lib.isr_tuning_trunk_knobs(c[0], c[1], 0, 0), "knobs")
            ch.fn(ctypes.byref(ch.desc), stream)  # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                ch.fn(ctypes.byref(ch.desc), stream)
            e1.record()
            torch.cuda.synchronize()
            t[c].append(e0.elapsed_time(e1) / args.reps)
            assert not ch.failed(), c
    _lib.check(lib.isr_tuning_trunk_knobs(0, 0, 0, 0), "knobs")
    for c in cfgs:
        print(json.dumps({"ablate": c[0], "per_cu": c[1], "ms_median": round(statistics.median(t[c]), 4),
                          "ms_min": round(min(t[c]), 4)}), flush=True)


if __name__ == "__main__":
    main()
