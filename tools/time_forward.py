#!/usr/bin/env python3
"""Whole-forward time of the bench workload (trained x4 weights, 16 held-out 128² tiles, fp16
default storage, HIP-graph replays, sustained: `--steps` replays per round, `--rounds` rounds) with
whatever library ISR_LIB names; prints one JSON line with the output's checksum so alternating
processes on two libraries can be compared (tools/r06_call22.sh: the XCD-aware trunk deal).
usage: ISR_LIB=... python tools/time_forward.py [--rounds 5 --steps 20]"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from image_super_resolution_amd import checkpoint, engine  # noqa: E402
from image_super_resolution_amd.weights import HELDOUT_SEED, heldout_tiles  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    sd = checkpoint.load_module_state(ROOT / "tests" / "golden" / "trained_resnet_x4.safetensors")
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
    x = heldout_tiles(16, 128, 4, seed=HELDOUT_SEED)[0].to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
    out = torch.empty(plan.out_shape, device=dev)
    g = engine.GraphedPlan(plan, x, out)
    for _ in range(5):
        g.run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            g.run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / a.steps)
    plan.verify()
    print(json.dumps({"lib": Path(os.environ.get("ISR_LIB", "libisr.so")).name, "ms_median": round(statistics.median(ts), 4),
                      "ms_min": round(min(ts), 4), "checksum": float(out.double().sum().item())}), flush=True)


if __name__ == "__main__":
    main()
