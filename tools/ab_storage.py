#!/usr/bin/env python3
"""A/B the activation storage type of the inference forward (bench workload: ResNet(16, 0.2, x4),
16 x 128² → 512²): bf16 (pack_generator(f16=False)) vs fp16 (the default since round 6), both
HIP-graph replays of the production plan (trunk on the persistent chain kernel), interleaved
rounds on one box; prints one JSON line per storage type.  Run under
`rocprofv3 --kernel-trace --stats` for the per-kernel split (the fp16 kernels are the `<..., true>`
instantiations).
usage: python tools/ab_storage.py [--rounds 7 --steps 10]"""
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
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--weights", default=str(Path(__file__).resolve().parents[1] / "tests" / "golden" /
                                             "trained_resnet_x4.safetensors"), help="'synth' or a state_dict file")
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.weights == "synth":
        sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
        lr, _ = synth_lr_batch(16, 128, 128, seed=1234)
        x = normalize(lr).to(dev).contiguous()
    else:  # bench.py's default workload: the trained weights on held-out tiles
        from image_super_resolution_amd import checkpoint
        from image_super_resolution_amd.weights import HELDOUT_SEED, heldout_tiles
        sd = checkpoint.load_module_state(args.weights)
        x = heldout_tiles(16, 128, 4, seed=HELDOUT_SEED)[0].to(dev).contiguous()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    runs = {}
    for name, f16 in (("bf16", False), ("fp16", True)):
        gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=f16)
        plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, mean, std, chain=True)
        assert plan.chain is not None
        out = torch.empty(plan.out_shape, device=dev)
        runs[name] = (engine.GraphedPlan(plan, x, out), out, plan)
    for g, _, _ in runs.values():
        g.run()
    torch.cuda.synchronize()
    t = {k: [] for k in runs}
    for _ in range(args.rounds):
        for k, (g, _, _) in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                g.run()
            e1.record()
            torch.cuda.synchronize()
            t[k].append(e0.elapsed_time(e1) / args.steps)
    for _, _, p in runs.values():
        p.verify()
    d = (runs["fp16"][1] - runs["bf16"][1]).abs().max().item()
    for k in runs:
        o = runs[k][1]
        print(json.dumps({"storage": k, "weights": Path(args.weights).name, "ms_median": round(statistics.median(t[k]), 4),
                          "ms_min": round(min(t[k]), 4), "rounds": len(t[k]),
                          "nonfinite_outputs": int((~torch.isfinite(o)).sum().item()),
                          "max_abs_diff_fp16_vs_bf16": round(d, 5)}), flush=True)


if __name__ == "__main__":
    main()
