#!/usr/bin/env python3
"""Denoise (utils/models.py:672-706) on libisr: inference throughput and one
`train.py --train_denoise` step (MSE, Adam, EMA) on synthetic data.

usage: python tools/bench_denoise.py [--blocks 16] [--batch 16] [--size 512] [--train-size 96]
Prints one JSON line.  FLOPs are algorithmic (2·MAC, stride-2 conv on the half grid)."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import models, optim  # noqa: E402
from image_super_resolution_amd.weights import synth_state_dict  # noqa: E402


def flops_per_px(blocks: int) -> float:
    c3 = 2 * 9 * 64 * 64
    return (2 * 243 * 64 + blocks * 2 * c3 + 2 * 9 * 64 * 256 / 4 + 2 * 2 * 2 * 9 * 256 * 256 / 4
            + c3 + 2 * 81 * 64 * 3)


def timed(fn, steps: int) -> float:
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--train-batch", type=int, default=16)
    ap.add_argument("--train-size", type=int, default=96)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda")
    m = models.Denoise(args.blocks)
    m.load_state_dict(synth_state_dict(m.state_dict(), 1))
    m = m.to(dev).eval()
    x = torch.rand(args.batch, 3, args.size, args.size, device=dev) * 2 - 1
    with torch.no_grad():
        for _ in range(3):
            m(x)
        t_inf = timed(lambda: m(x), args.steps)
    px = args.batch * args.size * args.size
    fl = flops_per_px(args.blocks) * px
    # one training step: forward, MSE, backward, clip, Adam, EMA (trainer.train body)
    m.train()
    ema = models.ModelEMA(m, tau=1000)
    opt = optim.FusedAdam(m.parameters(), lr=1e-4)
    xt = torch.rand(args.train_batch, 3, args.train_size, args.train_size, device=dev) * 2 - 1
    tt = (xt + 0.05 * torch.randn_like(xt)).clamp(-1, 1)

    def step():
        opt.zero_grad(set_to_none=True)
        F.mse_loss(m(xt), tt).backward()
        optim.clip_grad_norm_(m.parameters(), 10)
        opt.step()
        ema.update(m)

    for _ in range(3):
        step()
    t_tr = timed(step, args.steps)
    print(json.dumps({"model": f"Denoise({args.blocks})", "infer_batch": [args.batch, 3, args.size, args.size],
                      "infer_ms": round(t_inf * 1e3, 3), "infer_mpix_s": round(px / t_inf / 1e6, 1),
                      "infer_tflop_s": round(fl / t_inf / 1e12, 1), "gflop_per_batch": round(fl / 1e9, 1),
                      "train_batch": [args.train_batch, 3, args.train_size, args.train_size],
                      "train_step_ms": round(t_tr * 1e3, 3)}))


if __name__ == "__main__":
    main()
