#!/usr/bin/env python3
"""Per-phase host-enqueue time and GPU time of one SRGAN training step
(trainer.train_srgan's body, instrumented): shows whether a phase is bound by
the host (Python / launch overhead) or by the device.

python tools/train_phases.py [--steps 4] [--warmup 3]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
import warnings
from collections import defaultdict
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import data, loss as L, models, optim, trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=16)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
    batches = data.SyntheticSR(args.batch, 512, seed=0, device=dev)
    gen = models.SRGAN(16, 0.2, True, 4).to(dev)
    dis = models.Discriminator(3, 64, 8, 1024).to(dev, memory_format=torch.channels_last)
    torch.backends.cudnn.benchmark = True
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gl = L.gen_loss(device=dev, beforeAct=True)
    og = optim.FusedAdam(gen.parameters(), lr=1e-4)
    od = optim.FusedAdam(dis.parameters(), lr=1e-4)
    ema = models.ModelEMA(gen, tau=100)
    ema.ema.to(dev)
    tf = data.GPUTransform(4, hr_norm=True, mean=mean, std=std, device=dev)
    m = torch.tensor(mean, device=dev).view(1, 3, 1, 1)
    s = torch.tensor(std, device=dev).view(1, 3, 1, 1)
    host = defaultdict(list)
    gpu = defaultdict(list)

    def step(record: bool):
        marks = []

        def mark(name):
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            marks.append((name, time.perf_counter(), e))

        mark("start")
        hr, lr = tf(next(batches))
        mark("data")
        sr = gen(lr)
        sr = ((sr + 1.0) / 2.0 - m) / s
        mark("G fwd")
        with torch.autocast("cuda", dtype=torch.bfloat16), trainer._frozen(dis):
            srd = dis(sr)
        mark("D(sr) fwd")
        perc, adv, content = gl.calc_contentLoss(sr, hr, srd)
        mark("VGG fwd x2 + losses")
        og.zero_grad(set_to_none=True)
        perc.backward()
        mark("G loss backward (D dgrad, VGG dgrad, G bwd)")
        optim.clip_grad_norm_(gen.parameters(), 10)
        og.step()
        ema.update(gen)
        mark("G clip+adam+ema")
        with torch.autocast("cuda", dtype=torch.bfloat16):
            srd = dis(sr.detach())
            hrd = dis(hr)
        advd = gl.calc_advLoss(srd, hrd)
        mark("D fwd x2")
        od.zero_grad(set_to_none=True)
        advd.backward()
        mark("D backward")
        optim.clip_grad_norm_(dis.parameters(), 10)
        od.step()
        mark("D clip+adam")
        torch.cuda.synchronize()
        if record:
            for (n0, t0, e0), (n1, t1, e1) in zip(marks, marks[1:]):
                host[n1].append((t1 - t0) * 1e3)
                gpu[n1].append(e0.elapsed_time(e1))
            host["total"].append((marks[-1][1] - marks[0][1]) * 1e3)
            gpu["total"].append(marks[0][2].elapsed_time(marks[-1][2]))

    for _ in range(args.warmup):
        step(False)
    for _ in range(args.steps):
        step(True)
    for k in host:
        print(json.dumps({"phase": k, "host_ms": round(sorted(host[k])[len(host[k]) // 2], 2),
                          "gpu_ms": round(sorted(gpu[k])[len(gpu[k]) // 2], 2)}))


if __name__ == "__main__":
    main()
