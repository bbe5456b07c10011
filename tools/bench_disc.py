#!/usr/bin/env python3
"""Discriminator train-mode forward + backward (SRGAN cfg3 shape, [16,3,512,512]):
libisr conv stack vs the stock modules (NHWC, MIOpen find mode, bf16 autocast)."""
import copy
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import models  # noqa: E402

dev = torch.device("cuda")
torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
hip = models.Discriminator(3, 64, 8, 1024).to(dev).train().use_libisr(True)
stock = copy.deepcopy(hip).to(memory_format=torch.channels_last).use_libisr(False)
x = torch.randn(16, 3, 512, 512, device=dev)


def step(m, need_dx):
    xr = x.clone().requires_grad_(need_dx)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        o = m(xr)
    o.float().sum().backward()


impls = (("libisr", hip), ("miopen_nhwc_amp", stock))
if len(sys.argv) > 1:
    impls = [i for i in impls if i[0] == sys.argv[1]]
for name, m in impls:
    for need_dx in (False, True):
        for _ in range(3):
            step(m, need_dx)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            step(m, need_dx)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        print(json.dumps({"impl": name, "input_grad": need_dx, "fwd_bwd_ms": round(statistics.median(ts), 2)}))
