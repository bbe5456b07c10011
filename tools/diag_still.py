#!/usr/bin/env python3
"""Whole-image cfg4 forward (1 x 540x960 -> 2160x3840, ResNet x4) under the production plan vs
per-conv launches (chain off) and vs tail variants: mean |diff| in LSB.  Diagnostic only."""
from __future__ import annotations

import ctypes
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import engine, models, ops, _lib  # noqa: E402

torch.manual_seed(0)
dev = "cuda"
m = models.Model(models.ResNet(16, 0.2, 4)).eval()
m.init_normalize([0.45, 0.44, 0.40], [0.22, 0.22, 0.22]) if hasattr(m, "init_normalize") else None
m = m.to(dev)
img = (torch.rand(1, 3, 540, 960) * 255).to(torch.uint8).to(dev)
outs = {}
for chain in (True, False):
    engine.CHAIN_DEFAULT = chain
    engine._PLANS.clear() if hasattr(engine, "_PLANS") else None
    with torch.no_grad():
        outs[chain] = m(img).clone()
    torch.cuda.synchronize()
d = (outs[True].float() - outs[False].float()).abs()
print("chain vs per-conv: mean", d.mean().item(), "max", d.max().item())
