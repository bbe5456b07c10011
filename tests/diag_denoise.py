#!/usr/bin/env python3
"""Per-parameter gradient error of the libisr Denoise backward vs fp32 autograd
through the oracle (diagnostic for tests/test_gpu_denoise.py; lives under tests/
because only tests may import oracle/).  usage: python tests/diag_denoise.py"""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import models  # noqa: E402
from image_super_resolution_amd.weights import synth_state_dict  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402

for blocks, n, h, w in [(0, 3, 32, 32), (2, 2, 32, 48)]:
    m = models.Denoise(blocks)
    m.load_state_dict(synth_state_dict(m.state_dict(), 70 + blocks))
    gen = torch.Generator().manual_seed(5 + h)
    x = torch.rand(n, 3, h, w, generator=gen) * 2 - 1
    target = (x + 0.1 * torch.randn(n, 3, h, w, generator=gen)).clamp(-1, 1)
    sd = {k: v.detach().clone().float() for k, v in m.state_dict().items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items() if v.is_floating_point() and "running" not in k}
    y_ref = R.denoise(sd, x, train_bn=True)
    F.mse_loss(y_ref, target).backward()
    m = m.to("cuda").train()
    y = m(x.to("cuda"))
    print("blocks", blocks, "fwd psnr", round(R.psnr(y.detach().cpu(), y_ref.detach()), 2))
    F.mse_loss(y, target.to("cuda")).backward()
    # yardstick: the same oracle graph on the GPU under torch's bf16 autocast (MIOpen)
    sd_b = {k: v.detach().clone().float().cuda() for k, v in m.state_dict().items()}
    sd0 = synth_state_dict(models.Denoise(blocks).state_dict(), 70 + blocks)
    for k in sd_b:
        if "running" in k:
            sd_b[k] = sd0[k].float().cuda()
    par_b = {k: v.requires_grad_(True) for k, v in sd_b.items() if v.is_floating_point() and "running" not in k}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y_b = R.denoise(sd_b, x.cuda(), train_bn=True)
    F.mse_loss(y_b.float(), target.cuda()).backward()
    for name, p in m.named_parameters():
        r = params[name].grad.to("cuda")
        rel = ((p.grad - r).norm() / r.norm().clamp_min(1e-12)).item()
        cos = F.cosine_similarity(p.grad.flatten(), r.flatten(), dim=0).item()
        rb = ((par_b[name].grad - r).norm() / r.norm().clamp_min(1e-12)).item()
        print(f"  {name:40s} rel {rel:.3e} cos {cos:.5f}   torch-bf16-autocast rel {rb:.3e}")
