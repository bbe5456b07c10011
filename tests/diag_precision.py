#!/usr/bin/env python3
"""Diagnostic (not collected by pytest): where the bf16 HIP generator's error comes from.

Emulates the HIP inference numerics of ResNet/EResNet (engine.py's launch list) on the CPU on top
of the fp32 oracle's graph: every stored activation rounded to bf16 (head output, dense-buffer
channels, RDB / RRDB outputs, conv1 + trunk residual, scaler outputs), every conv's BN-folded
weights rounded to bf16, the head's normalised input rounded to bf16, fp32 accumulation and fp32
bias, the RDB final conv's epilogue ((acc*s1 + x)*s2 + r2) in fp32 with ONE rounding, the tail in
fp32 with tanh.  Switches turn single rounding sites off to attribute the error:

    python tests/diag_precision.py --weights tests/golden/trained_resnet_x4.safetensors
    python tests/diag_precision.py --synth 5          # the synthetic weights of the older tests
    python tests/diag_precision.py --weights tests/golden/trained_resnet_x2.safetensors --scale 2 \
        --hip gpurun_out/r06/trained_heldout_hip_y_x2.pt

Reports PSNR(emulation vs fp32 oracle), |dPSNR vs HR| per configuration, and optionally the same
for a saved HIP output (--hip gpurun_out/.../trained_heldout_hip_y.pt) to check the emulation.
"""
from __future__ import annotations

import argparse
import math
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle import ref_cpu as R  # noqa: E402


def bf(t):
    return t.to(torch.bfloat16).float()


def hf(t):
    return t.to(torch.float16).float()


# storage emulations (--storage): the rounding applied at the weight sites and at every other site
STORAGE = {"bf16": (bf, bf), "fp16": (hf, hf),
           # fp16 containers holding bf16-precision weights (weights' low 3 mantissa bits zero:
           # fewer toggling multiplier bits, the DVFS lever of MI355X_MICROARCH.md) and fp16 activations
           "wbf16": (lambda t: hf(bf(t)), hf),
           # the converse: fp16 weights, activations at bf16 precision
           "abf16": (hf, lambda t: hf(bf(t)))}


class Emu:
    """Rounding sites: inp (head input), w (weights), act (growth-conv / head / scaler outputs),
    res (RDB / RRDB outputs: the 64-ch residual stream), trunk (conv1 + feat)."""

    def __init__(self, sd, sites=("inp", "w", "act", "res", "trunk"), enchant=False, add_rate=0.2,
                 storage="bf16"):
        self.sd = R.fuse_state_dict(sd) if any(k.endswith(".bn.weight") for k in sd) else sd
        self.s = set(sites)
        self.enchant, self.ar = enchant, add_rate
        self.rw, self.ra = STORAGE[storage]

    def r(self, site, t):
        if site not in self.s:
            return t
        return self.rw(t) if site == "w" else self.ra(t)

    def conv(self, prefix, x, pad=None):
        w = self.sd[f"{prefix}.conv.weight"]
        b = self.sd.get(f"{prefix}.conv.bias")
        w = self.r("w", w)
        return F.conv2d(x.double(), w.double(), None if b is None else b.double(),
                        padding=w.shape[-1] // 2 if pad is None else pad).float()

    def rdb(self, p, x, r2=None):
        cat = x
        for k in range(4):
            o = F.leaky_relu(self.conv(f"{p}.conv{k}", cat), 0.01)
            cat = torch.cat([cat, self.r("act", o)], 1)
        v = self.conv(f"{p}.conv", cat) * self.ar + x
        if r2 is not None:
            v = v * self.ar + r2
        return self.r("res", v)

    def forward(self, x, num_blocks, scale):
        x = self.r("inp", x)
        feat = self.r("act", F.leaky_relu(self.conv("conv0", x), 0.01 if self.enchant else 0.2))
        y = feat
        for i in range(num_blocks):
            x0 = y
            y = self.rdb(f"residual.{i}.net.0", y)
            y = self.rdb(f"residual.{i}.net.1", y)
            y = self.rdb(f"residual.{i}.net.2", y, r2=x0)
        y = self.r("trunk", feat + self.conv("conv1", y))
        for s in range(scale // 2):
            y = self.r("act", F.leaky_relu(F.pixel_shuffle(self.conv(f"scaler.{s}.net.0", y), 2), 0.01))
        return torch.tanh(self.conv("conv2", y))


def psnr(a, b, peak=2.0):
    m = torch.mean((a.double() - b.double()) ** 2).item()
    return float("inf") if m == 0 else 10 * math.log10(peak * peak / m)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--weights", default=None)
    ap.add_argument("--synth", type=int, default=None)
    ap.add_argument("--tiles", type=int, default=2)
    ap.add_argument("--lr-size", type=int, default=128)
    ap.add_argument("--hip", default=None, help="saved HIP output of the first tiles (train_weights.py)")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--scale", type=int, default=4, choices=(2, 4))
    ap.add_argument("--storage", default="bf16", help="comma list of " + "/".join(STORAGE))
    ap.add_argument("--all-sites-only", action="store_true", help="only the all-sites configuration")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    torch.set_grad_enabled(False)
    from image_super_resolution_amd import checkpoint, models
    from image_super_resolution_amd.weights import heldout_tiles, normalize, synth_lr_batch, synth_state_dict
    if a.weights:
        sd = checkpoint.load_module_state(a.weights)
        lr, hr = heldout_tiles(a.tiles, a.lr_size, a.scale)
    else:
        sd = {k: v.float() for k, v in synth_state_dict(models.ResNet(16, 0.2, scaleRate=a.scale).state_dict(),
                                                            a.synth or 0).items()}
        lr01, hr = synth_lr_batch(a.tiles, a.lr_size, a.lr_size, seed=1234, scale=a.scale)
        lr = normalize(lr01)
    nb = R.count_blocks(sd)
    hr1 = hr * 2 - 1
    ref = R.generator(sd, lr, num_blocks=nb, scale=a.scale)
    p_ref = psnr(ref, hr1)
    print(f"oracle fp32: PSNR vs HR {p_ref:.3f} dB (MSE {4 / 10 ** (p_ref / 10):.3e})")
    if a.hip:
        y = torch.load(a.hip, weights_only=True)["y"][: a.tiles]
        print(f"HIP (saved): vs oracle {psnr(y, ref[: len(y)]):.2f} dB, dPSNR "
              f"{abs(psnr(y, hr1[: len(y)]) - psnr(ref[: len(y)], hr1[: len(y)])):.5f} dB")
    full = ("inp", "w", "act", "res", "trunk")
    cfgs = [("all sites", full)] + [(f"all but {s}", tuple(x for x in full if x != s)) for s in full] + \
           [(f"only {s}", (s,)) for s in full]
    if a.all_sites_only:
        cfgs = cfgs[:1]
    for storage in a.storage.split(","):
        for name, sites in cfgs:
            e = Emu(sd, sites, storage=storage).forward(lr, nb, a.scale)
            print(f"[{storage}] {name:16s}: vs oracle {psnr(e, ref):7.2f} dB   dPSNR vs HR "
                  f"{abs(psnr(e, hr1) - p_ref):.5f} dB", flush=True)


if __name__ == "__main__":
    main()
