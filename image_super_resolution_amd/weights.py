"""Deterministic synthetic weights and inputs.

There are no trained SR weights anywhere (the shipped
model.pt is a denoiser) and no network, so every parity fixture, test and the
benchmark use weights produced here.  Each tensor is drawn from numpy's PCG64
seeded by (seed, crc32 of its state_dict key), so the values depend only on
the key, the shape and the seed — not on module construction order or torch's
RNG — and the golden-vector script can install exactly the same weights into
the reference modules.
"""
from __future__ import annotations

import zlib

import numpy as np
import torch


def _rng(seed: int, key: str) -> np.random.Generator:
    return np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(key.encode())]))


def synth_tensor(key: str, shape: tuple[int, ...], seed: int = 0) -> np.ndarray:
    """fp32 array for state_dict entry `key` of `shape`."""
    g = _rng(seed, key)
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    parent = key.rsplit(".", 2)[-2] if key.count(".") >= 1 else ""
    is_bn = parent in ("bn", "store_bn")
    if is_bn:
        if leaf == "weight":
            return g.uniform(0.8, 1.2, shape).astype(np.float32)
        if leaf == "bias":
            return g.uniform(-0.1, 0.1, shape).astype(np.float32)
        if leaf == "running_mean":
            return g.uniform(-0.1, 0.1, shape).astype(np.float32)
        if leaf == "running_var":
            return g.uniform(0.5, 1.5, shape).astype(np.float32)
    if leaf == "weight" and len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        # unit-variance pre-activations; He gain for the ReLU VGG stack so that
        # conv5_4 features do not vanish
        gain = 2.0 if "vgg" in key else 1.0
        bound = np.sqrt(3.0 * gain / fan_in)
        return g.uniform(-bound, bound, shape).astype(np.float32)
    if leaf == "bias":
        return g.uniform(-0.05, 0.05, shape).astype(np.float32)
    return g.uniform(-0.1, 0.1, shape).astype(np.float32)


def synth_state_dict(template: dict[str, torch.Tensor], seed: int = 0) -> dict[str, torch.Tensor]:
    """Replace every entry of a state_dict template with deterministic values."""
    out = {}
    for k, v in template.items():
        a = synth_tensor(k, tuple(v.shape), seed)
        out[k] = torch.from_numpy(a).to(v.dtype) if v.is_floating_point() or v.dtype == torch.int64 else v.clone()
    return out


def synth_lr_batch(n: int, h: int, w: int, seed: int = 1234, scale: int = 4) -> tuple[torch.Tensor, torch.Tensor]:
    """Smooth 'natural-ish' HR images and their LR counterparts.

    HR [n,3,h*scale,w*scale] in [0,1]: bicubic upsampling of U[0,1] noise at
    1/16 resolution; LR = antialiased bilinear x(1/scale) downsample of HR.
    Returns (lr_unnormalised in [0,1], hr in [0,1]), both fp32 CPU.
    """
    import torch.nn.functional as F

    hs, ws = h * scale, w * scale
    hrs = []
    for i in range(n):
        g = torch.Generator().manual_seed(seed + i)
        base = torch.rand(1, 3, max(2, hs // 16), max(2, ws // 16), generator=g)
        hr = F.interpolate(base, size=(hs, ws), mode="bicubic", align_corners=False).clamp_(0, 1)
        hrs.append(hr)
    hr = torch.cat(hrs)
    lr = F.interpolate(hr, size=(h, w), mode="bilinear", align_corners=False, antialias=True).clamp_(0, 1)
    return lr, hr


IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def normalize(x01: torch.Tensor, mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    m = torch.tensor(mean, dtype=x01.dtype, device=x01.device).view(1, 3, 1, 1)
    s = torch.tensor(std, dtype=x01.dtype, device=x01.device).view(1, 3, 1, 1)
    return (x01 - m) / s


HELDOUT_SEED = 20_251_018  # never used by train.py's synthetic stream (seed*1_000_003 + i, seed = 100*131 + rank)


def heldout_tiles(n: int, lr_size: int = 128, scale: int = 4, seed: int = HELDOUT_SEED, device="cpu",
                  mean=IMAGENET_MEAN, std=IMAGENET_STD) -> tuple[torch.Tensor, torch.Tensor]:
    """Held-out tiles of the `leaves` synthetic distribution the committed trained weights were
    trained on (data.leaves_hr_u8: dead-leaves images with a 1/f texture).

    Tile i is drawn from its own generator (seed + i) on `device`, so it does not depend on n (the
    values do depend on the device's RNG: CPU and GPU tiles differ, each is reproducible).  HR:
    uint8 images of side lr_size*scale; LR: train.py's transform of them (cv2 INTER_LINEAR resize
    of the uint8 crop, rounded half up, then Normalize — data.GPUTransform's formula,
    utils/datasets.py:302-304).  Returns (lr normalised fp32 [n,3,h,w], hr in [0,1] fp32
    [n,3,h*scale,w*scale]), on the CPU."""
    import torch.nn.functional as F

    from .data import leaves_hr_u8
    t = lr_size * scale
    hr_u8 = torch.cat([leaves_hr_u8(1, t, torch.Generator(device=device).manual_seed(seed + i), device)
                       for i in range(n)]).cpu()
    x255 = hr_u8.float()
    lr = F.interpolate(x255, size=(lr_size, lr_size), mode="bilinear", align_corners=False, antialias=False)
    lr = (lr + 0.5).floor_().div_(255.0)
    return normalize(lr, mean, std).contiguous(), (x255 / 255.0).contiguous()


HELDOUT_STILL_SEED = 20_261_018


def heldout_still(h: int, w: int, scale: int, seed: int = HELDOUT_STILL_SEED, tile: int = 512, device="cuda"):
    """A large held-out image of the trained weights' distribution: an HR mosaic of `tile`² dead-leaves
    images (data.leaves_hr_u8 at the training crops' size, one generator per still), cropped to
    (scale*h, scale*w), and its LR = train.py's transform (uint8 bilinear resize rounded half up,
    heldout_tiles' formula).  Returns (LR uint8 [3, h, w], HR uint8 [3, scale*h, scale*w]) on the CPU —
    the cfg4 still (3840x2160 -> 15360x8640) and the cfg5 frames (1920x1080 -> 3840x2160) of the
    parity tests."""
    import torch.nn.functional as F

    from .data import leaves_hr_u8
    th, tw = -(-scale * h // tile), -(-scale * w // tile)
    g = torch.Generator(device=device).manual_seed(seed)
    hr = torch.empty(3, th * tile, tw * tile, dtype=torch.uint8, device=device)
    for i in range(th):
        for j in range(tw):
            hr[:, i * tile:(i + 1) * tile, j * tile:(j + 1) * tile] = leaves_hr_u8(1, tile, g, device)[0]
    hr = hr[:, :scale * h, :scale * w].contiguous()
    lr = F.interpolate(hr[None].float(), size=(h, w), mode="bilinear", align_corners=False, antialias=False)
    lr = (lr + 0.5).floor_().clamp_(0, 255).to(torch.uint8)[0]
    return lr.cpu(), hr.cpu()
