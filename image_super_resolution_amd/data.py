"""Training data for the SR generator (utils/datasets.py:274-355 SR_dataset).

The reference decodes, crops, resizes and normalises every sample on CPU
workers (cv2 + albumentations).  Here the CPU side only decodes and crops
(uint8, the smallest thing to move); resize to LR, Normalize and the HR
transform (PIL_to_tanh, utils/datasets.py:96-106, or Normalize for SRGAN
mode, :336-339) run batched on the GPU (`GPUTransform`).  `SyntheticSR`
generates smooth random HR crops directly on the GPU (no dataset is
available offline; SURVEY.md §8d's synthetic recipe).
"""
from __future__ import annotations

import json
import random
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import Dataset

IMG_FORMATS = (".bmp", ".jpg", ".jpeg", ".png", ".tif", ".tiff", ".webp")
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def ground_up(x: int, factor: int) -> int:
    """utils/general.py ground_up: round x up to a multiple of factor."""
    return (x + factor - 1) // factor * factor


def list_images(src) -> list[str]:
    """A JSON list of paths (train.py:191 train_images.json) or a directory."""
    src = Path(src)
    if src.suffix == ".json":
        with open(src) as f:
            return [str(p) for p in json.load(f)]
    return sorted(str(p) for p in src.rglob("*") if p.suffix.lower() in IMG_FORMATS)


class SRCropDataset(Dataset):
    """Random `target_size` RGB crops as uint8 CHW (SR_dataset's RandomCrop,
    utils/datasets.py:288, 344-347); images smaller than the crop are padded."""

    def __init__(self, src, target_size: int, scale: int, prefix: str = ""):
        self.samples = list_images(src)
        if not self.samples:
            raise FileNotFoundError(f"no images under {src}")
        self.target_size = ground_up(target_size, scale)
        self.scale = scale
        print(f"{prefix}{len(self.samples)} images with target shape {self.target_size} with scale factor {scale}.")

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        from PIL import Image
        with Image.open(self.samples[i]) as im:
            a = np.asarray(im.convert("RGB"))
        t = self.target_size
        h, w = a.shape[:2]
        if h < t or w < t:
            a = np.pad(a, ((0, max(0, t - h)), (0, max(0, t - w)), (0, 0)), mode="reflect")
            h, w = a.shape[:2]
        y, x = random.randint(0, h - t), random.randint(0, w - t)
        return torch.from_numpy(np.ascontiguousarray(a[y:y + t, x:x + t])).permute(2, 0, 1).contiguous()


class GPUTransform:
    """Batched (hr, lr) from uint8 HR crops on the device:
    lr = Normalize(Resize(crop, T/scale)) (albumentations Resize = cv2 INTER_LINEAR,
    utils/datasets.py:302-303); hr = 2*crop/255 - 1 (PIL_to_tanh) or
    Normalize(crop) when hr_norm (set_transform_hr, SRGAN mode).

    cv2 resizes the uint8 image and returns uint8: at the integer factors train.py uses
    (2, 3, 4) its fixed-point INTER_LINEAR (11-bit coefficients; x2 runs as INTER_AREA)
    samples at src = scale*(d + 0.5) - 0.5 with weights 0 / 0.5 / 1, i.e. the exact float
    bilinear value rounded half up — reproduced here by rounding the float interpolation
    of the uint8 values (oracle.ref_cpu.cv2_resize_linear_u8 restates the fixed-point
    arithmetic; tests/test_data_cpu.py)."""

    def __init__(self, scale: int, hr_norm: bool = False, mean=IMAGENET_MEAN, std=IMAGENET_STD, device="cuda"):
        self.scale, self.hr_norm = scale, hr_norm
        self.mean = torch.tensor(mean, device=device).view(1, 3, 1, 1)
        self.std = torch.tensor(std, device=device).view(1, 3, 1, 1)
        self.mean_f, self.std_f = tuple(float(v) for v in mean), tuple(float(v) for v in std)
        self.device = device

    def __call__(self, crops_u8: torch.Tensor):
        if torch.device(self.device).type == "cuda":
            return self._hip(crops_u8)
        # CPU device: the same formulas as torch ops (host-side tests; the GPU path is the kernel)
        x255 = crops_u8.to(self.device, non_blocking=True).float()
        t = x255.shape[-1]
        lr = F.interpolate(x255, size=(t // self.scale, t // self.scale), mode="bilinear", align_corners=False,
                           antialias=False)
        lr = (lr + 0.5).floor_().div_(255.0)  # cv2's uint8 result (round half up), then /255
        lr = (lr - self.mean) / self.std
        x = x255.div_(255.0)
        hr = (x - self.mean) / self.std if self.hr_norm else x * 2.0 - 1.0
        return hr.contiguous(), lr.contiguous()

    def _hip(self, crops_u8: torch.Tensor):
        """One HIP launch (isr_sr_transform): crop block reads, cv2 resize, both Normalizes."""
        import ctypes

        from . import _lib, ops
        if crops_u8.dtype != torch.uint8 or crops_u8.dim() != 4 or crops_u8.shape[1] != 3:
            raise ValueError(f"GPUTransform expects uint8 [n, 3, t, t] crops, got {crops_u8.dtype} "
                             f"{tuple(crops_u8.shape)}")
        n, _, t, tw = crops_u8.shape
        if t != tw or t % self.scale:
            raise ValueError(f"GPUTransform: square crops with side a multiple of {self.scale}, got {t}x{tw}")
        x = crops_u8.to(self.device, non_blocking=True).contiguous()
        hr = torch.empty((n, 3, t, t), device=x.device)
        lr = torch.empty((n, 3, t // self.scale, t // self.scale), device=x.device)
        d = _lib.IsrSrTransformDesc(x.data_ptr(), hr.data_ptr(), lr.data_ptr(), n, t, self.scale,
                                    int(self.hr_norm), (ctypes.c_float * 3)(*self.mean_f),
                                    (ctypes.c_float * 3)(*self.std_f))
        _lib.check(_lib.load().isr_sr_transform(ctypes.byref(d), ops._stream()), "isr_sr_transform")
        return hr, lr


class NoisyTransform:
    """Batched (clean, noisy) pairs for `train.py --train_denoise` from uint8 crops
    on the device (Noisy_dataset, utils/datasets.py:361-389): clean = 2*crop/255 - 1;
    noisy = Normalize(GaussNoise(crop)), albumentations GaussNoise defaults
    (var_limit (10, 50) on the 0-255 scale, per-channel, p = 0.5 per sample, result
    clipped to [0, 255]).  The reference's ISONoise and ImageCompression (also p = 0.5)
    need a host JPEG codec / HLS conversion and are not reproduced."""

    def __init__(self, mean=IMAGENET_MEAN, std=IMAGENET_STD, var_limit=(10.0, 50.0), p: float = 0.5,
                 device="cuda", seed: int = 0):
        self.mean = torch.tensor(mean, device=device).view(1, 3, 1, 1)
        self.std = torch.tensor(std, device=device).view(1, 3, 1, 1)
        self.var_limit, self.p, self.device = var_limit, p, device
        self.gen = torch.Generator(device=device).manual_seed(seed)

    def __call__(self, crops_u8: torch.Tensor):
        x = crops_u8.to(self.device, non_blocking=True).float()
        n = x.shape[0]
        g = self.gen
        var = torch.empty(n, 1, 1, 1, device=self.device).uniform_(*self.var_limit, generator=g)
        apply = (torch.rand(n, 1, 1, 1, device=self.device, generator=g) < self.p).float()
        noise = torch.randn(x.shape, device=self.device, generator=g) * var.sqrt() * apply
        noisy = (x + noise).clamp_(0, 255).div_(255.0)
        lr = (noisy - self.mean) / self.std
        hr = x / 255.0 * 2.0 - 1.0
        return hr.contiguous(), lr.contiguous()


NATURAL_ALPHA = 1.4  # amplitude spectrum 1/f^alpha: x4 bicubic PSNR ~27.7 dB, the regime of COCO crops


def natural_hr_u8(n: int, t: int, generator: torch.Generator, device="cuda", alpha: float = NATURAL_ALPHA,
                  contrast: float = 0.25) -> torch.Tensor:
    """uint8 [n, 3, t, t] Gaussian fields with a natural-image power spectrum.

    White noise (a luma field shared by the channels plus 0.35x independent colour noise) shaped
    by 1/f^alpha in the Fourier domain, unit standard deviation per image, mapped to
    0.5 + contrast*x and clipped to [0, 1].  At alpha = 1.4 the x4 task is as hard as natural
    photos are for bicubic upsampling (about 27.7 dB PSNR on the cv2 LR of train.py), unlike the
    smooth kind, where bicubic already reaches ~46 dB and the last bf16 bits never matter."""
    w = torch.randn(n, 3, t, t, generator=generator, device=device)
    luma = torch.randn(n, 1, t, t, generator=generator, device=device)
    w = 0.35 * w + luma
    fy = torch.fft.fftfreq(t, device=device).view(-1, 1)
    fx = torch.fft.rfftfreq(t, device=device).view(1, -1)
    f = torch.sqrt(fx * fx + fy * fy).clamp_min(1.0 / t)
    x = torch.fft.irfft2(torch.fft.rfft2(w) / f.pow(alpha), s=(t, t))
    x = x / x.flatten(1).std(1).view(-1, 1, 1, 1)
    return (0.5 + contrast * x).clamp_(0, 1).mul_(255).round_().to(torch.uint8)


def leaves_hr_u8(n: int, t: int, generator: torch.Generator, device="cuda", discs: int = 500, rmin: float = 4.0,
                  contrast: float = 0.6, texture: float = 0.3) -> torch.Tensor:
    """uint8 [n, 3, t, t] 'dead leaves' images: the standard synthetic model of natural-image
    statistics (occluding objects with a power-law size distribution give sharp edges and a
    1/f-like spectrum), plus a 1/f^1.4 texture (natural_hr_u8) on top.

    `discs` opaque discs per image, front to back: centre uniform over the image, radius
    r ~ r^-3 on [rmin, t/3], a uniform random RGB colour; every pixel shows the first disc that
    covers it (grey where none does); colours enter as 0.5 + contrast*(c - 0.5), the texture as
    texture*(its [0, 1] value - 0.5).  x4 bicubic on these reaches ~27 dB, a trained x4 RRDB
    generator a few dB more (edges are what SR recovers; a Gaussian field has none)."""
    ys = torch.arange(t, dtype=torch.float32, device=device).view(1, t, 1)
    xs = torch.arange(t, dtype=torch.float32, device=device).view(1, 1, t)
    rmax, a1 = t / 3.0, -2.0  # 1 - alpha for alpha = 3
    out = torch.empty(n, 3, t, t, device=device)
    for i in range(n):
        cy = torch.rand(discs, generator=generator, device=device) * t
        cx = torch.rand(discs, generator=generator, device=device) * t
        u = torch.rand(discs, generator=generator, device=device)
        r2 = ((rmin ** a1 + u * (rmax ** a1 - rmin ** a1)) ** (1.0 / a1)) ** 2
        col = 0.5 + contrast * (torch.rand(discs, 3, generator=generator, device=device) - 0.5)
        top = torch.full((t, t), discs, dtype=torch.long, device=device)  # index of the top disc
        for j0 in range(0, discs, 64):  # front to back: a pixel keeps the first disc that covers it
            sl = slice(j0, min(j0 + 64, discs))
            inside = (ys - cy[sl].view(-1, 1, 1)) ** 2 + (xs - cx[sl].view(-1, 1, 1)) ** 2 <= r2[sl].view(-1, 1, 1)
            first = inside.to(torch.uint8).argmax(0) + j0
            top = torch.where(inside.any(0) & (top == discs), first, top)
        pal = torch.cat([col, torch.full((1, 3), 0.5, device=device)])
        out[i] = pal[top].permute(2, 0, 1)
    tex = natural_hr_u8(n, t, generator, device).float().div_(255.0).sub_(0.5)
    return (out + texture * tex).clamp_(0, 1).mul_(255).round_().to(torch.uint8)


class SyntheticSR:
    """Endless synthetic uint8 HR crops on the GPU, seed per batch and rank.

    kind "smooth": bicubic-upsampled 32x32 uniform noise (a smooth 'natural-ish' image);
    kind "natural": 1/f^1.4 Gaussian fields (natural_hr_u8);
    kind "leaves": dead-leaves images with a 1/f texture (leaves_hr_u8), the data the committed
    trained weights (tests/golden/trained_resnet_x4.safetensors) were made from."""

    def __init__(self, batch: int, target_size: int, seed: int = 0, device="cuda", kind: str = "smooth"):
        if kind not in ("smooth", "natural", "leaves"):
            raise ValueError(f"SyntheticSR kind {kind!r}: 'smooth', 'natural' or 'leaves'")
        self.batch, self.t, self.seed, self.device, self.kind = batch, target_size, seed, device, kind
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self) -> torch.Tensor:
        g = torch.Generator(device=self.device).manual_seed(self.seed * 1_000_003 + self.i)
        self.i += 1
        if self.kind == "natural":
            return natural_hr_u8(self.batch, self.t, g, self.device)
        if self.kind == "leaves":
            return leaves_hr_u8(self.batch, self.t, g, self.device)
        base = torch.rand(self.batch, 3, 32, 32, generator=g, device=self.device)
        hr = F.interpolate(base, size=(self.t, self.t), mode="bicubic", align_corners=False).clamp_(0, 1)
        return (hr * 255).round_().to(torch.uint8)
