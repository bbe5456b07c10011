#!/usr/bin/env python3
"""Drop-in for the reference's rs.py image branch (rs.py:118-124 CLI,
rs.py:78-114 tiling loop): upscale one still with the HIP generator.

    python rs.py --model res_checkpoint_16_0.2.pt --src in.png --save_dir out.png \
                 --window_size 512 --batch_size 8 [--halo 32]

Multi-GPU: launch with torch.distributed.run; tiles are
dealt across ranks and rank 0 writes the image.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 rs.py ...

`--model` takes a checkpoint written by this package's train.py (state_dicts,
loaded with weights_only=True) or a state_dict / .safetensors file; the
reference's TorchScript export is not executed.
Video inputs (rs.py:54-76) need the ffmpeg binary and are not handled here.
"""
from __future__ import annotations

import argparse
import os
import time
from pathlib import Path

import numpy as np
import torch

from image_super_resolution_amd import checkpoint, models, tiler

VID_FORMATS = ('.mp4', '.avi', '.mkv', '.mov', '.wmv', '.flv', '.webm', '.mpeg', '.mpg', '.m4v', '.ts')


def read_image(path: Path) -> torch.Tensor:
    """uint8 [3,H,W] RGB (torchvision.io.read_image(..., ImageReadMode.RGB))."""
    from PIL import Image
    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGB"))
    return torch.from_numpy(arr.copy()).permute(2, 0, 1).contiguous()


def write_png(img: torch.Tensor, path: Path) -> None:
    from PIL import Image
    Image.fromarray(img.permute(1, 2, 0).contiguous().cpu().numpy()).save(path.as_posix(), format="PNG")


def build_model(path: str, add_rate: float, mean, std) -> models.Model:
    sd = checkpoint.load_module_state(path, ("ema", "gen_net"))
    gen = checkpoint.generator_from_state(sd, add_rate)
    m = models.Model(gen)
    m.init_normalize(mean, std)
    return m.fuse().eval()


def runer(**kw):
    src, result = Path(kw["src"]), Path(kw["save_dir"])
    if src.suffix.lower() in VID_FORMATS:
        raise NotImplementedError("video super-resolution (rs.py:54-76) needs ffmpeg, which this image lacks")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("rs.py runs the HIP generator and needs a GPU")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)
    mean, std = kw["mean"], kw["std"]
    model = build_model(kw["model"], kw["add_rate"], mean, std)
    runner = tiler.runner_for(model, device)
    up = tiler.TileUpscaler(runner, runner.scale, window=kw["window_size"], halo=kw["halo"],
                            batch=kw["batch_size"], device=device)
    image = read_image(src)
    if rank == 0:
        print("input shape", tuple(image.shape))
    t0 = time.perf_counter()
    out = up(image, rank=rank, world=world)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if rank == 0:
        result = result.with_suffix(".png")
        write_png(out, result)
        mpix = out.shape[1] * out.shape[2] / 1e6
        print("output shape", tuple(out.shape), result.as_posix(), f"{dt:.3f}s {mpix / dt:.1f} MPix/s")
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--model", type=str, default="")
    p.add_argument("--src", type=str, default="")
    p.add_argument("--save_dir", type=str, default="result.jpg")
    p.add_argument("--window_size", type=int, default=96)
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--worker", type=int, default=4, help="accepted for CLI compatibility (decode is in-process)")
    p.add_argument("--halo", type=int, default=0, help="LR pixels of context around each window (0 = reference)")
    p.add_argument("--add_rate", type=float, default=0.2)
    p.add_argument("--mean", type=float, nargs=3, default=(0.485, 0.456, 0.406))
    p.add_argument("--std", type=float, nargs=3, default=(0.229, 0.224, 0.225))
    runer(**vars(p.parse_args()))
