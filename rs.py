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
Video (rs.py:54-76, BASELINE cfg5): container formats are decoded / encoded by
the ffmpeg binary through raw pipes (as the reference does); headerless rgb24
input (.rgb, with --video_size WxH) and bgr24 output (.bgr / .raw save_dir) work
without ffmpeg.  The per-batch forward is a captured HIP graph (video.py).

    python rs.py --model ck.pt --src clip.mp4 --save_dir out.mp4 --batch_size 2
"""
from __future__ import annotations

import argparse
import os
import time
from pathlib import Path

import numpy as np
import torch

from image_super_resolution_amd import checkpoint, models, tiler, video

VID_FORMATS = video.VID_FORMATS
RAW_FORMATS = (".rgb", ".raw", ".rgb24")


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


def run_video(kw, device) -> None:
    """rs.py:54-76: frames → HIP graph forward → BGR frames → recorder."""
    src, result = Path(kw["src"]), Path(kw["save_dir"])
    wh = kw.get("video_size")
    w, h = (int(v) for v in wh.lower().split("x")) if wh else (None, None)
    source = video.open_video(src, w, h, kw.get("fps") or 30.0)
    model = build_model(kw["model"], kw["add_rate"], kw["mean"], kw["std"])
    runner = tiler.runner_for(model, device)
    up = video.FrameUpscaler(runner.gw, source.height, source.width, kw["batch_size"], runner.mean, runner.std,
                             device)
    H, W = up.out_hw
    if result.suffix.lower() in (".bgr", ".raw"):
        rec = video.RawRecorder(result, (W, H), source.fps)
    else:
        result = result.with_suffix(".mp4")
        rec = video.FFMPEG_recorder(result.as_posix(), (W, H), source.fps)
    t0 = time.perf_counter()
    n = video.VideoUpscaler(up).run(source, rec)
    rec.stopRecorder()
    dt = time.perf_counter() - t0
    if src.suffix.lower() in VID_FORMATS:
        rec.addAudio(src.as_posix())
    print(f"{n} frames {source.width}x{source.height} -> {W}x{H} in {dt:.2f}s ({n / dt:.2f} fps) -> {result}")


def runer(**kw):
    src, result = Path(kw["src"]), Path(kw["save_dir"])
    if src.suffix.lower() in VID_FORMATS + RAW_FORMATS:
        if not torch.cuda.is_available():
            raise RuntimeError("rs.py runs the HIP generator and needs a GPU")
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(device)
        return run_video(kw, device)
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
                            batch=kw["batch_size"], device=device, shard=kw.get("shard", "windows"),
                            gather=kw.get("gather", "device"))
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
    p.add_argument("--shard", choices=("windows", "bands", "blocks"), default="windows",
                   help="windows (the reference's, default), full-width bands or a 2-D grid of blocks with the "
                        "same halo: fewer, larger forwards (cfg4 on one MI355X: 576 vs 460 MPix/s with --halo 32)")
    p.add_argument("--gather", choices=("device", "host"), default="device",
                   help="multi-GPU: finished tiles to rank 0's device (p2p) or into one shared host canvas")
    p.add_argument("--add_rate", type=float, default=0.2)
    p.add_argument("--mean", type=float, nargs=3, default=(0.485, 0.456, 0.406))
    p.add_argument("--std", type=float, nargs=3, default=(0.229, 0.224, 0.225))
    p.add_argument("--video_size", type=str, default=None, help="WxH of a raw rgb24 video input")
    p.add_argument("--fps", type=float, default=None, help="frame rate of a raw rgb24 video input")
    runer(**vars(p.parse_args()))
