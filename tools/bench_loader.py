#!/usr/bin/env python3
"""f2: can the host data path feed one GPU's training step?

Writes `--images` synthetic 640x480 JPEGs (smooth random content, PIL quality 90, the size of a
typical COCO image train.py's SR_dataset reads), then times data.SRCropDataset (PIL decode +
random 512² crop, reflect-padded where the image is smaller, utils/datasets.py:344-347) behind
the DataLoader train.py builds (batch 16, shuffle, drop_last, pin_memory on a GPU box) at each
`--workers` count, in samples/s.  The GPU side (resize to LR + Normalize) is one HIP launch
(data.GPUTransform, tests/test_gpu_data.py) and is not part of this figure.

Reference point: one MI355X consumes 16 samples per cfg3 SRGAN step (~51.8 ms) = ~309 samples/s.
usage: python tools/bench_loader.py [--workers 4 8 16] [--images 256] [--batches 24]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import data  # noqa: E402


def make_jpegs(root: Path, n: int, seed: int = 0) -> None:
    from PIL import Image
    rng = np.random.default_rng(seed)
    for i in range(n):
        lo = torch.from_numpy(rng.random((1, 3, 15, 20), dtype=np.float32))
        im = torch.nn.functional.interpolate(lo, size=(480, 640), mode="bicubic", align_corners=False)
        im = im + torch.from_numpy(rng.normal(0, 0.03, (1, 3, 480, 640)).astype(np.float32))  # texture
        a = (im.clamp(0, 1)[0].permute(1, 2, 0).numpy() * 255).round().astype(np.uint8)
        Image.fromarray(a).save(root / f"img_{i:05d}.jpg", quality=90)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, nargs="+", default=[4, 8, 16])
    ap.add_argument("--images", type=int, default=256)
    ap.add_argument("--batches", type=int, default=24)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--target", type=int, default=512)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from torch.utils.data import DataLoader
    pin = torch.cuda.is_available()
    res = {"metric": "SRCropDataset + DataLoader samples/s (640x480 JPEG, 512 crop)", "batch": args.batch,
           "images": args.images, "pin_memory": pin, "cpu_count": os.cpu_count(),
           "affinity": len(os.sched_getaffinity(0)), "gpu_step_consumption": 309.0, "runs": []}
    with tempfile.TemporaryDirectory() as d:
        root = Path(d)
        t0 = time.perf_counter()
        make_jpegs(root, args.images)
        res["jpeg_write_s"] = round(time.perf_counter() - t0, 2)
        ds = data.SRCropDataset(root, args.target, 4)
        for w in args.workers:
            dl = DataLoader(ds, batch_size=args.batch, shuffle=True, num_workers=w, drop_last=True,
                            pin_memory=pin, persistent_workers=w > 0)
            it, seen = iter(dl), 0
            for _ in range(2):  # warm-up: workers started, first files in the page cache
                next(it)
            t0 = time.perf_counter()
            for _ in range(args.batches):
                try:
                    b = next(it)
                except StopIteration:
                    it = iter(dl)
                    b = next(it)
                seen += b.shape[0]
            dt = time.perf_counter() - t0
            run = {"workers": w, "samples_per_s": round(seen / dt, 1), "ms_per_batch": round(dt * 1e3 / args.batches, 2)}
            res["runs"].append(run)
            print(json.dumps(run), flush=True)
            del it, dl
    best = max(r["samples_per_s"] for r in res["runs"])
    res["best_samples_per_s"] = best
    res["feeds_one_gpu"] = best >= res["gpu_step_consumption"]
    print(json.dumps(res), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
