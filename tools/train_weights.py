#!/usr/bin/env python3
"""Make the trained ResNet(16, 0.2, x4 / x2) weights the parity tests and bench use (GPU).

Runs this repo's own `train.py --resnet` (pixel MSE, Adam, LinearLR, EMA; utils/models.py:592-618,
train.py:41-67 of the reference) on synthetic `leaves` crops (data.leaves_hr_u8: dead-leaves images with a
1/f texture, the standard synthetic stand-in for natural-image statistics), then stores the EMA generator exactly as
train.py's checkpoint holds it (fp16 state_dict, checkpoint.save_checkpoint) as safetensors, and
reports PSNR on held-out tiles (the test set of tests/test_gpu_trained.py) for the HIP path and
bicubic upsampling; the HIP output of two of them is saved for the CPU comparison with the oracle.

    python tools/train_weights.py --epochs 8 --steps 500 --out gpurun_out/trained_resnet_x4.safetensors
    python tools/train_weights.py --scale 2 --shape 256 --epochs 12 --steps 500   # the x2 model of cfg5
"""
from __future__ import annotations

import argparse
import json
import math
import sys
import time
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def psnr(a, b, peak=2.0):
    return 10 * math.log10(peak * peak / torch.mean((a.double() - b.double()) ** 2).item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--scale", type=int, default=4, choices=(2, 4))
    ap.add_argument("--shape", type=int, default=512, help="HR crop side (LR = shape / scale)")
    ap.add_argument("--work_dir", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    sc = a.scale
    if a.work_dir is None:
        a.work_dir = f"/tmp/isr_train_weights_x{sc}"
    if a.out is None:
        a.out = f"gpurun_out/trained_resnet_x{sc}.safetensors"

    import train
    from image_super_resolution_amd import checkpoint, models
    from image_super_resolution_amd.weights import heldout_tiles

    argv = ["--resnet", "--scale", str(sc), "--synthetic", "--synthetic_kind", "leaves", "--shape", str(a.shape),
            "--batch_size", str(a.batch), "--epochs", str(a.epochs), "--steps", str(a.steps), "--rs_deep", "16",
            "--add_rate", "0.2", "--lr", str(a.lr), "--work_dir", a.work_dir, "--save_name", "leaves"]
    t0 = time.time()
    train.main(train.parse(argv))
    t_train = time.time() - t0
    ck = Path(a.work_dir) / "res_leaves_16_0.2.pt"
    sd = checkpoint.load_module_state(ck, "ema")  # fp32 values of the fp16 EMA state_dict
    from safetensors.torch import save_file
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    save_file({k: (v.half() if v.is_floating_point() else v).contiguous() for k, v in sd.items()}, out.as_posix())

    net = models.ResNet(16, 0.2, scaleRate=sc)
    net.load_state_dict(sd)
    net = net.eval().to("cuda")
    lr, hr = heldout_tiles(16, 128, scale=sc, device="cuda")
    with torch.no_grad():
        y = net(lr.to("cuda")).float().cpu()
    hr1 = hr * 2 - 1
    lr01 = lr * torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1) + torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    bic = F.interpolate(lr01, scale_factor=sc, mode="bicubic", align_corners=False).clamp(0, 1) * 2 - 1
    res = {"scale": sc, "hr_crop": a.shape, "train_s": round(t_train, 1), "steps": a.epochs * a.steps, "batch": a.batch,
           "psnr_hip_vs_hr_db": round(psnr(y, hr1), 3), "psnr_bicubic_vs_hr_db": round(psnr(bic, hr1), 3)}
    # the HIP output of the first two tiles, for the CPU-side comparison against the oracle
    # (tests/diag_precision.py; tools/ never imports the oracle)
    torch.save({"y": y[:2].clone(), "lr": lr[:2].clone(), "hr": hr[:2].clone()}, (out.parent / ("trained_heldout_hip_y.pt" if sc == 4 else f"trained_heldout_hip_y_x{sc}.pt")).as_posix())
    print(json.dumps(res), flush=True)
    (out.parent / ("train_weights.json" if sc == 4 else f"train_weights_x{sc}.json")).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
