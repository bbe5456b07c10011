#!/usr/bin/env python3
"""Training-step throughput: SRGAN-mode step of the 4x
EResNet generator with the VGG19 conv5_4 (pre-activation, L1) perceptual loss
and the adversarial term, batch 16 of 128² LR → 512² HR per GPU, Adam + EMA.

python tools/bench_train.py [--steps 5] [--warmup 2] [--mode srgan|pixel]
Launch with torch.distributed.run for N GPUs (one process per GPU, RCCL).
Prints one JSON line on rank 0 (HR megapixels/s and samples/s, whole job).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import data, loss as L, models, optim, trainer  # noqa: E402
from image_super_resolution_amd.train_engine import enable_grad_allreduce  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--hr", type=int, default=512)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--mode", default="srgan", choices=["srgan", "pixel"])
    ap.add_argument("--torch-profile", action="store_true", help="print the PyTorch copy/fill ops per step")
    ap.add_argument("--dis-layout", default="nhwc", choices=["nchw", "nhwc"],
                    help="discriminator memory format (stock MIOpen convs)")
    ap.add_argument("--dis-miopen", action="store_true", help="discriminator conv stack on stock MIOpen convs")
    ap.add_argument("--no-miopen-find", dest="miopen_find", action="store_false",
                    help="torch.backends.cudnn.benchmark = False (default: MIOpen find mode on, as train.py)")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    group = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
        group = True
    torch.manual_seed(0)
    mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
    batches = data.SyntheticSR(args.batch, args.hr, seed=rank, device=dev)
    total = args.steps + args.warmup
    if args.mode == "srgan":
        gen = models.SRGAN(args.blocks, 0.2, True, 4).to(dev)
        dis = models.Discriminator(3, 64, 8, 1024).to(dev)
        dis.use_libisr(not args.dis_miopen)
        if args.dis_miopen and args.dis_layout == "nhwc":
            dis = dis.to(memory_format=torch.channels_last)
        torch.backends.cudnn.benchmark = args.miopen_find and args.dis_miopen
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            gl = L.gen_loss(device=dev, beforeAct=True)
        og = optim.FusedAdam(gen.parameters(), lr=1e-4, betas=(0.9, 0.999))
        od = optim.FusedAdam(dis.parameters(), lr=1e-4, betas=(0.9, 0.999))
        sg = torch.optim.lr_scheduler.LinearLR(og, 1, 0.01, total_iters=total)
        sd = torch.optim.lr_scheduler.LinearLR(od, 1, 0.01, total_iters=total)
        ema = models.ModelEMA(gen, tau=total)
        ema.ema.to(dev)
        if group:
            enable_grad_allreduce(gen, group)
        sc = (torch.amp.GradScaler("cuda", enabled=False), torch.amp.GradScaler("cuda", enabled=False))
        tf = data.GPUTransform(4, hr_norm=True, mean=mean, std=std, device=dev)

        def run(n):
            trainer.train_srgan(gen, ema, dis, batches, tf, gl, og, od, sc, (sg, sd), 0, None, mean=mean, std=std,
                                steps=n, log_every=10 ** 9, dist_group=group)
    else:
        gen = models.EResNet(args.blocks, 0.2, 4).to(dev)
        og = optim.FusedAdam(gen.parameters(), lr=1e-4)
        sg = torch.optim.lr_scheduler.LinearLR(og, 1, 0.01, total_iters=total)
        ema = models.ModelEMA(gen, tau=total)
        ema.ema.to(dev)
        if group:
            enable_grad_allreduce(gen, group)
        tf = data.GPUTransform(4, hr_norm=False, mean=mean, std=std, device=dev)
        l1 = L.L1Loss().to(dev)

        def run(n):
            trainer.train(gen, ema, batches, tf, l1, og, torch.amp.GradScaler("cuda", enabled=False), sg, 0, None,
                          steps=n, log_every=10 ** 9)
    run(args.warmup)
    torch.cuda.synchronize()
    if args.torch_profile:  # which PyTorch ops (copies / fills / adds) a step issues, with call sites
        import collections
        import traceback
        from torch.utils._python_dispatch import TorchDispatchMode
        keys = {"copy_", "fill_", "zero_", "clone", "add_", "add", "mul", "mul_", "sub", "div", "_to_copy", "cat",
                "stack", "zeros_like", "ones_like", "where", "abs", "sum", "mean"}
        root = str(Path(__file__).resolve().parents[1])
        # ISR_TORCH_PROFILE_ALL=1: every aten op that may launch a kernel, sorted by count
        ALL = os.environ.get("ISR_TORCH_PROFILE_ALL") == "1"
        NOLAUNCH = {"view", "_unsafe_view", "reshape", "as_strided", "t", "permute", "detach", "expand", "slice",
                    "select", "alias", "empty", "empty_strided", "empty_like", "unsqueeze", "squeeze", "transpose",
                    "split", "split_with_sizes", "unbind", "new_empty", "new_empty_strided", "set_", "lift_fresh",
                    "_local_scalar_dense", "is_nonzero", "resolve_conj", "resolve_neg", "record_stream"}

        class _Count(TorchDispatchMode):
            def __init__(self):
                super().__init__()
                self.n = collections.Counter()
                self.bytes = collections.Counter()

            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                name = func.overloadpacket.__name__
                if name in keys or (ALL and name not in NOLAUNCH):
                    fr = [f for f in traceback.extract_stack()[:-1]
                          if f.filename.startswith(root) and "bench_train" not in f.filename]
                    site = " <- ".join(f"{Path(f.filename).name}:{f.lineno}" for f in fr[::-1][:3])
                    a0 = args[0] if args and isinstance(args[0], torch.Tensor) else None
                    self.n[(name, site)] += 1
                    self.bytes[(name, site)] += 0 if a0 is None else a0.numel() * a0.element_size()
                return func(*args, **(kwargs or {}))

        mode = _Count()
        with mode:
            run(args.steps)
            torch.cuda.synchronize()
        order = (lambda kv: -kv[1]) if ALL else (lambda kv: -mode.bytes[kv[0]])
        for (name, site), c in sorted(mode.n.items(), key=order)[:60]:
            print(f"{c / args.steps:7.1f}/step {mode.bytes[(name, site)] / args.steps / 2**20:10.1f} MiB/step "
                  f"{name:10s} {site}")
        return
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = torch.tensor(time.perf_counter() - t0, device=dev)
    if world > 1:
        torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    dt = dt.item()
    samples = args.steps * args.batch * world
    # algorithmic FLOPs of one step per GPU (2*MAC of every conv the step runs):
    # G fwd (engine.generator_flops) + G bwd (dgrad + wgrad = 2x fwd); VGG19 to conv5_4 on SR
    # and HR (203.8 GFLOP per 512² image) + its input-gradient on SR; D (49.26 GFLOP per 512²
    # image, torch FlopCounterMode of models.Discriminator): D(sr) fwd + dgrad for the G loss,
    # D(sr), D(hr) fwd + dgrad + wgrad for the D loss.  srgan mode only.
    from image_super_resolution_amd import engine
    lr = args.hr // 4
    g_fwd = engine.generator_flops(lr, lr, args.blocks, 2) * args.batch
    scale = (args.hr / 512) ** 2 * args.batch
    vgg_fwd, d_fwd = 203.8e9 * scale, 49.26e9 * scale
    step_flops = (3 * g_fwd + 3 * vgg_fwd + 2 * d_fwd + 2 * d_fwd + 2 * 2 * d_fwd) if args.mode == "srgan" else 3 * g_fwd
    tflops = step_flops / (dt / args.steps) / 1e12
    if rank == 0:
        print(json.dumps({"metric": f"{args.mode} train step throughput (4x EResNet, VGG19 5_4 L1 + adv)",
                          "value": round(samples * args.hr * args.hr / 1e6 / dt, 2), "unit": "HR MPix/s",
                          "samples_per_s": round(samples / dt, 2), "ms_per_step": round(dt * 1e3 / args.steps, 2),
                          "n_gpus": world, "global_batch": args.batch * world, "steps": args.steps,
                          "discriminator": "miopen" if args.dis_miopen else "libisr",
                          "mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1),
                          "tflop_per_step": round(step_flops / 1e12, 2), "tflops_per_s": round(tflops, 1),
                          "mfma_frac": round(tflops / 2500.0, 4)}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
