#!/usr/bin/env python3
"""Drop-in for the reference's train.py CLI (train.py:141-163) on MI355X.

    python train.py --resnet --enchant --scale 4 --batch_size 16 --shape 512 --epochs 300
    python train.py --enchant --scale 4 ...              # SRGAN mode: VGG perceptual + adversarial
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py ...  # data parallel

Same flags and checkpoint names (res_/gen_{save_name}_{rs_deep}_{add_rate}.pt)
as the reference; checkpoints hold state_dicts (loaded with weights_only=True),
see checkpoint.py.  Data: `--data` takes a directory of images or a JSON list
(the reference reads ./train_images.json); without one, or with --synthetic,
smooth random crops are generated on the GPU.  `--steps` caps iterations per
epoch.  Every mode trains on the HIP path: ResNet (train-mode BatchNorm kernels)
and EResNet (`--enchant`) in `--resnet` pixel-loss mode and in SRGAN mode (VGG
perceptual + adversarial, discriminator on libisr), and the Denoise model
(`--train_denoise`).
"""
from __future__ import annotations

import argparse
import os
import random
from copy import deepcopy
from pathlib import Path

import numpy as np
import torch
from torch import nn

from image_super_resolution_amd import checkpoint, data, loss as L, models, optim, trainer
from image_super_resolution_amd.train_engine import broadcast_params, enable_grad_allreduce


def first_setup(seed):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)


class _Batches:
    """Batches of uint8 HR crops: a DataLoader over SRCropDataset (sharded per
    rank) or the GPU synthetic generator."""

    def __init__(self, opt, target, rank, world, device):
        self.synthetic = opt.synthetic or not opt.data
        if self.synthetic:
            self.src = data.SyntheticSR(opt.batch_size, target, seed=opt.seed * 131 + rank, device=device,
                                        kind=opt.synthetic_kind)
            self.n = opt.steps or 100
        else:
            from torch.utils.data import DataLoader, DistributedSampler
            ds = data.SRCropDataset(opt.data, target, opt.scale, "Train: ")
            sampler = DistributedSampler(ds, world, rank, shuffle=True, seed=opt.seed) if world > 1 else None
            self.sampler = sampler
            self.src = DataLoader(ds, batch_size=opt.batch_size, shuffle=sampler is None, sampler=sampler,
                                  num_workers=opt.worker, drop_last=True, pin_memory=True, persistent_workers=opt.worker > 0)
            self.n = len(self.src)

    def __len__(self):
        return self.n

    def __iter__(self):
        """One endless iterator shared by every epoch (trainer.train takes `steps`
        batches per epoch from it), so --steps below the loader length walks on
        through the data instead of restarting at its head; each pass over the
        loader reshuffles (DistributedSampler.set_epoch per pass, as shuffle=True
        does for the reference's single-process loader)."""
        if self.synthetic:
            return self.src
        if getattr(self, "_it", None) is None:
            def gen():
                npass = 0
                while True:
                    if self.sampler is not None:
                        self.sampler.set_epoch(npass)
                    yield from self.src
                    npass += 1
            self._it = gen()
        return self._it


def setup_resnet(opt, device, group, iters: int, res_ck: Path):
    """`--resnet` pixel-loss mode (train.py:258-302 of the reference): generator,
    EMA, loss, Adam and LinearLR, resumed from `res_ck` with --resume; with a process
    group the gradient all-reduce is enabled and parameters broadcast from rank 0."""
    model = (models.EResNet(opt.rs_deep, opt.add_rate, opt.scale) if opt.enchant
             else models.ResNet(opt.rs_deep, opt.add_rate, scaleRate=opt.scale))
    ema = models.ModelEMA(model, tau=opt.epochs * iters)
    model.to(device)
    ema.ema.to(device)
    compute_loss = L.L1Loss().to(device) if opt.enchant else nn.MSELoss()
    optimizer = optim.FusedAdam(model.parameters(), lr=opt.lr, betas=(0.9, 0.999), weight_decay=opt.weight_decay)
    schedule = torch.optim.lr_scheduler.LinearLR(optimizer, 1, opt.lr2, total_iters=opt.epochs * iters)
    start = 0
    if opt.resume and res_ck.is_file():
        ck = checkpoint.load_checkpoint(res_ck)
        sd = checkpoint.intersect_dicts({k: v.float() for k, v in ck["ema"].items()}, model.state_dict())
        ema.ema.load_state_dict({k: v.float() for k, v in ck["ema"].items()})
        ema.updates = ck["updates"]
        model.load_state_dict(sd, strict=False)
        if len(sd) == len(model.state_dict()):
            if ck.get("optimizer") is not None:
                optimizer.load_state_dict(ck["optimizer"])
            start = ck["epoch"] + 1
    if group is not None:
        enable_grad_allreduce(model, group)
        for p in model.parameters():  # identical start on every rank
            torch.distributed.broadcast(p.data, 0)
    return model, ema, compute_loss, optimizer, schedule, start


def setup_srgan(opt, device, group, iters: int, gen_ck: Path, res_ck: Path):
    """SRGAN-mode models, optimisers, schedules and loss (train.py:304-366 of the
    reference), resumed from `gen_ck` with --resume; with a process group
    (`group` not None) the generator's gradient all-reduce is enabled and every
    parameter is broadcast from rank 0 (DDP's initial sync)."""
    gen_net = models.SRGAN(opt.rs_deep, opt.add_rate, opt.enchant, opt.scale)
    gen_net.init_weight(pretrained=res_ck.as_posix())
    dis_net = models.Discriminator(3, 64, 8, 1024).use_libisr(not opt.dis_miopen)
    ema = models.ModelEMA(gen_net, tau=opt.epochs * iters)
    optimizer_g = optim.FusedAdam(gen_net.parameters(), lr=opt.lr, betas=(0.9, 0.999),
                                   weight_decay=opt.weight_decay)
    optimizer_d = optim.FusedAdam(dis_net.parameters(), lr=opt.lr, betas=(0.9, 0.999),
                                   weight_decay=opt.weight_decay)
    schedule_g = torch.optim.lr_scheduler.LinearLR(optimizer_g, 1, opt.lr2, total_iters=opt.epochs * iters)
    schedule_d = torch.optim.lr_scheduler.LinearLR(optimizer_d, 1, opt.lr2, total_iters=opt.epochs * iters)
    start = 0
    if opt.resume and gen_ck.is_file():
        ck = checkpoint.load_checkpoint(gen_ck)
        gen_net.load_state_dict(checkpoint.intersect_dicts({k: v.float() for k, v in ck["ema"].items()},
                                                           gen_net.state_dict()), strict=False)
        dis_net.load_state_dict(checkpoint.intersect_dicts({k: v.float() for k, v in ck["dis_net"].items()},
                                                           dis_net.state_dict()), strict=False)
        if ck.get("optimizer_g") is not None:
            optimizer_g.load_state_dict(ck["optimizer_g"])
            optimizer_d.load_state_dict(ck["optimizer_d"])
        ema.ema.load_state_dict({k: v.float() for k, v in ck["ema"].items()})
        ema.updates = ck["updates"]
        start = ck["epoch"] + 1
    compute_loss = L.gen_loss(device=device, beforeAct=opt.enchant, vgg_weights=opt.vgg_weights)
    gen_net.to(device)
    if opt.dis_miopen:  # stock convs: NHWC (channels_last) + find mode, ~17 % faster than NCHW
        dis_net.to(device, memory_format=torch.channels_last)
        torch.backends.cudnn.benchmark = True
    else:
        dis_net.to(device)
    ema.ema.to(device)
    if group is not None:
        enable_grad_allreduce(gen_net, group)
        broadcast_params(list(gen_net.parameters()) + list(dis_net.parameters()))
    return gen_net, dis_net, ema, optimizer_g, optimizer_d, schedule_g, schedule_d, compute_loss, start


def main(opt):
    first_setup(opt.seed)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise RuntimeError("train.py runs the HIP training path and needs a GPU")
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    group = None
    if world > 1:
        import torch.distributed as dist
        if opt.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)  # RCCL over xGMI
        else:  # gloo: rehearsal of several ranks on one GPU (RCCL needs one GPU per rank)
            dist.init_process_group(opt.dist_backend)
        group = True
    work_dir = Path(opt.work_dir)
    work_dir.mkdir(exist_ok=True)
    res_ck = work_dir / f"res_{opt.save_name}_{opt.rs_deep}_{opt.add_rate}.pt"
    gen_ck = work_dir / f"gen_{opt.save_name}_{opt.rs_deep}_{opt.add_rate}.pt"
    writer = None
    if rank == 0:
        try:
            from torch.utils.tensorboard import SummaryWriter
            writer = SummaryWriter(work_dir.as_posix(), comment=opt.save_name, flush_secs=30, max_queue=200)
        except Exception:
            writer = None
    target = data.ground_up(opt.shape, opt.scale)
    mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
    batches = _Batches(opt, target, rank, world, device)
    iters = len(batches)
    scaler_gen = torch.amp.GradScaler("cuda", enabled=False)  # bf16: no loss scaling needed
    scaler_dis = torch.amp.GradScaler("cuda", enabled=False)

    if opt.train_denoise:  # train.py:204-243 of the reference
        dn_ck = work_dir / f"denoise_{opt.save_name}_{opt.rs_deep}_{opt.add_rate}.pt"
        model = models.Denoise(opt.rs_deep)
        ema = models.ModelEMA(model)  # reference train.py:206: default tau (2000)
        model.to(device)
        ema.ema.to(device)
        optimizer = optim.FusedAdam(model.parameters(), lr=opt.lr)
        start = 0
        if dn_ck.is_file():
            ck = checkpoint.load_checkpoint(dn_ck)
            print(f"load from {dn_ck.as_posix()}")
            sd = checkpoint.intersect_dicts({k: v.float() if v.is_floating_point() else v
                                             for k, v in ck["gen_net"].items()}, model.state_dict())
            model.load_state_dict(sd, strict=False)
            if len(sd) == len(model.state_dict()) and ck.get("optimizer") is not None:
                optimizer.load_state_dict(ck["optimizer"])
                start = ck["epoch"] + 1
            print(f"Loaded pre-trained {len(sd)}/{len(model.state_dict())} model")
        if group is not None:
            enable_grad_allreduce(model, group)
            broadcast_params(model.parameters())
        schedule = torch.optim.lr_scheduler.LinearLR(optimizer, 1, opt.lr2, total_iters=opt.epochs * iters)
        n_p = sum(p.numel() for p in model.parameters())
        print(f"Model: {n_p:,} parameters, {n_p:,} gradients")
        transform = data.NoisyTransform(mean, std, device=device, seed=opt.seed * 7 + rank)
        for epoch in range(start, opt.epochs):
            losses = trainer.train(model, ema, batches, transform, nn.MSELoss(), optimizer, scaler_gen, schedule,
                                   epoch, writer, steps=iters)
            if rank == 0:
                print(f"epoch {epoch}: loss {np.mean(losses):.5f}")
                checkpoint.save_checkpoint(dn_ck, gen_net=model, optimizer=optimizer.state_dict()
                                           if epoch != opt.epochs - 1 else None, epoch=epoch, mean=mean, std=std)
        return

    if opt.resnet:
        model, ema, compute_loss, optimizer, schedule, start = setup_resnet(opt, device, group, iters, res_ck)
        print(f"Train: ResNet {opt.epochs} epochs, {sum(p.numel() for p in model.parameters()):,} parameters")
        transform = data.GPUTransform(opt.scale, hr_norm=False, mean=mean, std=std, device=device)
        for epoch in range(start, opt.epochs):
            losses = trainer.train(model, ema, batches, transform, compute_loss, optimizer, scaler_gen, schedule,
                                   epoch, writer, steps=iters)
            if rank == 0:
                print(f"epoch {epoch}: loss {np.mean(losses):.5f}")
                checkpoint.save_checkpoint(res_ck, gen_net=model, optimizer=optimizer.state_dict()
                                           if epoch != opt.epochs - 1 else None, epoch=epoch, mean=mean, std=std,
                                           loss=losses, scaler=scaler_gen.state_dict(), ema=ema.ema,
                                           updates=ema.updates)
    else:
        gen_net, dis_net, ema, optimizer_g, optimizer_d, schedule_g, schedule_d, compute_loss, start = \
            setup_srgan(opt, device, group, iters, gen_ck, res_ck)
        print(f"Train: {opt.epochs} epochs, gen {sum(p.numel() for p in gen_net.parameters()):,} parameters, "
              f"dis {sum(p.numel() for p in dis_net.parameters()):,} parameters")
        transform = data.GPUTransform(opt.scale, hr_norm=True, mean=mean, std=std, device=device)
        for epoch in range(start, opt.epochs):
            losses = trainer.train_srgan(gen_net, ema, dis_net, batches, transform, compute_loss, optimizer_g,
                                         optimizer_d, (scaler_gen, scaler_dis), (schedule_g, schedule_d), epoch,
                                         writer, mean=mean, std=std, steps=iters, dist_group=group)
            if rank == 0:
                print(f"epoch {epoch}: content loss {np.mean(losses):.5f}")
                checkpoint.save_checkpoint(gen_ck, gen_net=gen_net, dis_net=dis_net,
                                           optimizer_g=optimizer_g.state_dict() if epoch != opt.epochs - 1 else None,
                                           optimizer_d=optimizer_d.state_dict() if epoch != opt.epochs - 1 else None,
                                           mean=mean, std=std, loss=losses, epoch=epoch,
                                           scaler_gen=scaler_dis.state_dict(), scaler_res=scaler_gen.state_dict(),
                                           ema=ema.ema, updates=ema.updates)
    if writer is not None:
        writer.close()
    if world > 1:
        torch.distributed.destroy_process_group()


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--resnet", action="store_true")
    p.add_argument("--scale", type=int, default=2)
    p.add_argument("--train_denoise", action="store_true")
    p.add_argument("--worker", type=int, default=2)
    p.add_argument("--batch_size", type=int, default=16)
    p.add_argument("--work_dir", type=str, default="./")
    p.add_argument("--momentum", type=float, default=0.999)
    p.add_argument("--weight_decay", type=float, default=0.000)
    p.add_argument("--lr", type=float, default=1e-4)
    p.add_argument("--epochs", type=int, default=300)
    p.add_argument("--dml", action="store_true", help="accepted for CLI compatibility; ignored")
    p.add_argument("--mean", action="store_true", help="accepted for CLI compatibility (the reference's "
                   "calculateNorm path crashes, SURVEY App. A); ImageNet statistics are used")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--L1_loss", action="store_true")
    p.add_argument("--rs_deep", type=int, default=16)
    p.add_argument("--shape", type=int, default=96)
    p.add_argument("--save_name", type=str, default="checkpoint")
    p.add_argument("--lr2", type=float, default=0.01)
    p.add_argument("--seed", type=int, default=100)
    p.add_argument("--add_rate", type=float, default=0.2)
    p.add_argument("--enchant", action="store_true")
    p.add_argument("--tpu", action="store_true", help="accepted for CLI compatibility; ignored")
    # additions
    p.add_argument("--data", type=str, default="", help="image directory or JSON list (default: ./train_images.json "
                   "if present, else synthetic)")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--synthetic_kind", default="smooth", choices=("smooth", "natural", "leaves"),
                   help="synthetic HR crops: smooth (bicubic noise), natural (1/f^1.4 Gaussian fields) or "
                        "leaves (dead-leaves images with a 1/f texture)")
    p.add_argument("--dist_backend", default="nccl", help="process-group backend for WORLD_SIZE > 1 "
                   "(nccl = RCCL; gloo only to rehearse several ranks sharing one GPU)")
    p.add_argument("--steps", type=int, default=0, help="iterations per epoch (0 = one pass over the data)")
    p.add_argument("--vgg_weights", type=str, default=None)
    p.add_argument("--dis_miopen", action="store_true", help="run the discriminator's conv stack on stock MIOpen "
                   "convs (NHWC + find mode) instead of libisr")
    opt = p.parse_args(argv)
    if not opt.data and Path("train_images.json").is_file():
        opt.data = "train_images.json"
    if opt.steps == 0:
        opt.steps = None
    return opt


if __name__ == "__main__":
    main(parse())
