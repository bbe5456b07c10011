"""Training loops of train.py (train.py:41-67 `train`, :70-129 `train_srgan`).

Same structure and optimiser semantics as the reference — Adam, LinearLR per
iteration, clip_grad_norm_(10), ModelEMA after every generator step — with
the generator forward/backward on the HIP training path (train_engine.py),
the VGG19 perceptual loss on HIP (vgg.py), and data arriving as uint8 crops
transformed on the GPU (data.py).

Differences, all deliberate:
* bf16 storage with fp32 accumulation and fp32 master weights replaces fp16
  autocast, so the GradScaler is disabled (bf16 has fp32's exponent range);
  the GradScaler objects are kept for checkpoint compatibility.
* the discriminator's conv stack runs on libisr (discriminator.py, bf16 storage,
  fp32 accumulation); its pool + Linear head under bf16 autocast where the
  reference uses fp16 autocast (train.py:91, :114).
* Adam (optim.FusedAdam, built by train.py), clip_grad_norm_ and the EMA update
  run as one HIP multi-tensor launch each (optim.py) instead of per-tensor loops.
* the discriminator's parameters are frozen during the generator-loss forward,
  so its discarded parameter gradients (train.py:102, zeroed at :119) are not computed.
* loss.item() host syncs happen once per `log_every` iterations instead of
  every iteration (train.py:64-65, :101-112).
* a forward whose persistent trunk kernel gave up (engine.ChainFailed, reported at the latest
  at epoch end) changes no parameter: every Adam / EMA update of that step and of later steps
  is skipped on the device (optim.step_guard) until the host has reported the failure.  Under
  data parallelism the guard is global (train_engine.step_guard_ptr: the give-up flags are
  summed over the ranks before the optimiser runs), so every rank skips together and every
  rank raises at epoch end.  What a skipped step still advances: the host-side counters
  (FusedAdam's per-parameter step used for bias correction, ModelEMA.updates, the LR
  schedules) and the discriminator's BatchNorm running statistics (its train-mode forwards ran
  on the invalid sr images).  ChainFailed means "this epoch's results are void": resume from
  the last checkpoint rather than from the in-memory state.
* multi-GPU (one process per GPU): the generator's gradients are averaged by
  one RCCL all-reduce of its flat gradient buffer inside the HIP backward
  (train_engine.enable_grad_allreduce); the discriminator's by one flat
  all-reduce after its backward (allreduce_grads).  Same math as DDP.
"""
from __future__ import annotations

import contextlib
import os
import time

import torch
from .models import ModelEMA
from .optim import clip_grad_norm_  # HIP multi-tensor clip (same signature as torch's)
from .optim import step_guard
from .train_engine import allreduce_grads, step_guard_ptr, trunk_done_event


def _scalar(writer, tag, value, step):
    if writer is not None:
        writer.add_scalar(tag, value, step)


def _unwrap(m):
    return m.module if hasattr(m, "module") else m


@contextlib.contextmanager
def _frozen(module):
    """requires_grad=False on `module`'s trainable parameters for the graphs built inside."""
    ps = [p for p in module.parameters() if p.requires_grad]
    for p in ps:
        p.requires_grad_(False)
    try:
        yield
    finally:
        for p in ps:
            p.requires_grad_(True)


def train(model, ema: ModelEMA, batches, transform, compute_loss, optimizer, gradscaler, schedule, epoch: int,
          tensorBoard=None, steps: int | None = None, log_every: int = 50):
    """train.py:41-67: one epoch of pixel-loss (MSE / L1Loss) generator training."""
    model.train()
    losses = []
    total = steps if steps is not None else len(batches)
    it = iter(batches)
    pending = []
    for idx in range(total):
        hr, lr = transform(next(it))
        optimizer.zero_grad(set_to_none=True)
        preds = model(lr)
        loss = compute_loss(preds, hr)
        gradscaler.scale(loss).backward()
        gradscaler.unscale_(optimizer)
        clip_grad_norm_(model.parameters(), 10)
        with step_guard(step_guard_ptr(_unwrap(model))):  # a failed trunk forward updates nothing
            gradscaler.step(optimizer)
            gradscaler.update()
            schedule.step()
            ema.update(_unwrap(model))
        pending.append(loss.detach())
        if len(pending) == log_every or idx == total - 1:
            vals = torch.stack(pending).cpu().tolist()
            for k, v in enumerate(vals):
                _scalar(tensorBoard, "loss", v, epoch * total + idx - len(vals) + k + 2)
            losses += vals
            pending = []
    _verify(model)
    return losses


def _verify(gen) -> None:
    """Epoch end: a persistent-chain give-up anywhere in the epoch raises here (engine.ChainFailed),
    before the caller logs the epoch or saves its checkpoint."""
    from .train_engine import verify_chains
    verify_chains(_unwrap(gen))


def train_srgan(gen_net, ema: ModelEMA, dis_net, batches, transform, compute_loss, optimizer_g, optimizer_d,
                gradscaler, schedules, epoch: int, tensorBoard=None, mean=None, std=None,
                steps: int | None = None, log_every: int = 50, dist_group=None):
    """train.py:70-129: one epoch of SRGAN training (VGG perceptual + adversarial)."""
    gen_net.train()
    dis_net.train()
    loss_g = []
    gradscaler_gen, gradscaler_dis = gradscaler
    schedule_g, schedule_d = schedules
    device = next(_unwrap(gen_net).parameters()).device
    mean = torch.tensor(mean, device=device).view(1, 3, 1, 1)
    std = torch.tensor(std, device=device).view(1, 3, 1, 1)
    total = steps if steps is not None else len(batches)
    it = iter(batches)
    pending = []
    # the discriminator's forwards + backward on a second stream beside the generator's backward
    # (same results, tests/test_gpu_train_cfg3.py; A/B: ISR_TRAIN_D_OVERLAP=0)
    # (not beside a persistent backward chain: its grid must own the chip, ISR_TRAIN_BWD_CHAIN)
    overlap = (os.environ.get("ISR_TRAIN_D_OVERLAP", "1") == "1"
               and os.environ.get("ISR_TRAIN_BWD_CHAIN", "0") != "1")
    hr_overlap = overlap and os.environ.get("ISR_TRAIN_HR_OVERLAP", "1") == "1"
    dsr_side = hr_overlap and os.environ.get("ISR_TRAIN_DSR_SIDE", "1") == "1"
    hr_early = hr_overlap and os.environ.get("ISR_TRAIN_HR_EARLY", "1") == "1"
    d_stream = torch.cuda.Stream(device) if overlap and device.type == "cuda" else None
    # test-only: the generator's clip / Adam / EMA enqueued before the discriminator step instead
    # of after it (a legal order: the two touch disjoint state; tests/test_gpu_dist_train.py)
    g_first = os.environ.get("ISR_TRAIN_G_FIRST", "0") == "1"
    for idx in range(total):
        hr_images, lr_images = transform(next(it))
        sr_images = gen_net(lr_images)
        _tap("sr", [sr_images])
        if TAPS is not None and sr_images.requires_grad:  # the generator's upstream gradient (tests)
            sr_images.register_hook(lambda g: _tap("sr_grad", [g]))
        sr_images = (sr_images + 1.0) / 2.0
        sr_images = (sr_images - mean) / std
        hr_features = None
        if d_stream is not None and hr_overlap:
            # VGG(hr) on the second stream beside the D(sr) and VGG(sr) forwards; enqueued after the
            # generator forward, whose persistent trunk grid must have the chip to itself
            g_done = torch.cuda.Event()
            g_done.record()
            # VGG(hr) needs only the trunk kernel to be done (not the upsampler / tail after it)
            t_done = trunk_done_event(_unwrap(gen_net)) if hr_early else None
            d_stream.wait_event(t_done if t_done is not None else g_done)
            with torch.cuda.stream(d_stream):
                with torch.no_grad():
                    hr_features = compute_loss.vgg_net(hr_images)
                if dsr_side:  # D(sr) too (VGG(sr) on the main stream beside both); its input-gradient
                    # backward then runs on this stream too, autograd joining the streams
                    d_stream.wait_event(g_done)
                    sr_discriminated = _d_frozen_forward(dis_net, sr_images)
        if hr_features is None or not dsr_side:
            sr_discriminated = _d_frozen_forward(dis_net, sr_images)
        if hr_features is not None:
            if dsr_side:
                sr_discriminated = _joined(sr_discriminated, d_stream)
            perceptual_loss, adversarial_loss_, content_loss = compute_loss.calc_contentLoss(
                sr_images, hr_images, sr_discriminated, hr_features=_joined(hr_features, d_stream))
        else:
            perceptual_loss, adversarial_loss_, content_loss = compute_loss.calc_contentLoss(sr_images, hr_images,
                                                                                             sr_discriminated)
        _tap("g_loss", [perceptual_loss, adversarial_loss_, content_loss])
        optimizer_g.zero_grad(set_to_none=True)
        if d_stream is not None:
            fwd_done = torch.cuda.Event()
            fwd_done.record()  # sr / hr and every forward the D step reads
        gradscaler_gen.scale(perceptual_loss).backward()
        _tap("g_grad", [p.grad for p in gen_net.parameters()])
        if d_stream is not None and not g_first:
            # the discriminator's forwards and backward on a second stream, beside the generator's
            # backward (they read neither its gradients nor anything it writes; D's weights change
            # only in D's optimiser step, after both)
            d_stream.wait_event(fwd_done)
            with torch.cuda.stream(d_stream):
                adversarial_loss = _d_forward_backward(dis_net, compute_loss, sr_images, hr_images, optimizer_d,
                                                       gradscaler_dis)
        gradscaler_gen.unscale_(optimizer_g)
        clip_grad_norm_(gen_net.parameters(), 10)
        _tap("g_grad_clipped", [p.grad for p in gen_net.parameters()])
        guard = step_guard_ptr(_unwrap(gen_net))  # a failed trunk forward updates neither G nor D
        with step_guard(guard):
            gradscaler_gen.step(optimizer_g)
            gradscaler_gen.update()
            schedule_g.step()
            ema.update(_unwrap(gen_net))
        _tap("g_param", list(gen_net.parameters()))
        if d_stream is not None and g_first:  # test-only order (ISR_TRAIN_G_FIRST=1)
            d_stream.wait_event(fwd_done)
            with torch.cuda.stream(d_stream):
                adversarial_loss = _d_forward_backward(dis_net, compute_loss, sr_images, hr_images, optimizer_d,
                                                       gradscaler_dis)

        if d_stream is not None:
            torch.cuda.current_stream().wait_stream(d_stream)
        else:
            adversarial_loss = _d_forward_backward(dis_net, compute_loss, sr_images, hr_images, optimizer_d,
                                                   gradscaler_dis)
        _tap("d_grad_local", [p.grad for p in dis_net.parameters()])
        if dist_group is not None:
            allreduce_grads(dis_net.parameters(), None if dist_group is True else dist_group)
        _tap("d_grad", [p.grad for p in dis_net.parameters()])
        gradscaler_dis.unscale_(optimizer_d)
        clip_grad_norm_(dis_net.parameters(), 10)
        with step_guard(guard):
            gradscaler_dis.step(optimizer_d)
            gradscaler_dis.update()
            schedule_d.step()
        _tap("d_param", list(dis_net.parameters()))
        pending.append(torch.stack([content_loss.detach(), adversarial_loss_.detach(), adversarial_loss.detach()]))
        if len(pending) == log_every or idx == total - 1:
            vals = torch.stack(pending).cpu().tolist()
            for k, (c, a, d) in enumerate(vals):
                step = epoch * total + idx - len(vals) + k + 2
                _scalar(tensorBoard, "loss/content", c, step)
                _scalar(tensorBoard, "loss/adv", a, step)
                _scalar(tensorBoard, "loss/dis", d, step)
                loss_g.append(c)
            pending = []
    _verify(gen_net)
    return loss_g


# Diagnostic taps (tests only): when TAPS is a list, train_srgan appends (name, step, [tensors])
# with every tensor cloned on the current stream at that point of the step's enqueue order — no
# host synchronisation, so the stream schedule being diagnosed stays as it is.
TAPS: list | None = None


def _tap(name: str, tensors) -> None:
    if TAPS is not None:
        TAPS.append((name, [None if t is None else t.detach().clone() for t in tensors]))


def _d_frozen_forward(dis_net, sr_images):
    """The reference computes the discriminator's parameter gradients from the generator loss and
    then discards them (optimizer_d.zero_grad, train.py:119); D's parameters are frozen for this
    forward so only its input gradient is computed — same parameter updates, one weight-gradient
    pass fewer."""
    with torch.autocast("cuda", dtype=torch.bfloat16), _frozen(dis_net):  # reference: fp16 autocast
        return dis_net(sr_images)


def _joined(t: torch.Tensor, side):
    """A callable handing `t` (made on stream `side`) to the current stream once side's work is done."""
    def get():
        cur = torch.cuda.current_stream()
        cur.wait_stream(side)
        t.record_stream(cur)
        return t
    return get


def _d_forward_backward(dis_net, compute_loss, sr_images, hr_images, optimizer_d, gradscaler_dis):
    """train.py:114-119 up to the discriminator's backward (its step follows in the caller)."""
    with torch.autocast("cuda", dtype=torch.bfloat16):
        sr_discriminated = dis_net(sr_images.detach())
        hr_discriminated = dis_net(hr_images)
    adversarial_loss = compute_loss.calc_advLoss(sr_discriminated, hr_discriminated)
    optimizer_d.zero_grad(set_to_none=True)
    gradscaler_dis.scale(adversarial_loss).backward()
    return adversarial_loss


class StepTimer:
    """Wall-clock per step with a device sync at the ends (for logs / bench)."""

    def __init__(self):
        self.t0 = None

    def __enter__(self):
        torch.cuda.synchronize()
        self.t0 = time.perf_counter()
        return self

    def __exit__(self, *a):
        torch.cuda.synchronize()
        self.dt = time.perf_counter() - self.t0
