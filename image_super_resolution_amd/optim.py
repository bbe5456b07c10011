"""Optimiser-side HIP kernels: Adam, clip_grad_norm_ and
the EMA update as one multi-tensor launch each over every parameter, instead of
the reference's per-tensor loops (train.py:57-60, :101-105, :116-119;
utils/models.py:31-40 ModelEMA.update).

* `FusedAdam` — drop-in for torch.optim.Adam (same constructor, param_groups,
  state keys 'step' / 'exp_avg' / 'exp_avg_sq', so LinearLR and checkpoints
  work unchanged); fp32 parameters on the GPU only.
* `clip_grad_norm_(params, max_norm)` — torch.nn.utils.clip_grad_norm_ (L2):
  per-chunk sums of squares → total norm and clip coefficient on the device →
  in-place scale; no host sync; returns the total norm as a 0-d device tensor.
* `ema_update_(ema_tensors, model_tensors, d)` — v = v*d + (1-d)*m.

Tensors must be dense (contiguous or channels_last) and share strides with
their grad / state; the kernels treat each as a flat run of numel floats.
"""
from __future__ import annotations

import contextlib
import ctypes
import math

import torch

from . import _lib, ops

CHUNK = 65536


def _dense(t: torch.Tensor) -> bool:
    return t.is_contiguous() or t.is_contiguous(memory_format=torch.channels_last)


class _Uploader:
    """Host → device upload of small int64 tables without a host sync: a ring of
    pinned staging slots copied with non_blocking=True into a ring of device
    slots (a pageable copy would block the host until the stream drains).  A
    slot is reused `slots` uploads later, after its copy event has completed."""

    def __init__(self, device, slots: int = 16, cap: int = 1 << 16):
        self.device, self.cap = device, cap
        self.host = [torch.empty(cap, dtype=torch.int64).pin_memory() for _ in range(slots)]
        self.dev = [torch.empty(cap, dtype=torch.int64, device=device) for _ in range(slots)]
        self.ev = [None] * slots
        self.i = 0

    def put(self, values: list[int]) -> torch.Tensor:
        n = len(values)
        if n > self.cap:
            return torch.tensor(values, dtype=torch.int64).to(self.device)
        k = self.i
        self.i = (self.i + 1) % len(self.host)
        if self.ev[k] is not None:
            self.ev[k].synchronize()
        self.host[k][:n] = torch.tensor(values, dtype=torch.int64)
        d = self.dev[k][:n]
        d.copy_(self.host[k][:n], non_blocking=True)
        e = torch.cuda.Event()
        e.record()
        self.ev[k] = e
        return d


_UPLOADERS: dict = {}


def _uploader(device) -> _Uploader:
    key = str(device)
    if key not in _UPLOADERS:
        _UPLOADERS[key] = _Uploader(device)
    return _UPLOADERS[key]


class _Tables:
    """isr_mt_tensor / isr_mt_chunk tables in device memory.  The chunk table
    depends only on the tensor sizes (cached); the pointer table is uploaded
    through the pinned ring whenever the pointers change (grads are new tensors
    every step under zero_grad(set_to_none=True))."""

    def __init__(self):
        self.chunks: dict[tuple, tuple[torch.Tensor, int]] = {}
        self.ptrs: dict[tuple, torch.Tensor] = {}

    def get(self, rows: list[tuple[int, int, int, int, int]], device) -> tuple[torch.Tensor, torch.Tensor, int]:
        sizes = tuple(r[4] for r in rows)
        ch = self.chunks.get(sizes)
        if ch is None:
            flat = []
            for ti, n in enumerate(sizes):
                for s in range(0, n, CHUNK):
                    flat += [ti | (min(CHUNK, n - s) << 32), s]
            ch = self.chunks[sizes] = (torch.tensor(flat, dtype=torch.int64).to(device), len(flat) // 2)
        key = tuple(rows)
        pt = self.ptrs.get(key)
        if pt is None:
            pt = _uploader(device).put([v for r in rows for v in r])
            if len(self.ptrs) >= 4:  # keep a few stable pointer sets (params / EMA) resident
                self.ptrs.pop(next(iter(self.ptrs)))
            self.ptrs[key] = pt = pt.clone()
        return pt, ch[0], ch[1]


def _check(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the fused optimiser runs on the MI355X HIP path only (got {t.device})")
    if t.dtype != torch.float32:
        raise TypeError(f"{what}: fp32 tensors only, got {t.dtype}")
    if not _dense(t):
        raise ValueError(f"{what}: tensor must be dense (contiguous or channels_last)")


# The trunk give-up guard of the step being applied (a device pointer to the trunk state's words
# [2] (sticky give-up count) and [3] (the count the host accepted), engine.ConvChain.guard_ptr),
# or None.  Set by the trainer around each step's optimiser / EMA updates (step_guard); the HIP
# Adam and EMA kernels then skip their update on the device when the two words differ.
_GUARD: list = [None]


@contextlib.contextmanager
def step_guard(ptr):
    """Guard every FusedAdam.step / ema_update_ enqueued inside with the trunk state at `ptr`
    (None: unguarded)."""
    prev, _GUARD[0] = _GUARD[0], ptr
    try:
        yield
    finally:
        _GUARD[0] = prev


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, maximize=False) as one HIP launch per
    parameter group and step (isr_mt_adam)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, **kw):
        if amsgrad or kw.get("maximize"):
            raise NotImplementedError("FusedAdam: amsgrad / maximize are not supported")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))
        self._cache = _Tables()

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            by_step: dict[float, list] = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                _check(p, "FusedAdam param")
                g = p.grad
                if g.is_sparse or g.dtype != p.dtype or g.stride() != p.stride():
                    raise ValueError("FusedAdam: grad must be dense fp32 with the parameter's strides")
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                p.__dict__["_isr_wv"] = p.__dict__.get("_isr_wv", 0) + 1  # raw-pointer write: no _version bump
                by_step.setdefault(float(st["step"]), []).append(
                    (p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), p.numel()))
            for t, rows in by_step.items():
                pt, ch, n = self._cache.get(rows, group["params"][0].device)
                if n == 0:
                    continue
                bc1 = 1.0 - b1 ** t
                a = _lib.IsrAdamArgs(step=-group["lr"] / bc1, beta1=b1, beta2=b2, eps=group["eps"],
                                     weight_decay=group["weight_decay"], bc2_sqrt=math.sqrt(1.0 - b2 ** t))
                _lib.check(lib.isr_mt_adam_guarded(pt.data_ptr(), ch.data_ptr(), n, ctypes.byref(a),
                                                   None, _GUARD[0], ops._stream()), "isr_mt_adam")
                ops.bump_param_epoch()  # packed-weight caches must repack (raw-pointer writes)
        return loss


_CLIP_CACHE = _Tables()


@torch.no_grad()
def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, error_if_nonfinite: bool = False,
                    foreach=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ (L2) on the HIP multi-tensor kernels."""
    if isinstance(parameters, torch.Tensor):
        parameters = [parameters]
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    if float(norm_type) != 2.0:
        raise NotImplementedError("clip_grad_norm_: only the L2 norm (the reference's) is fused")
    for g in grads:
        _check(g, "clip_grad_norm_ grad")
    lib = _lib.load()
    dev = grads[0].device
    rows = [(0, g.data_ptr(), 0, 0, g.numel()) for g in grads]
    pt, ch, n = _CLIP_CACHE.get(rows, dev)
    partial = torch.empty(n, dtype=torch.float32, device=dev)
    out = torch.empty(2, dtype=torch.float32, device=dev)
    s = ops._stream()
    _lib.check(lib.isr_mt_sumsq(pt.data_ptr(), ch.data_ptr(), n, partial.data_ptr(), s), "isr_mt_sumsq")
    _lib.check(lib.isr_clip_coef(partial.data_ptr(), n, float(max_norm), out.data_ptr(), s), "isr_clip_coef")
    _lib.check(lib.isr_mt_scale(pt.data_ptr(), ch.data_ptr(), n, out[1:].data_ptr(), s), "isr_mt_scale")
    if error_if_nonfinite and not torch.isfinite(out[0]).item():
        raise RuntimeError("clip_grad_norm_: the total norm of gradients is non-finite")
    return out[0]


_EMA_CACHE = _Tables()


@torch.no_grad()
def ema_update_(ema: list[torch.Tensor], model: list[torch.Tensor], d: float) -> None:
    """v = v*d + (1-d)*m for every pair (ModelEMA.update, utils/models.py:37-40)."""
    if not ema:
        return
    rows, keep = [], []
    for v, m in zip(ema, model):
        _check(v, "ema tensor")
        if m.dtype != v.dtype or m.stride() != v.stride() or m.numel() != v.numel():
            m = m.to(v.dtype).contiguous(memory_format=torch.channels_last if v.dim() == 4 and
                                         not v.is_contiguous() else torch.contiguous_format)
            keep.append(m)  # alive until the launch is enqueued (stream-ordered reuse after that)
        rows.append((v.data_ptr(), m.data_ptr(), 0, 0, v.numel()))
    pt, ch, n = _EMA_CACHE.get(rows, ema[0].device)
    _lib.check(_lib.load().isr_mt_lerp_guarded(pt.data_ptr(), ch.data_ptr(), n, float(d), _GUARD[0],
                                                ops._stream()), "isr_mt_lerp")
    ops.bump_param_epoch()
