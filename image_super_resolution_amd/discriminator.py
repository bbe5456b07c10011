"""SRGAN discriminator conv stack on libisr: the eight
3x3 conv blocks of `Discriminator` (utils/models.py:513-569) — ConvWithoutBN
3→64 + LeakyReLU(0.2), then Conv(+train-mode BatchNorm) + LeakyReLU(0.2) with
stride 2 on every second block — forward and backward, in train mode.  The
adaptive pool and the two Linear layers (≈0.6 GFLOP) stay torch ops.

Stride 2 on the stride-1 kernel, exactly (no zero taps beyond a 2x2 window):
  forward   out(y,x) = Σ W[dy][dx] in(2y+dy-1, 2x+dx-1)  is a conv over the
            PixelUnshuffle'd input (x_sub2 view: channel s*cin + c = in[c] at
            (2y'+a, 2x'+b), s = 2a+b) with phase-expanded weights
            W'[co][s*cin+c][ty][tx] = W[co][c][2ty+a-1][2tx+b-1] on taps {0,1}²;
  dgrad     dx(c, 2y'+a, 2x'+b) is a conv over dz with 4*cin outputs
            W''[4c+s][co][ty][tx] = W[co][c][dy][dx] on taps {1,2}²
            (a=0: ty=1↔dy=1; a=1: ty=2↔dy=0, ty=1↔dy=2), stored through the
            PixelShuffle(2) epilogue;
  wgrad     over the x_sub2 view on taps {0,1}² (isr_wgrad_desc.x_sub2 / taps),
            dW gathered from dW'.
The first layer's 3 input channels are zero-padded to 32 (the wgrad K tile).
Activations are bf16 channel-blocked (ops.ActBuffer), accumulation fp32, BN
statistics in double (isr_bn_*).
"""
from __future__ import annotations

import ctypes
import os as _os

import torch
from torch import nn

from . import ops
from ._lib import load as _load_lib
from .ops import ActBuffer, round_up

SLOPE = 0.2


def expand_fwd(w: torch.Tensor) -> torch.Tensor:
    """W [co][ci][3][3] → W' [co][4ci][3][3] for the x_sub2 conv on taps {0,1}²."""
    co, ci = w.shape[:2]
    out = torch.zeros(co, 4 * ci, 3, 3, device=w.device, dtype=torch.float32)
    # phase a: (ty, dy) pairs with dy = 2ty + a - 1 in [0, 2]
    pairs = {0: [(1, 1)], 1: [(0, 0), (1, 2)]}
    for a in (0, 1):
        for b in (0, 1):
            s = 2 * a + b
            for ty, dy in pairs[a]:
                for tx, dx in pairs[b]:
                    out[:, s * ci:(s + 1) * ci, ty, tx] = w[:, :, dy, dx]
    return out


def expand_dgrad(w: torch.Tensor) -> torch.Tensor:
    """W [co][ci][3][3] → W'' [4ci][co][3][3] (output channel 4c+s) on taps {1,2}²."""
    co, ci = w.shape[:2]
    out = torch.zeros(ci, 4, co, 3, 3, device=w.device, dtype=torch.float32)
    pairs = {0: [(1, 1)], 1: [(2, 0), (1, 2)]}  # (ty, dy)
    wt = w.transpose(0, 1)  # [ci][co][3][3]
    for a in (0, 1):
        for b in (0, 1):
            s = 2 * a + b
            for ty, dy in pairs[a]:
                for tx, dx in pairs[b]:
                    out[:, s, :, ty, tx] = wt[:, :, dy, dx]
    return out.reshape(4 * ci, co, 3, 3).contiguous()


def gather_wgrad(dwp: torch.Tensor, ci: int) -> torch.Tensor:
    """dW' [co][4ci][3][3] (wgrad over the unshuffled input) → dW [co][ci][3][3]."""
    co = dwp.shape[0]
    dw = torch.empty(co, ci, 3, 3, device=dwp.device, dtype=dwp.dtype)
    ty_a = {0: (0, 1), 1: (1, 0), 2: (1, 1)}  # dy → (ty, a)
    for dy in range(3):
        ty, a = ty_a[dy]
        for dx in range(3):
            tx, b = ty_a[dx]
            s = 2 * a + b
            dw[:, :, dy, dx] = dwp[:, s * ci:(s + 1) * ci, ty, tx]
    return dw


# ISR_DISC_REUSE=0: always recompute (A/B)
REUSE = _os.environ.get("ISR_DISC_REUSE", "1") == "1"


class _Layer:
    def __init__(self, block: nn.Module):
        conv = block.conv
        self.w, self.b = conv.weight, conv.bias
        self.bn = getattr(block, "bn", None)
        self.cin, self.cout = conv.in_channels, conv.out_channels
        self.stride = conv.stride[0]
        self.cin_p = 32 if self.cin < 32 else self.cin  # first layer: 3 → 32 zero-padded channels (wgrad K tile)
        self.fwd = self.bwd = None
        self.bn_state = None


class DiscriminatorPlan:
    """Fixed-geometry train-mode plan of the conv stack for input [n, 3, h, w]."""

    def __init__(self, dis: nn.Module, n: int, h: int, w: int, device):
        self.key = (n, h, w, str(device))
        self.device = dev = torch.device(device)
        self.layers = [_Layer(b) for b in dis.conv_blocks]
        L = self.layers
        if L[0].stride != 1 or any(l.bn is None for l in L[1:]) or L[0].bn is not None:
            raise NotImplementedError("DiscriminatorPlan expects the reference block layout")
        if any(l.cin_p % 16 or l.cout % 64 for l in L):
            raise NotImplementedError("DiscriminatorPlan: channel counts must be multiples of 64 (first input: 3)")
        f = 2 ** sum(l.stride == 2 for l in L)
        if h % f or w % f:
            raise ValueError(f"discriminator input {h}x{w} must be a multiple of {f} (its stride-2 stages)")
        self.lib = _load_lib()
        # grids: res[i] = output grid of layer i; inp grid = (h, w)
        res, hh, ww = [], h, w
        for l in L:
            hh, ww = hh // l.stride, ww // l.stride
            res.append((hh, ww))
        self.res = res
        ha = [round_up(r[0], ops.TILE_H) for r in res]
        wa = [round_up(r[1], ops.TILE_W) for r in res]

        def pad_of(i):  # buffer read as the input of layer i+1
            return 2 if i + 1 < len(L) and L[i + 1].stride == 2 else 1

        def slack(i, pad):  # rows/cols a stride-2 consumer (layer i+1) reads
            if i + 1 < len(L) and L[i + 1].stride == 2:
                return 2 * ha[i + 1] + 2 * pad, 2 * wa[i + 1] + 2 * pad
            return 0, 0

        self.xin = ActBuffer.alloc(n, h, w, L[0].cin_p, 1, dev)
        self.A, self.Z, self.gA, self.dZ = [], [], [], []
        for i, l in enumerate(L):
            p = pad_of(i)
            mh, mw = slack(i, p)
            self.A.append(ActBuffer.alloc(n, *res[i], l.cout, p, dev, ha=ha[i], wa=wa[i], min_hp=mh, min_wp=mw))
            self.Z.append(ActBuffer.alloc(n, *res[i], l.cout, 0, dev, ha=ha[i], wa=wa[i]) if l.bn is not None else None)
            # gradient wrt this layer's BN output (masked by LeakyReLU'); a stride-2 layer i+1 writes it
            # through the PixelShuffle epilogue over 2*ha[i+1] rows; the first layer's is a conv input
            gh, gwd = slack(i, 1)
            self.gA.append(ActBuffer.alloc(n, *res[i], l.cout, 1, dev, ha=ha[i], wa=wa[i], min_hp=gh, min_wp=gwd))
            self.dZ.append(ActBuffer.alloc(n, *res[i], l.cout, 1, dev, ha=ha[i], wa=wa[i]) if l.bn is not None
                           else None)
            if l.bn is not None:
                l.bn_state = ops.BNState(l.cout, dev)
        self.gin = ActBuffer.alloc(n, h, w, 32, 0, dev)  # layer-0 input gradient (3 of 32 channels used)
        self.feat_shape = (n, L[-1].cout, *res[-1])
        self.busy = False
        self.pack()

    # ----------------------------------------------------------------- weights
    def params(self) -> list[torch.Tensor]:
        out = []
        for l in self.layers:
            out.append(l.w)
            if l.b is not None:
                out.append(l.b)
            if l.bn is not None:
                out += [l.bn.weight, l.bn.bias]
        return out

    def pack(self) -> None:
        # repack only when a weight changed since this plan's last pack (an SRGAN step runs three
        # forwards on the same weights); HIP optimiser writes bump ops.param_write_epoch
        key = (ops.param_write_epoch(),) + tuple((l.w.data_ptr(), l.w._version) for l in self.layers)
        if key == getattr(self, "_pack_key", None):
            return
        self._pack_key = key
        for l in self.layers:
            w = l.w.detach().float()
            if l.cin_p != l.cin:
                w = torch.nn.functional.pad(w, (0, 0, 0, 0, 0, l.cin_p - l.cin))
            if l.stride == 2:
                l.fwd = ops.pack_conv3x3(expand_fwd(w), out=l.fwd)
                l.bwd = ops.pack_conv3x3(expand_dgrad(w), out=l.bwd)
            else:
                l.fwd = ops.pack_conv3x3(w, out=l.fwd)
                wb = w if l.cin_p % 32 == 0 else torch.nn.functional.pad(w, (0, 0, 0, 0, 0, 32 - l.cin_p % 32))
                l.bwd = ops.pack_conv3x3_dgrad(wb, out=l.bwd)

    # ----------------------------------------------------------------- forward
    def _input_key(self, x: torch.Tensor):
        """Identity of this forward's input and weights: the same storage (held by the plan, so
        its address cannot be reused meanwhile), view, version counter and the same parameter
        versions (torch optimisers bump _version; the HIP optimisers bump `_isr_wv`)."""
        return ((x.untyped_storage().data_ptr(), x.storage_offset(), tuple(x.shape), x.stride(), x._version,
                 x.dtype)
                + tuple((p.data_ptr(), p._version, p.__dict__.get("_isr_wv", 0)) for p in self.params()))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x [n, 3, h, w] fp32 → conv-stack features [n, C, h/16, w/16] fp32 (BN in train mode).

        A forward of the same input with unchanged weights right after this plan's previous one
        (SRGAN: the discriminator step's D(sr.detach()) repeats the generator step's D(sr),
        train.py:104 / :126, with D not yet updated) reuses the stored activations: only the
        BatchNorm running-statistics update of each layer is replayed, from the forward's own
        batch sums (bit-identical to recomputing)."""
        key = self._input_key(x) if REUSE else None
        if key is not None and key == getattr(self, "_fwd_key", None):
            for l, d in zip(self.layers, self._bn_descs):
                if l.bn is not None:
                    l.bn_state.acc.copy_(l.fwd_acc)
                    ops.check(ops._lib.load().isr_bn_finalize(ctypes.byref(d), ops._stream()), "isr_bn_finalize")
                    if l.bn.num_batches_tracked is not None:
                        l.bn.num_batches_tracked.add_(1)
            return ops.blocked_to_nchw(self.A[-1], torch.empty(self.feat_shape, device=self.device))
        self._fwd_key, self._fwd_x = key, (x.untyped_storage() if key is not None else None)
        self._bn_descs = []
        ops.nchw_to_blocked(x.float().contiguous(), self.xin)
        prev = self.xin
        for i, l in enumerate(self.layers):
            bias = l.b.detach() if l.b is not None else None
            y = self.A[i] if l.bn is None else self.Z[i]
            if l.stride == 2:
                ops.conv3x3(prev, 4 * l.cin, l.fwd, bias, l.cout, y, slope=1.0 if l.bn is not None else SLOPE,
                            x_sub2=True, taps=1)
            else:
                ops.conv3x3(prev, l.cin_p, l.fwd, bias, l.cout, y, slope=1.0 if l.bn is not None else SLOPE)
            d = None
            if l.bn is not None:
                d = ops.bn_desc(self.Z[i], self.A[i], l.cout, l.bn_state, l.bn, slope=SLOPE)
                ops.bn_forward(d, l.bn_state)
                if REUSE:
                    if getattr(l, "fwd_acc", None) is None:
                        l.fwd_acc = torch.empty_like(l.bn_state.acc)
                    l.fwd_acc.copy_(l.bn_state.acc)  # this batch's sums, for a replayed running update
                if l.bn.num_batches_tracked is not None:
                    l.bn.num_batches_tracked.add_(1)
            self._bn_descs.append(d)
            prev = self.A[i]
        return ops.blocked_to_nchw(self.A[-1], torch.empty(self.feat_shape, device=self.device))

    # ----------------------------------------------------------------- backward
    def _wgrad(self, x: ActBuffer, cin: int, g: ActBuffer, cout: int, dw: torch.Tensor, db) -> None:
        ops.launch_wgrad3x3(ops.wgrad3x3_desc(x, cin, g, cout, dw, db), self.device)

    def backward(self, gfeat: torch.Tensor, need_input_grad: bool,
                 need_param_grads: bool = True) -> tuple[torch.Tensor | None, list]:
        """Input gradient and parameter gradients (all None when `need_param_grads`
        is False: the weight-gradient convs are skipped, only dgrad runs)."""
        L = self.layers
        last = len(L) - 1
        # gradient wrt the last activation → wrt its BN output (LeakyReLU')
        ops.nchw_to_blocked(gfeat.float().contiguous(), self.gA[last], m=self.A[last], mslope=SLOPE)
        grads: dict[int, list] = {}
        for i in range(last, -1, -1):
            l = L[i]
            gw = []
            g = self.gA[i]
            if l.bn is not None:
                dgam = torch.empty(l.cout, device=self.device)
                dbet = torch.empty(l.cout, device=self.device)
                ops.bn_backward(ops.bn_desc(self.Z[i], g, l.cout, l.bn_state, l.bn, dz=self.dZ[i], dgamma=dgam,
                                            dbeta=dbet, update_running=False), l.bn_state)
                g = self.dZ[i]
            xin = self.A[i - 1] if i > 0 else self.xin
            # weight (+ bias) gradient
            if not need_param_grads:
                gw = [None] * (2 if l.b is not None else 1)
            elif l.stride == 2:  # phase-decomposed: x read through the x_sub2 view, taps {0,1}^2
                dwp = torch.empty(l.cout, 4 * l.cin, 3, 3, device=self.device)
                ops.launch_wgrad3x3(ops.wgrad3x3_desc(xin, 4 * l.cin, g, l.cout, dwp, None, x_sub2=True, taps=1),
                                    self.device)
                gw.append(gather_wgrad(dwp, l.cin))
            else:
                dw = torch.empty(l.cout, l.cin_p, 3, 3, device=self.device)
                db = torch.empty(l.cout, device=self.device) if l.b is not None else None
                self._wgrad(xin, l.cin_p, g, l.cout, dw, db)
                gw.append(dw[:, :l.cin].contiguous() if l.cin_p != l.cin else dw)
                if db is not None:
                    gw.append(db)
            if l.bn is not None:
                gw += [dgam, dbet] if need_param_grads else [None, None]
            grads[i] = gw
            # input gradient
            if i > 0:
                if l.stride == 2:
                    ops.conv3x3(g, l.cout, l.bwd, None, 4 * l.cin, self.gA[i - 1], slope=1.0, shuffle=2, taps=2,
                                m=self.A[i - 1], mslope=SLOPE)
                else:
                    ops.conv3x3(g, l.cout, l.bwd, None, l.cin, self.gA[i - 1], m=self.A[i - 1], mslope=SLOPE)
        dx = None
        if need_input_grad:
            l = L[0]
            ops.conv3x3(self.gA[0], l.cout, l.bwd, None, 32, self.gin, slope=1.0)
            dx = torch.empty(self.feat_shape[0], 3, self.xin.h, self.xin.w, device=self.device)
            ops.blocked_to_nchw(self.gin, dx)
        out = []
        for i in range(len(L)):
            out += grads[i]
        return dx, out


class _Lease:
    """Holds a plan (its saved activations) until the backward ran or the graph died."""

    def __init__(self, plan: DiscriminatorPlan):
        self.plan = plan
        plan.busy = True

    def release(self):
        if self.plan is not None:
            self.plan.busy = False
            self.plan = None

    def __del__(self):
        self.release()


class _DiscFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan, *params):
        out = plan.forward(x)
        ctx.lease = _Lease(plan)
        return out

    @staticmethod
    def backward(ctx, gfeat):
        plan = ctx.lease.plan
        dx, grads = plan.backward(gfeat.contiguous(), ctx.needs_input_grad[0], any(ctx.needs_input_grad[2:]))
        # the plan's buffers (activations, BN accumulators, gradient buffers) are in use until this
        # backward's kernels finish on this stream: a call on another stream waits for this event
        plan.done_event = torch.cuda.Event()
        plan.done_event.record()
        plan.done_stream = torch.cuda.current_stream()
        ctx.lease.release()
        return (dx, None, *grads)


def conv_stack_train(dis: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Differentiable train-mode conv stack of the discriminator on libisr.  Each
    call whose graph is still alive holds its own plan (SRGAN runs D(sr.detach())
    and D(hr) before one backward), so plans are pooled per input geometry."""
    n, _, h, w = x.shape
    key = (n, h, w, str(x.device))
    pool = dis.__dict__.setdefault("_isr_plans", {})
    plans = pool.setdefault(key, [])
    # prefer an idle plan whose stored forward this call repeats (see DiscriminatorPlan.forward)
    plan = None
    if REUSE and len(plans) > 1:
        plan = next((p for p in plans if not p.busy and getattr(p, "_fwd_key", None) is not None
                     and p._fwd_key == p._input_key(x)), None)
    if plan is None:
        plan = next((p for p in plans if not p.busy), None)
    if plan is None:
        if len(plans) >= 8:
            raise RuntimeError("discriminator: more than 8 live forward graphs")
        plan = DiscriminatorPlan(dis, n, h, w, x.device)
        plans.append(plan)
    ev = getattr(plan, "done_event", None)
    if ev is not None and getattr(plan, "done_stream", None) != torch.cuda.current_stream():
        torch.cuda.current_stream().wait_event(ev)  # an earlier backward on another stream used it
    plan.pack()
    with torch.autocast("cuda", enabled=False):
        if not (torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in plan.params()))):
            return plan.forward(x.float())
        return _DiscFn.apply(x.float(), plan, *plan.params())
