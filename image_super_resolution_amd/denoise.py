"""Denoise network (utils/models.py:672-706) on libisr — inference and training.

The denoiser `train.py --train_denoise` builds (train.py:204-205) and whose
older variant ships as the reference's model.pt.  Same-resolution image in,
same-resolution tanh image out, with one half-resolution 256-channel stage:

  head9x9   conv0: 9x9 3→64 + LeakyReLU(0.2)                       → F
  residual_0: R/2 x ResidualBlock1(64) (:202-209), each
    conv3x3 64→64 (+folded BN) + LeakyReLU(0.2)                    → H
    conv3x3 64→64 (+folded BN), + block input in the epilogue      → A / B
  residual_conv0: ConvWithoutBN(64, 256, 3, stride 2) + LeakyReLU(0.2)
    = conv3x3 over the x_sub2 (PixelUnshuffle) view, phase-expanded
      weights on taps {0,1}^2 (the discriminator's stride-2 form)   → Q (H/2 x W/2)
  residual_1: 2 x ResidualBlock1(256) at half resolution           → Q
  residual_conv1: PixelShuffle(2) + LeakyReLU(0.2)  (isr_pixel_shuffle2: the
    block's residual add precedes the shuffle, so it is its own pass) → A / B
  residual_2: R/2 x ResidualBlock1(64)
  conv1: Conv 64→64 (+folded BN), + F in the epilogue (:704)        → T
  tail9x9   conv2: 9x9 64→3 + tanh                                 → NCHW fp32

Inputs must have even height and width: the reference's `inputs +
conv1(residual)` (:704) only type-checks when the stride-2 conv and the
PixelShuffle restore the input size.  BN is folded at pack time
(fuse_conv_and_bn, :366-406), i.e. eval-mode semantics.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import torch

from . import ops
from .discriminator import expand_fwd
from .engine import PackedConv, _fold, _pack3
from .ops import ActBuffer, round_up

SLOPE = 0.2  # every activation of Denoise is LeakyReLU(0.2) (utils/models.py:676-690)


@dataclass
class DenoiseWeights:
    head: PackedConv
    res0: list[tuple[PackedConv, PackedConv]]
    down: PackedConv          # residual_conv0, phase-expanded (cin = 4 * 64)
    res1: list[tuple[PackedConv, PackedConv]]
    res2: list[tuple[PackedConv, PackedConv]]
    conv1: PackedConv
    tail: PackedConv
    buffers: dict = field(default_factory=dict)


def _count(sd: dict, prefix: str) -> int:
    return len({int(k[len(prefix):].split(".")[0]) for k in sd if k.startswith(prefix)})


def pack_denoise(sd: dict, prefix: str = "", device="cuda") -> DenoiseWeights:
    """Pack a Denoise state_dict (reference key schema, BN fused or not)."""
    p = prefix

    def blocks(name):
        return [(_pack3(sd, f"{p}{name}.{i}.m.0", device), _pack3(sd, f"{p}{name}.{i}.m.1", device))
                for i in range(_count(sd, f"{p}{name}."))]

    w0, b0 = _fold(sd, f"{p}conv0.0", device)
    head = PackedConv(ops.pack_head9x9(w0), b0, 3, 64)
    wd, bd = _fold(sd, f"{p}residual_conv0", device)
    if tuple(wd.shape) != (256, 64, 3, 3):
        raise NotImplementedError(f"Denoise.residual_conv0 weight {tuple(wd.shape)} != (256, 64, 3, 3)")
    down = PackedConv(ops.pack_conv3x3(expand_fwd(wd)), bd, 4 * 64, 256)
    w2, b2 = _fold(sd, f"{p}conv2.0", device)
    tail = PackedConv(ops.pack_tail9x9(w2), b2, 64, 3)
    return DenoiseWeights(head, blocks("residual_0"), down, blocks("residual_1"), blocks("residual_2"),
                          _pack3(sd, f"{p}conv1", device), tail)


class DenoisePlan:
    """Pre-built launch list of one Denoise forward for a fixed [n, 3, h, w] fp32 input."""

    def __init__(self, dw: DenoiseWeights, n: int, h: int, w: int, device):
        if h % 2 or w % 2:
            raise ValueError(f"Denoise needs an even input size (stride-2 conv + PixelShuffle(2) restore it), "
                             f"got {h}x{w}")
        self.key = (n, h, w, str(device))
        lib = ops._lib.load()
        h2, w2 = h // 2, w // 2
        ha2, wa2 = round_up(h2, ops.TILE_H), round_up(w2, ops.TILE_W)
        # full-resolution 64-channel buffers read by the stride-2 conv need pad 2 and
        # 2*ha2 + 4 rows / 2*wa2 + 4 columns (its x_sub2 view spans the half grid's
        # computed region); all three candidates (F, A, B) get that geometry
        sub = dict(min_hp=2 * ha2 + 4, min_wp=2 * wa2 + 4)
        F, A, B = (ActBuffer.alloc(n, h, w, 64, 2, device, **sub) for _ in range(3))
        H = ActBuffer.alloc(n, h, w, 64, 1, device)
        Q0, Q1, QH = (ActBuffer.alloc(n, h2, w2, 256, 1, device, ha=ha2, wa=wa2) for _ in range(3))
        T = ActBuffer.alloc(n, h, w, 64, 4, device)
        self.bufs = (F, A, B, H, Q0, Q1, QH, T)
        self.out_shape = (n, 3, h, w)
        dummy_x = torch.empty((n, 3, h, w), dtype=torch.float32, device=device)
        dummy_out = torch.empty(self.out_shape, dtype=torch.float32, device=device)
        self._keep = (dummy_x, dummy_out)

        conv = lib.isr_conv3x3_fwd
        L = []
        self.head_desc = ops.head9x9_desc(dummy_x, dw.head.w, dw.head.b, F, slope=SLOPE)
        L.append((lib.isr_head9x9_fwd, self.head_desc))

        def c3(src, pc, dst, **kw):
            L.append((conv, ops.conv3x3_desc(src, pc.cin, pc.w, pc.b, pc.cout, dst, **kw)))

        def res_chain(blocks, cur, pool, hidden):
            """ResidualBlock1 x len(blocks): out = x + Conv(act=False)(Conv(act=LReLU)(x))."""
            for m0, m1 in blocks:
                nxt = pool[0] if pool[0] is not cur else pool[1]
                c3(cur, m0, hidden, slope=SLOPE)
                c3(hidden, m1, nxt, slope=1.0, r1=cur, s1=1.0)
                cur = nxt
            return cur

        cur = res_chain(dw.res0, F, (A, B), H)
        c3(cur, dw.down, Q0, slope=SLOPE, x_sub2=True, taps=1)
        q = res_chain(dw.res1, Q0, (Q1, Q0), QH)
        s_out = A if cur is not A else B  # any full-resolution buffer but F
        L.append((lib.isr_pixel_shuffle2, ops.pixel_shuffle2_desc(s_out, q, 64, slope=SLOPE)))
        cur = res_chain(dw.res2, s_out, (A, B) if s_out is A else (B, A), H)
        c3(cur, dw.conv1, T, slope=1.0, r1=F, s1=1.0)
        self.tail_desc = ops.tail9x9_desc(T, dw.tail.w, dw.tail.b, dummy_out)
        L.append((lib.isr_tail9x9_fwd, self.tail_desc))
        self.launches = L

    def run(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        if tuple(x.shape) != self.out_shape or x.dtype != torch.float32 or not x.is_contiguous():
            raise ValueError("DenoisePlan.run: input does not match the plan")
        if tuple(out.shape) != self.out_shape or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("DenoisePlan.run: output does not match the plan")
        self.head_desc.x = x.data_ptr()
        self.tail_desc.y = out.data_ptr()
        stream = ops._stream()
        for fn, d in self.launches:
            ops.check(fn(ctypes.byref(d), stream), fn.__name__)
        return out


def run_denoise(dw: DenoiseWeights, x: torch.Tensor) -> torch.Tensor:
    """x: NCHW [n, 3, h, w] fp32 (h, w even) on the GPU → tanh image [n, 3, h, w] fp32."""
    if x.dim() != 4 or x.shape[1] != 3:
        raise ValueError(f"Denoise expects [n, 3, h, w], got {tuple(x.shape)}")
    x = x.float().contiguous()
    n, _, h, w = x.shape
    key = (n, h, w, str(x.device))
    plan = dw.buffers.get("plan")
    if plan is None or plan.key != key:
        dw.buffers["plan"] = None
        plan = dw.buffers["plan"] = DenoisePlan(dw, n, h, w, x.device)
    return plan.run(x, torch.empty(plan.out_shape, dtype=torch.float32, device=x.device))


# ===================================================================== training
class _TLayer:
    """One conv of the Denoise network in training: parameter refs + packed copies."""

    def __init__(self, conv_mod, kind: str):
        self.mod = conv_mod                      # reference Conv / ConvWithoutBN
        self.w = conv_mod.conv.weight
        self.b = conv_mod.conv.bias
        bn = getattr(conv_mod, "bn", None)
        self.bn = bn if isinstance(bn, torch.nn.BatchNorm2d) else None
        self.kind = kind                         # "3x3", "s2" (stride 2), "head", "tail"
        self.cout, self.cin = self.w.shape[:2]
        self.fwd = self.bwd = None
        self.bn_state = None

    def params(self) -> list[torch.Tensor]:
        out = [self.w] + ([self.b] if self.b is not None else [])
        return out + ([self.bn.weight, self.bn.bias] if self.bn is not None else [])

    def pack(self) -> None:
        w = self.w.detach().float()
        if self.kind == "3x3":
            self.fwd = ops.pack_conv3x3(w, out=self.fwd)
            self.bwd = ops.pack_conv3x3_dgrad(w, out=self.bwd)
        elif self.kind == "s2":
            from .discriminator import expand_dgrad
            self.fwd = ops.pack_conv3x3(expand_fwd(w), out=self.fwd)
            self.bwd = ops.pack_conv3x3(expand_dgrad(w), out=self.bwd)
        elif self.kind == "head":
            self.fwd = ops.pack_head9x9(w, out=self.fwd)
        else:  # tail: its input gradient is a head9x9 conv with 180°-rotated, transposed weights
            self.fwd = ops.pack_tail9x9(w, out=self.fwd)
            self.bwd = ops.pack_head9x9(w.flip(2, 3).transpose(0, 1).contiguous(), out=self.bwd)


class _TBlock:
    """ResidualBlock1 (utils/models.py:202-209) with its saved activations."""

    def __init__(self, blk, n, h, w, c, dev, ha, wa, out_sub: dict):
        self.a, self.b = _TLayer(blk.m[0], "3x3"), _TLayer(blk.m[1], "3x3")
        self.Za = ActBuffer.alloc(n, h, w, c, 0, dev, ha=ha, wa=wa)
        self.Ha = ActBuffer.alloc(n, h, w, c, 1, dev, ha=ha, wa=wa)
        self.Zb = ActBuffer.alloc(n, h, w, c, 0, dev, ha=ha, wa=wa)
        self.Y = ActBuffer.alloc(n, h, w, c, 2 if out_sub else 1, dev, ha=ha, wa=wa, **out_sub)
        for l in (self.a, self.b):
            if l.bn is None:
                raise NotImplementedError("ResidualBlock1 training expects Conv layers with BatchNorm (unfused)")
            l.bn_state = ops.BNState(c, dev)


class DenoiseTrainPlan:
    """Train-mode forward (BatchNorm on batch statistics, running stats updated) and
    backward of Denoise on libisr for a fixed [n, 3, h, w] input.

    Backward per ResidualBlock1 (reverse): BN_b backward on the block-output
    gradient, wgrad(Ha), dgrad with LeakyReLU'(Ha) in the epilogue, BN_a backward,
    wgrad(X), dgrad + the skip gradient (r1) → the block-input gradient.  The
    stride-2 conv: wgrad over the x_sub2 view (taps {0,1}²) gathered to 3x3, dgrad
    as the 2x2-tap conv with the PixelShuffle store (discriminator.py); the
    PixelShuffle + LeakyReLU: isr_pixel_unshuffle2 with the LeakyReLU' mask;
    the tail: tanh' then wgrad9x9 and a head9x9 dgrad; the head: wgrad9x9 on the
    masked trunk gradient (ew_combine of chain + trunk)."""

    def __init__(self, model, n: int, h: int, w: int, device):
        if h % 2 or w % 2:
            raise ValueError(f"Denoise needs an even input size, got {h}x{w}")
        dev = self.device = torch.device(device)
        self.key = (n, h, w, str(dev))
        self.busy = False
        self.grad_group = None
        h2, w2 = h // 2, w // 2
        ha2, wa2 = round_up(h2, ops.TILE_H), round_up(w2, ops.TILE_W)
        sub = dict(min_hp=2 * ha2 + 4, min_wp=2 * wa2 + 4)
        self.head = _TLayer(model.conv0[0], "head")
        self.down = _TLayer(model.residual_conv0, "s2")
        self.conv1 = _TLayer(model.conv1, "3x3")
        self.tail = _TLayer(model.conv2[0], "tail")
        if self.conv1.bn is None:
            raise NotImplementedError("Denoise training expects an unfused model (Conv layers with BatchNorm)")
        self.conv1.bn_state = ops.BNState(64, dev)
        self.F = ActBuffer.alloc(n, h, w, 64, 2, dev, **sub)
        self.res0 = [_TBlock(b, n, h, w, 64, dev, None, None, sub) for b in model.residual_0]
        self.Q0 = ActBuffer.alloc(n, h2, w2, 256, 1, dev, ha=ha2, wa=wa2)
        self.res1 = [_TBlock(b, n, h2, w2, 256, dev, ha2, wa2, {}) for b in model.residual_1]
        self.S = ActBuffer.alloc(n, h, w, 64, 1, dev, min_hp=2 * ha2 + 2, min_wp=2 * wa2 + 2)  # unshuffle mask
        self.res2 = [_TBlock(b, n, h, w, 64, dev, None, None, {}) for b in model.residual_2]
        self.Z1 = ActBuffer.alloc(n, h, w, 64, 0, dev)
        self.T = ActBuffer.alloc(n, h, w, 64, 4, dev)
        # gradient scratch: full resolution (slack for the stride-2 dgrad's shuffled store) and half
        self.gf = [ActBuffer.alloc(n, h, w, 64, 1, dev, min_hp=2 * ha2 + 2, min_wp=2 * wa2 + 2) for _ in range(5)]
        self.gq = [ActBuffer.alloc(n, h2, w2, 256, 1, dev, ha=ha2, wa=wa2) for _ in range(4)]
        self.out_shape = (n, 3, h, w)
        self.layers = ([self.head] + [l for b in self.res0 for l in (b.a, b.b)] + [self.down]
                       + [l for b in self.res1 for l in (b.a, b.b)] + [l for b in self.res2 for l in (b.a, b.b)]
                       + [self.conv1, self.tail])
        self.x = self.y = None

    def params(self) -> list[torch.Tensor]:
        return [p for l in self.layers for p in l.params()]

    def pack(self) -> None:
        for l in self.layers:
            l.pack()

    # ----------------------------------------------------------------- forward
    @staticmethod
    def _bn_fwd(l: _TLayer, z: ActBuffer, y: ActBuffer, c: int, **kw) -> None:
        ops.bn_forward(ops.bn_desc(z, y, c, l.bn_state, l.bn, **kw), l.bn_state)
        if l.bn.num_batches_tracked is not None:
            l.bn.num_batches_tracked.add_(1)

    def _chain_fwd(self, blocks, x: ActBuffer, c: int) -> ActBuffer:
        for b in blocks:
            ops.conv3x3(x, c, b.a.fwd, None, c, b.Za, slope=1.0)
            self._bn_fwd(b.a, b.Za, b.Ha, c, slope=SLOPE)
            ops.conv3x3(b.Ha, c, b.b.fwd, None, c, b.Zb, slope=1.0)
            self._bn_fwd(b.b, b.Zb, b.Y, c, slope=1.0, r1=x, s1=1.0)
            x = b.Y
        return x

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        self.x = x = x.float().contiguous()
        ops.head9x9(x, self.head.fwd, self.head.b.detach(), self.F, slope=SLOPE)
        self.x_last0 = self._chain_fwd(self.res0, self.F, 64)
        ops.conv3x3(self.x_last0, 256, self.down.fwd, self.down.b.detach(), 256, self.Q0, slope=SLOPE,
                    x_sub2=True, taps=1)
        self.q_last = self._chain_fwd(self.res1, self.Q0, 256)
        ops.pixel_shuffle2(self.S, self.q_last, 64, slope=SLOPE)
        self.r_last = self._chain_fwd(self.res2, self.S, 64)
        ops.conv3x3(self.r_last, 64, self.conv1.fwd, None, 64, self.Z1, slope=1.0)
        self._bn_fwd(self.conv1, self.Z1, self.T, 64, slope=1.0, r1=self.F, s1=1.0)
        y = torch.empty(self.out_shape, device=self.device)
        ops.tail9x9(self.T, self.tail.fwd, self.tail.b.detach(), y)
        self.y = y
        return y

    # ----------------------------------------------------------------- backward
    def _bn_bwd(self, l: _TLayer, z: ActBuffer, g: ActBuffer, dz: ActBuffer, c: int, grads: dict) -> None:
        dgam = torch.empty(c, device=self.device)
        dbet = torch.empty(c, device=self.device)
        ops.bn_backward(ops.bn_desc(z, g, c, l.bn_state, l.bn, dz=dz, dgamma=dgam, dbeta=dbet,
                                    update_running=False), l.bn_state)
        grads[id(l.bn.weight)], grads[id(l.bn.bias)] = dgam, dbet

    def _wgrad(self, l: _TLayer, x: ActBuffer, g: ActBuffer, grads: dict) -> None:
        dw = torch.empty(l.cout, l.cin, 3, 3, device=self.device)
        ops.wgrad3x3(x, l.cin, g, l.cout, dw, None)
        grads[id(l.w)] = dw

    def _chain_bwd(self, blocks, x_in: ActBuffer, g: ActBuffer, pool: list, c: int, grads: dict,
                   m_in: ActBuffer | None = None) -> ActBuffer:
        """Reverse through a ResidualBlock1 chain; g = gradient wrt the chain output.
        Returns the gradient wrt the chain input (times LeakyReLU'(m_in) when given).
        `pool` holds four scratch buffers of the chain's grid (g may be one of them)."""
        for i in range(len(blocks) - 1, -1, -1):
            b = blocks[i]
            xi = blocks[i - 1].Y if i > 0 else x_in
            dz, gh, gin = [p for p in pool if p is not g][:3]
            self._bn_bwd(b.b, b.Zb, g, dz, c, grads)
            self._wgrad(b.b, b.Ha, dz, grads)
            ops.conv3x3(dz, c, b.b.bwd, None, c, gh, slope=1.0, m=b.Ha, mslope=SLOPE)
            self._bn_bwd(b.a, b.Za, gh, dz, c, grads)
            self._wgrad(b.a, xi, dz, grads)
            mk = dict(m=m_in, mslope=SLOPE) if (i == 0 and m_in is not None) else {}
            ops.conv3x3(dz, c, b.a.bwd, None, c, gin, slope=1.0, r1=g, s1=1.0, **mk)
            g = gin
        if not blocks and m_in is not None:
            raise NotImplementedError("masked chain input needs at least one block")
        return g

    def backward(self, gy: torch.Tensor) -> dict:
        from .discriminator import gather_wgrad
        dev = self.device
        grads: dict = {}
        gp = (gy.float() * (1.0 - self.y * self.y)).contiguous()  # tanh' (utils/models.py:692, act=nn.Tanh())
        # tail (conv2): weight / bias gradient, input gradient by the head kernel
        dw2 = torch.empty(3, 64, 9, 9, device=dev)
        db2 = torch.empty(3, device=dev)
        ops.wgrad9x9(gp, self.T, dw2, db2, head=False)
        grads[id(self.tail.w)], grads[id(self.tail.b)] = dw2, db2
        gT, pool = self.gf[4], self.gf[:4]
        ops.head9x9(gp, self.tail.bwd, None, gT, slope=1.0)
        # conv1 (+BN) — gT also reaches F through the trunk residual
        f0, f1 = pool[0], pool[1]
        self._bn_bwd(self.conv1, self.Z1, gT, f0, 64, grads)
        self._wgrad(self.conv1, self.r_last, f0, grads)
        ops.conv3x3(f0, 64, self.conv1.bwd, None, 64, f1, slope=1.0)
        # residual_2, then PixelShuffle(2) + LeakyReLU backward into the half grid
        g = self._chain_bwd(self.res2, self.S, f1, pool, 64, grads)
        gq = self.gq[0]
        ops.pixel_unshuffle2(gq, g, 256, m=self.S, mslope=SLOPE)
        # residual_1; its first block's input gradient is masked by LeakyReLU'(Q0)
        g = self._chain_bwd(self.res1, self.Q0, gq, self.gq, 256, grads, m_in=self.Q0)
        # stride-2 conv: weight (+bias) gradient on the phase view, input gradient by the shuffled store
        dwp = torch.empty(256, 256, 3, 3, device=dev)
        db = torch.empty(256, device=dev)
        ops.wgrad3x3(self.x_last0, 256, g, 256, dwp, db, x_sub2=True, taps=1)
        grads[id(self.down.w)], grads[id(self.down.b)] = gather_wgrad(dwp, 64), db
        gx = pool[0]
        ops.conv3x3(g, 256, self.down.bwd, None, 256, gx, slope=1.0, shuffle=2, taps=2)
        # residual_0, then the trunk: g_F = chain + gT, times LeakyReLU'(F) (conv0's act)
        g = self._chain_bwd(self.res0, self.F, gx, pool, 64, grads)
        gF = next(p for p in pool if p is not g)
        ops.ew_combine(gF, g, 64, sa=1.0, b=gT, sb=1.0, m=self.F, mslope=SLOPE)
        dw0 = torch.empty(64, 3, 9, 9, device=dev)
        db0 = torch.empty(64, device=dev)
        ops.wgrad9x9(self.x, gF, dw0, db0, head=True)
        grads[id(self.head.w)], grads[id(self.head.b)] = dw0, db0
        return grads


class _DenoiseFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan, *params):
        y = plan.forward(x)
        ctx.plan = plan
        plan.busy = True
        return y

    @staticmethod
    def backward(ctx, gy):
        plan = ctx.plan
        grads = plan.backward(gy.contiguous())
        plan.busy = False
        out = [grads.get(id(p)) for p in plan.params()]
        if plan.grad_group is not None:  # data parallel: one flat RCCL all-reduce (mean), as DDP
            from .train_engine import allreduce_mean
            out = allreduce_mean(out, None if plan.grad_group is True else plan.grad_group)
        return (None, None, *out)


def train_forward(model, x: torch.Tensor) -> torch.Tensor:
    """Differentiable train-mode Denoise forward on libisr (train.py:52-63 with
    --train_denoise).  One plan per input geometry; the graph of one call must be
    backpropagated before the next call (the plan holds its activations)."""
    n, _, h, w = x.shape
    key = (n, h, w, str(x.device))
    plan = model.__dict__.get("_isr_train_plan")
    if plan is None or plan.key != key:
        model.__dict__["_isr_train_plan"] = None
        plan = model.__dict__["_isr_train_plan"] = DenoiseTrainPlan(model, n, h, w, x.device)
    if plan.busy:
        raise RuntimeError("Denoise train_forward: the previous forward's graph was not backpropagated")
    plan.pack()
    plan.grad_group = model.__dict__.get("_isr_grad_group")  # train_engine.enable_grad_allreduce
    with torch.autocast("cuda", enabled=False):
        return _DenoiseFn.apply(x.float(), plan, *plan.params())
