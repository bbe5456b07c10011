"""Denoise network (utils/models.py:672-706) on libisr — inference.

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
