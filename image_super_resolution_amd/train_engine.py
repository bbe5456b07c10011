"""Training (forward + backward) of the RRDB generator on libisr (MI355X).

Replaces autograd through EResNet / SRGAN(enchant) (utils/models.py:621-650,
245-317, 572-589) as driven by train.py:52-63 and :88-102.  The forward keeps
one 192-channel dense buffer per RDB (the block input in channels [0, 64) and
the four growth outputs after it), so every activation the backward needs is
resident and no concat is ever materialised.  The backward walks the network
in reverse with three rotating 192-channel gradient buffers:

  tail    wgrad9x9 (dW2, db2);  dgrad = head9x9 kernel with 180°-rotated W2ᵀ,
          masked by LeakyReLU'(last Scaler output)
  scalers wgrad3x3 reading the PixelShuffle'd gradient (g_sub2);  dgrad =
          conv3x3 reading it as PixelShuffleᵀ (x_sub2) with LeakyReLU' mask
  conv1   wgrad + dgrad into the last RRDB's output gradient
  RRDB    per RDB (reverse): dgrad of the final conv writes the 192-channel
          gradient [g_x0 + residual | g_slot1..4] with LeakyReLU' of slot 4;
          growth conv k: wgrad, then dgrad accumulating into channels
          [0, 64+32k) in place and masking slot k-1 — the cat-backward and
          the activation backward are both epilogue work
  trunk   g_f0 = chain + g_T, LeakyReLU'(f0) (ew_combine);  head wgrad9x9

ResNet's Conv layers carry train-mode BatchNorm (utils/models.py:75-111): the
conv writes its pre-BN output z into a per-RDB z buffer, the BN kernels
(isr_bn_*) reduce batch statistics, update the running stats and apply
BN + activation (+ residuals) into the dense buffer; in the backward the BN
input gradient is formed in place on the masked slot gradient before that
conv's wgrad/dgrad, and dgamma/dbeta land in the flat gradient buffer.
"""
from __future__ import annotations

import os as _os

import ctypes
from dataclasses import dataclass

import torch
import torch.distributed as dist
from torch import nn

from . import _lib, ops
from ._lib import load as _load_lib
from .ops import ActBuffer

LEAKY = 0.01


@dataclass
class TConv:
    """One conv layer of the generator: parameter references + packed copies."""
    w: torch.Tensor
    b: torch.Tensor | None
    cin: int
    cout: int
    kind: str                  # "3x3", "head", "tail"
    dgrad_scale: float = 1.0
    sub2: bool = False         # dgrad reads the PixelShuffle'd gradient (Scaler)
    fwd: torch.Tensor | None = None
    bwd: torch.Tensor | None = None
    bn: nn.Module | None = None          # train-mode BatchNorm2d after the conv (ResNet's Conv)
    bn_state: object | None = None

    def pack(self):
        w = self.w.detach()
        if self.kind == "3x3":
            self.fwd = ops.pack_conv3x3(w, out=self.fwd)
            self.bwd = ops.pack_conv3x3_dgrad(w, scale=self.dgrad_scale, sub2=self.sub2, out=self.bwd)
        elif self.kind == "head":
            self.fwd = ops.pack_head9x9(w, out=self.fwd)
        else:  # tail: forward pack + its input-gradient conv run by the head kernel
            self.fwd = ops.pack_tail9x9(w, out=self.fwd)
            self.bwd = ops.pack_head9x9(w.float().flip(2, 3).transpose(0, 1).contiguous(), out=self.bwd)

    @property
    def bias(self) -> torch.Tensor:
        return self.b.detach() if self.b is not None else None


def _bn_of(m: nn.Module):
    bn = getattr(m, "bn", None)
    return bn if isinstance(bn, nn.BatchNorm2d) else None


def _generator_convs(gen: nn.Module) -> tuple[TConv, list[list[TConv]], TConv, list[TConv], TConv]:
    """Conv layers of a ResNet / EResNet in execution order (reference module paths)."""
    def t(m: nn.Module, kind="3x3", **kw):
        conv = m.conv
        return TConv(conv.weight, conv.bias, conv.in_channels, conv.out_channels, kind, bn=_bn_of(m), **kw)

    a = gen.add_rate
    head = t(gen.conv0, "head")
    rdbs = []
    for i, rrdb in enumerate(gen.residual):
        for r, rdb in enumerate(rrdb.net):
            # without BN the dgrad of the final conv carries the RDB (x add_rate) scale in the
            # weights (the RRDB-level x add_rate of the third RDB is the epilogue's s2); with BN
            # the scale is applied by the BN backward (gscale) instead
            fin = _bn_of(rdb.conv)
            rdbs.append([t(rdb.conv0), t(rdb.conv1), t(rdb.conv2), t(rdb.conv3),
                         t(rdb.conv, dgrad_scale=(1.0 if fin is not None else a))])
    conv1 = t(gen.conv1)
    scalers = [t(s.net[0], sub2=True) for s in gen.scaler]
    tail = t(gen.conv2, "tail")
    return head, rdbs, conv1, scalers, tail


class GeneratorTrainPlan:
    """Fixed-geometry training plan: buffers, packed weights and prebuilt
    descriptors for one (n, h, w).  `forward(x)` / `backward(gy)`; parameter
    gradients come back in the order of `params()`."""

    def __init__(self, gen: nn.Module, n: int, h: int, w: int, device):
        from .models import EResNet, ResNet, SRGAN
        if isinstance(gen, SRGAN):
            gen = gen.res_net
        if not isinstance(gen, (EResNet, ResNet)):
            raise NotImplementedError(f"HIP training path covers ResNet / EResNet / SRGAN, got {type(gen).__name__}")
        self.gen, self.key = gen, (n, h, w, str(device))
        self.device = torch.device(device)
        self.a = float(gen.add_rate)
        self.slope0 = float(gen.conv0.act.negative_slope)
        self.head, self.rdbs, self.conv1, self.scalers, self.tail = _generator_convs(gen)
        self.lib = _load_lib()
        S = len(self.scalers)
        dev = self.device
        # ---- activations (saved for the backward)
        self.f0 = ActBuffer.alloc(n, h, w, 64, 1, dev)
        nr = len(self.rdbs)
        # the trunk output buffer carries 192 channels too (only [0, 64) is used): the persistent
        # trunk kernel needs every layer's views in one buffer geometry (trunk.hip records)
        self.D = [ActBuffer.alloc(n, h, w, 192, 1, dev) for _ in range(nr + 1)]
        self.T = ActBuffer.alloc(n, h, w, 64, 1, dev)
        self.ups = []
        hh, ww, ha, wa = h, w, self.f0.ha, self.f0.wa
        for s in range(S):
            hh, ww, ha, wa = 2 * hh, 2 * ww, 2 * ha, 2 * wa
            self.ups.append(ActBuffer.alloc(n, hh, ww, 64, 4 if s == S - 1 else 1, dev, ha=ha, wa=wa))
        self.out_shape = (n, 3, hh, ww)
        # ---- gradients
        self.G = [ActBuffer.alloc(n, h, w, 192, 1, dev) for _ in range(3)]
        self.gT = ActBuffer.alloc(n, h, w, 64, 1, dev)
        self.gups = [ActBuffer.alloc(u.n, u.h, u.w, 64, 2, dev, ha=u.ha, wa=u.wa) for u in self.ups]
        self.gf0 = ActBuffer.alloc(n, h, w, 64, 1, dev)
        self.convs = [self.head] + [c for r in self.rdbs for c in r] + [self.conv1] + self.scalers + [self.tail]
        # ---- train-mode BatchNorm (ResNet): pre-BN conv outputs z and per-layer BN scratch
        self.has_bn = any(c.bn is not None for c in self.convs)
        if self.has_bn:
            self.Zb = [ActBuffer.alloc(n, h, w, 192, 1, dev) for _ in range(nr)]
            self.Tz = ActBuffer.alloc(n, h, w, 64, 1, dev)
            self.gtmp = ActBuffer.alloc(n, h, w, 64, 1, dev)
            for c in self.convs:
                if c.bn is not None:
                    c.bn_state = ops.BNState(c.cout, dev)
        self.bn_counters = [c.bn.num_batches_tracked for c in self.convs
                            if c.bn is not None and c.bn.num_batches_tracked is not None]
        # ---- parameters / gradient layout (one flat fp32 gradient buffer per backward)
        self._params, self._goff = [], []
        off = 0
        for c in self.convs:
            ps = [c.w, c.b] + ([c.bn.weight, c.bn.bias] if c.bn is not None else [])
            for p in ps:
                if p is not None:
                    self._params.append(p)
                    self._goff.append(off)
                    off += (p.numel() + 3) // 4 * 4  # 16-byte aligned views
        self._gsize = off
        # RDB input gradients as "gather" convs (no BatchNorm): per RDB, one conv per dense-buffer
        # block — the gradient of block o_t (and of x) is ONE conv over the concatenated output
        # gradients of every conv that read it (forward-shaped: K 576..1728, 32 / 64 outputs,
        # each output written once) instead of an accumulate-into-all-channels transposed conv
        # per layer (K 288, read-modify-write of 64..192 channels).  Weights: slices of the
        # layers' transposed weights, packed per step by the same batched launch.
        self.gather = (not self.has_bn) and _os.environ.get("ISR_TRAIN_GATHER", "1") == "1"
        if self.gather:
            nbytes = self.lib.isr_conv3x3_packed_bytes
            self.gpacks = []
            for _ in self.rdbs:
                gp = {t: torch.empty(nbytes(32, 64 + 32 * (3 - t)) // 2, dtype=torch.bfloat16, device=dev)
                      for t in range(4)}
                gp["x"] = torch.empty(nbytes(64, 192) // 2, dtype=torch.bfloat16, device=dev)
                self.gpacks.append(gp)
        self.pack()
        self._build()

    # ------------------------------------------------------------------ setup
    def params(self) -> list[torch.Tensor]:
        return list(self._params)

    def pack(self) -> None:
        """Refresh the packed bf16 weights from the fp32 parameters (every step):
        every 3x3 conv's forward and dgrad pack in ONE launch (isr_pack_conv3x3_batch),
        the two 9x9 convs separately."""
        if getattr(self, "_pack_items", None) is None:
            for c in self.convs:  # first call: allocate the packed buffers
                c.pack()
            rdb_convs = {id(c) for r in self.rdbs for c in r} if self.gather else set()
            self._pack_items = ops.pack_batch_table(
                [(c.w, c.fwd, c.cout, c.cin, False, False, 1.0) for c in self.convs if c.kind == "3x3"]
                + [(c.w, c.bwd, c.cout, c.cin, True, c.sub2, c.dgrad_scale) for c in self.convs
                   if c.kind == "3x3" and id(c) not in rdb_convs]
                + (self._gather_items() if self.gather else []),
                self.device)
            ops.pack_batch(self._pack_items)
            return
        ops.pack_batch(self._pack_items)
        for c in self.convs:
            if c.kind != "3x3":
                c.pack()

    def _gather_items(self) -> list:
        """isr_pack_item windows for the RDB input-gradient gather convs (see __init__).
        Target o_t (t = 3..0): output = the 32 input channels [64+32t, 96+32t) of the RDB's
        dense buffer; input = [g_f | g_3 | ... | g_{t+1}] (64 + 32 (3-t) channels: the final
        conv's output gradient, then each growth conv's); target x: output = channels [0, 64),
        input = all 192.  Block weights = the producing layer's transposed weights restricted
        to the target's channels; the final conv's block carries its RDB scale a (and the
        RRDB's a for the third RDB: utils/models.py:265-271, 316-317)."""
        a, items = self.a, []
        for j, cs in enumerate(self.rdbs):
            res = a if j % 3 == 2 else 1.0
            c5 = cs[4]
            gp = self.gpacks[j]
            for t in list(range(3, -1, -1)) + ["x"]:
                out = gp[t]
                # the x target's pack carries 1 / res: its conv adds the RDB output gradient with s1 = 1
                # (v = (acc / res + g_out) * res), which the persistent backward chain folds exactly
                sx = 1.0 / res if t == "x" else 1.0
                if t == "x":
                    n0, co, srcs = 0, 64, list(range(3, -1, -1))
                else:
                    n0, co, srcs = 64 + 32 * t, 32, list(range(3, t, -1))
                items.append((c5.w, out, 64, co, True, False, a * res * sx, n0, 192, 0))
                for k in srcs:
                    off = 64 + 32 * (3 - k)  # input-channel offset of g_k in the gather input
                    items.append((cs[k].w, out, 32, co, True, False, sx, n0, cs[k].cin, (off // 16) * 9 * co * 16))
        return items

    def _build(self):
        a, lib = self.a, self.lib
        conv, head, tail = lib.isr_conv3x3_fwd, lib.isr_head9x9_fwd, lib.isr_tail9x9_fwd
        D, f0, T = self.D, self.f0, self.T
        self.dummy_x = torch.empty(self.out_shape[0], 3, f0.h, f0.w, device=self.device)
        self.dummy_y = torch.empty(self.out_shape, device=self.device)
        F = []
        self.head_desc = ops.head9x9_desc(self.dummy_x, self.head.fwd, self.head.bias, f0, slope=self.slope0, y2=D[0])
        F.append((head, self.head_desc))
        def conv_bn(x, cin, c, y, y_coff, z, z_coff, slope, **res):
            """conv → y directly, or (BN layer) conv → z, batch stats, BN+act(+residuals) → y."""
            if c.bn is None:
                F.append((conv, ops.conv3x3_desc(x, cin, c.fwd, c.bias, c.cout, y, y_coff=y_coff, slope=slope, **res)))
            else:
                F.append((conv, ops.conv3x3_desc(x, cin, c.fwd, c.bias, c.cout, z, y_coff=z_coff, slope=1.0)))
                F.append(("bnf", ops.bn_desc(z, y, c.cout, c.bn_state, c.bn, z_coff=z_coff, y_coff=y_coff,
                                             slope=slope, **res), c.bn_state))

        trunk0 = len(F)
        for j, cs in enumerate(self.rdbs):
            Zj = self.Zb[j] if self.has_bn else None
            for k in range(4):
                c = cs[k]
                conv_bn(D[j], c.cin, c, D[j], c.cin, Zj, c.cin, LEAKY)
            c = cs[4]
            extra = dict(r2=D[j - 2], s2=a) if j % 3 == 2 else {}
            conv_bn(D[j], 192, c, D[j + 1], 0, Zj, 0, 1.0, r1=D[j], s1=a, **extra)
        self.chain = None
        if not self.has_bn and self.rdbs and _os.environ.get("ISR_TRAIN_CHAIN", "1") == "1" and not _device_shared():
            # no BatchNorm: the whole trunk forward as ONE persistent isr_conv_chain launch (as
            # inference, engine.ConvChain); every RDB writes its own dense buffer here
            from .engine import ConvChain
            try:
                from .engine import CHAIN_ACQUIRE
                self.chain = ConvChain([e[1] for e in F[trunk0:]], D[0], self.device, acquire=CHAIN_ACQUIRE)
            except ValueError as e:  # not silent: the per-conv trunk costs ~3.5 ms per SRGAN step
                import warnings
                warnings.warn(f"training trunk runs per conv (persistent trunk kernel refused the layers: {e})")
                self.chain = None
            if self.chain is not None:
                F[trunk0:] = [(self.chain.fn, self.chain.desc)]
        c = self.conv1
        conv_bn(D[-1], 64, c, T, 0, self.Tz if self.has_bn else None, 0, 1.0, r1=f0, s1=1.0)
        cur = T
        for s, c in enumerate(self.scalers):
            F.append((conv, ops.conv3x3_desc(cur, 64, c.fwd, c.bias, 256, self.ups[s], slope=LEAKY, shuffle=2)))
            cur = self.ups[s]
        self.tail_desc = ops.tail9x9_desc(cur, self.tail.fwd, self.tail.bias, self.dummy_y)
        F.append((tail, self.tail_desc))
        self.fwd_launches = F

        # ---- backward.  Entries: ("conv", desc) | ("wg3", desc, conv_index) | ("wg9", desc, conv_index)
        #      | ("head", desc) | ("ew", desc).  dw/db pointers are patched per call.
        B = []
        ci = {id(c): i for i, c in enumerate(self.convs)}
        dev = self.device

        def wg3(x, cin, g, cout, c, *, x_coff=0, g_coff=0, scale=1.0, g_sub2=False, side=False):
            d = ops.wgrad3x3_desc(x, cin, g, cout, _meta_dw(cout, cin, 3, dev), None, x_coff=x_coff, g_coff=g_coff,
                                  scale=scale, g_sub2=g_sub2)
            B.append(("wg3", d, ci[id(c)], side))

        # tail
        self.gp = torch.empty(self.out_shape, device=dev)
        ut = self.ups[-1]
        d9 = ops.wgrad9x9_desc(self.gp, ut, _meta_dw(3, 64, 9, dev), None, head=False)
        B.append(("wg9", d9, ci[id(self.tail)]))
        B.append(("head", ops.head9x9_desc(self.gp, self.tail.bwd, None, self.gups[-1], slope=1.0, m=ut,
                                           mslope=LEAKY)))
        # scalers (reverse)
        for s in range(len(self.scalers) - 1, -1, -1):
            c = self.scalers[s]
            xin = self.ups[s - 1] if s > 0 else T
            wg3(xin, 64, self.gups[s], 256, c, g_sub2=True)
            out = self.gups[s - 1] if s > 0 else self.gT
            kw = dict(m=self.ups[s - 1], mslope=LEAKY) if s > 0 else {}
            B.append(("conv", ops.conv3x3_desc(self.gups[s], 256, c.bwd, None, 64, out, x_sub2=True, **kw)))
        def bn_bwd(c, z, g, *, z_coff=0, g_coff=0, dz=None, gscale=1.0):
            """BN input gradient of conv c: g (gradient wrt the BN output) → dz (in place if dz is None)."""
            B.append(("bnb", ops.bn_desc(z, g, c.cout, c.bn_state, c.bn, z_coff=z_coff, y_coff=g_coff, dz=dz,
                                         gscale=gscale), ci[id(c)], c.bn_state))

        # conv1:  T = BN?(conv1(D[-1][0:64])) + f0
        c = self.conv1
        U, V, W = self.G
        g1 = self.gT
        if c.bn is not None:
            bn_bwd(c, self.Tz, self.gT, dz=self.gtmp)
            g1 = self.gtmp
        wg3(D[-1], 64, g1, 64, c)
        B.append(("ready", "tail", False))  # conv1 / Scaler / tail gradients complete (main stream)
        B.append(("conv", ops.conv3x3_desc(g1, 64, c.bwd, None, 64, U)))
        # RRDBs, reverse
        nb = len(self.rdbs) // 3
        if self.gather:
            # gather form (no BN): one gradient dense buffer per RDB, E_j = [g_out | g_3 | g_2 |
            # g_1 | g_0]; g_out (the RDB output gradient) arrives in E_j[0:64], each target conv
            # appends its block, the x target writes the RDB input gradient into E_{j-1}[0:64]
            # (RDB 0: into `self.gtrunk`).  Nothing is overwritten, so the five weight gradients
            # of RDB j run on a second HIP stream (`side`) as soon as its target 0 is done
            # ("evrec" / "evwait"), beside the next RDBs' gather convs.
            nr = len(self.rdbs)
            self.Eg = [ActBuffer.alloc(n_, h_, w_, 192, 1, dev) for n_, h_, w_ in [(D[0].n, D[0].h, D[0].w)] * nr]
            # 192 channels (64 used): the persistent backward chain needs one buffer geometry
            self.gtrunk = ActBuffer.alloc(D[0].n, D[0].h, D[0].w, 192, 1, dev)
            # conv1's input gradient (g_R of the last RRDB) goes straight into E_{nr-1}[0:64]
            B[-1] = ("conv", ops.conv3x3_desc(g1, 64, c.bwd, None, 64, self.Eg[nr - 1]))
            for i in range(nb - 1, -1, -1):
                for step, j in enumerate((3 * i + 2, 3 * i + 1, 3 * i)):
                    cs, Dj, gp, E = self.rdbs[j], D[j], self.gpacks[j], self.Eg[j]
                    gout = self.Eg[j - 1] if j > 0 else self.gtrunk
                    res = a if step == 0 else 1.0
                    for t in range(3, -1, -1):
                        slot = 64 + 32 * (3 - t)
                        B.append(("conv", ops.conv3x3_desc(E, slot, gp[t], None, 32, E, y_coff=slot, m=Dj,
                                                           m_coff=64 + 32 * t, m_c0=0, mslope=LEAKY), "gather"))
                    B.append(("evrec", j))
                    B.append(("evwait", j))
                    wg3(Dj, 192, E, 64, cs[4], scale=a * res, side=True)
                    for t in range(3, -1, -1):
                        wg3(Dj, cs[t].cin, E, 32, cs[t], g_coff=64 + 32 * (3 - t), side=True)
                    if step == 2:  # RRDB i's weight gradients are all enqueued (side stream)
                        B.append(("ready", i, True))
                    # v = (acc' + g_out) * res (+ g_R: the RRDB's own residual, first RDB); the pack
                    # carries 1 / res, so acc' = acc / res
                    kw = dict(r2=self.Eg[3 * i + 2]) if step == 2 else {}
                    # r1_cn=64 (= every output channel, the same sums) keeps the per-conv launch on the
                    # plain 192->64 kernel; the persistent backward chain folds r1 (r1_cn = 0)
                    B.append(("conv", ops.conv3x3_desc(E, 192, gp["x"], None, 64, gout, r1=E, s1=1.0, s2=res,
                                                       r1_cn=64, **kw), "gather"))
            U = self.gtrunk
        for i in range(nb - 1, -1, -1) if not self.gather else ():
            # g_R (gradient wrt the RRDB output) is in U[0:64]
            seq = [(3 * i + 2, U, V), (3 * i + 1, V, W), (3 * i, W, V)]
            for step, (j, gin, gout) in enumerate(seq):
                cs = self.rdbs[j]
                Dj = D[j]
                c5 = cs[4]
                last_rdb = step == 0  # the third RDB of the RRDB (first in reverse)
                # final conv: out = conv*a + Dj[0:64]  (third RDB: (...)*a + RRDB input)
                res = a if last_rdb else 1.0       # coefficient of Dj[0:64] in the RRDB output
                if c5.bn is None:
                    wg3(Dj, 192, gin, 64, c5, scale=(a * a if last_rdb else a))
                    B.append(("conv", ops.conv3x3_desc(gin, 64, c5.bwd, None, 192, gout, r1=gin, r1_cn=64,
                                                       s2=res, m=Dj, m_c0=160, mslope=LEAKY)))
                else:
                    # dz5 = BN'(a*res * g_R) into gtmp; residual keeps g_R: y = (v/res + g_R) * res
                    bn_bwd(c5, self.Zb[j], gin, dz=self.gtmp, gscale=a * res)
                    wg3(Dj, 192, self.gtmp, 64, c5)
                    B.append(("conv", ops.conv3x3_desc(self.gtmp, 64, c5.bwd, None, 192, gout, r1=gin, r1_cn=64,
                                                       s1=1.0 / res, s2=res, m=Dj, m_c0=160, mslope=LEAKY)))
                for k in range(3, -1, -1):
                    ck = cs[k]
                    slot = 64 + 32 * k
                    if ck.bn is not None:  # slot k is complete and LeakyReLU'-masked: BN backward in place
                        bn_bwd(ck, self.Zb[j], gout, z_coff=slot, g_coff=slot)
                    wg3(Dj, ck.cin, gout, 32, ck, g_coff=slot)
                    kw = dict(m=Dj, m_c0=slot - 32, mslope=LEAKY) if k > 0 else {}
                    if k == 0 and step == 2:
                        kw = dict(r2=U, s2=1.0)  # + g_R: the RRDB's own residual
                    B.append(("conv", ops.conv3x3_desc(gout, 32, ck.bwd, None, ck.cin, gout, x_coff=slot,
                                                       r1=gout, **kw)))
            B.append(("ready", i, False))  # RRDB i's gradients complete (main stream)
            # RRDB input gradient now in V[0:64]; rotate so it becomes the next g_R
            U, V, W = V, W, U
        # trunk: g_f0 = chain + g_T, then LeakyReLU'(f0) of conv0
        B.append(("ew", ops.ew_combine_desc(self.gf0, U, 64, sa=1.0, b=self.gT, sb=1.0, m=f0,
                                            mslope=self.slope0)))
        d9h = ops.wgrad9x9_desc(self.dummy_x, self.gf0, _meta_dw(64, 3, 9, dev), None, head=True)
        B.append(("wg9", d9h, ci[id(self.head)]))
        B.append(("ready", "head", False))
        self.bchain = None
        if self.gather and _os.environ.get("ISR_TRAIN_BWD_CHAIN", "0") == "1" and not _device_shared():
            B = self._backward_chain(B)
        wg_group = _os.environ.get("ISR_TRAIN_WG_GROUP", "1")
        if wg_group in ("1", "4"):  # "4": the RDB final conv stays on its own ci-split launch (A/B)
            B = _group_side_wgrads(B, lib, skip_final=wg_group == "4")
        self.bwd_launches = B
        self.head_wg = d9h
        # workspace for the split-K partial sums
        nbytes = 0
        for e in B:
            if e[0] == "wg3":
                nbytes = max(nbytes, lib.isr_wgrad3x3_workspace_bytes(ctypes.byref(e[1])))
            elif e[0] == "wg3g":
                nbytes = max(nbytes, lib.isr_wgrad3x3_group_workspace_bytes(e[1], len(e[2])))
            elif e[0] == "wg9":
                nbytes = max(nbytes, lib.isr_wgrad9x9_workspace_bytes(ctypes.byref(e[1])))
        if nbytes == 0:
            raise RuntimeError("train plan: could not size the wgrad workspace: "
                               + lib.isr_last_error().decode(errors="replace"))
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        # the side stream's weight gradients get a workspace of their own (they run concurrently
        # with the main stream's)
        self.ws_side = torch.empty(nbytes, dtype=torch.uint8, device=dev) if self.gather else None
        self.side = (torch.cuda.Stream(dev) if self.gather and _os.environ.get("ISR_TRAIN_SIDE", "1") == "1"
                     else None)
        # A/B option (ISR_TRAIN_RED_STREAM=1, off): the side stream's split-K reductions on a third
        # stream over a ring of RED_RING workspaces (a slot is reused once the reduce that read it
        # has finished), so the side stream chains only the weight-gradient kernels.  Skipping the
        # reductions altogether saves 3.3 ms per cfg3 step (tuning probe, tools/r04_train_probe.sh),
        # but moving them off the chain loses 1.2 ms (51.7 / 51.8 vs 50.5 / 50.6 ms, alternating
        # processes, profiles/r04_train_red_stream_ab.jsonl): their cost is the partials' traffic,
        # not their place in the chain
        self.red = None
        if self.side is not None and _os.environ.get("ISR_TRAIN_RED_STREAM", "0") == "1":
            self.red = torch.cuda.Stream(dev)
            self.ws_ring = [self.ws_side] + [torch.empty(nbytes, dtype=torch.uint8, device=dev)
                                             for _ in range(RED_RING - 1)]
            self.ev_part = [torch.cuda.Event() for _ in range(RED_RING)]
            self.ev_red = [torch.cuda.Event() for _ in range(RED_RING)]
        self.events = {}
        # gradient offsets per conv: (w, b or None, bn weight or None, bn bias or None)
        self._conv_goff = []
        pi = 0
        for c in self.convs:
            wo = self._goff[pi]
            pi += 1
            bo = None
            if c.b is not None:
                bo = self._goff[pi]
                pi += 1
            go = bo2 = None
            if c.bn is not None:
                go, bo2 = self._goff[pi], self._goff[pi + 1]
                pi += 2
            self._conv_goff.append((wo, bo, go, bo2))
        # data-parallel gradient buckets: the flat buffer in backward order is
        # [conv1 .. tail] (end of the buffer), RRDB nb-1, ..., RRDB 0, head (start) — contiguous
        # descending ranges, each complete at its ("ready", id) entry of the backward list
        first = lambda conv_index: self._conv_goff[conv_index][0]
        nr = len(self.rdbs)
        seg = {"tail": (first(1 + 5 * nr), self._gsize), "head": (0, first(1) if nr else self._gsize)}
        for i in range(nr // 3):
            seg[i] = (first(1 + 15 * i), first(1 + 15 * (i + 1)))
        self._segments = seg

    def _backward_chain(self, B: list) -> list:
        """The RDB gather convs of the backward (240 for 16 RRDBs) as ONE persistent isr_conv_chain
        launch (trunk.hip: the forward dense block's dependency shape — gather t reads
        E[0:64 + 32 (3 - t)) and writes the next 32 channels, masked by LeakyReLU' of the forward
        activation (kind 2); the x gather folds the RDB output gradient, r1 = E[0:64]).  The chain
        owns the whole chip, so the side stream's weight gradients start after it, and DDP's first
        bucket is flushed after it too (an all-reduce beside it would take CUs its grid needs).
        Shares the forward chain's state: one give-up count guards the step's optimiser updates.
        A/B option (ISR_TRAIN_BWD_CHAIN=1, off): correct (tests/test_gpu_train.py) but 52.87 vs
        52.23 ms per cfg3 step, same box (profiles/r04_train_bwd_chain_ab.jsonl) — the weight
        gradients it pushes behind the chain had been overlapping the per-conv gathers."""
        from .engine import CHAIN_ACQUIRE, ConvChain
        gathers = [k for k, e in enumerate(B) if e[0] == "conv" and len(e) > 2 and e[2] == "gather"]
        if not gathers:
            return B
        zb = torch.zeros(64, device=self.device)
        self._bchain_bias = zb
        descs = []
        for k in gathers:
            d = IsrConvDescCopy(B[k][1])
            d.bias = zb.data_ptr()
            if d.cout == 64:
                d.r1_cn = 0  # fold the RDB output gradient (r1 aliases the gather input)
            descs.append(d)
        try:
            self.bchain = ConvChain(descs, self.D[0], self.device, acquire=CHAIN_ACQUIRE, variant=0,
                                    state=self.chain.state if self.chain is not None else None)
        except ValueError as err:
            import warnings
            warnings.warn(f"training backward gathers run per conv (persistent chain refused: {err})")
            self.bchain = None
            return B
        first, last = gathers[0], gathers[-1]
        body = [e for e in B[first:last + 1] if not (e[0] == "conv" and len(e) > 2 and e[2] == "gather")
                and e[0] not in ("evrec", "evwait")]
        head = [e for e in B[:first] if not (e[0] == "ready" and e[1] == "tail")]
        tail_ready = [e for e in B[:first] if e[0] == "ready" and e[1] == "tail"]
        return (head + [("bchain", self.bchain)] + tail_ready + [("evrec", "bchain"), ("evwait", "bchain")]
                + body + B[last + 1:])

    # -------------------------------------------------------------- execution
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """x: normalised NCHW fp32 [n, 3, h, w] on the device; returns tanh output."""
        if tuple(x.shape) != (self.out_shape[0], 3, self.f0.h, self.f0.w) or x.dtype != torch.float32:
            raise ValueError(f"train plan built for {self.key}, got {tuple(x.shape)} {x.dtype}")
        x = x.contiguous()
        self.x = x
        y = torch.empty(self.out_shape, device=self.device)
        self.head_desc.x = x.data_ptr()
        self.tail_desc.y = y.data_ptr()
        self.head_wg.p = x.data_ptr()
        st = ops._stream()
        byref = ctypes.byref
        lib = self.lib
        for e in self.fwd_launches:
            if e[0] == "bnf":
                d, bst = e[1], e[2]
                bst.acc.zero_()
                for fn in (lib.isr_bn_stats, lib.isr_bn_finalize, lib.isr_bn_apply):
                    rc = fn(byref(d), st)
                    if rc != 0:
                        ops.check(rc, "train forward (bn)")
                continue
            rc = e[0](byref(e[1]), st)
            if rc != 0:
                ops.check(rc, "train forward")
            if self.chain is not None and e[1] is self.chain.desc:
                self.trunk_done = torch.cuda.Event()
                self.trunk_done.record()
        if self.chain is not None:
            self.chain.poll()  # lagged, non-blocking give-up check (engine.ConvChain.poll)
        if self.bn_counters:
            torch._foreach_add_(self.bn_counters, 1)  # nn.BatchNorm2d.train() bookkeeping
        self.y = y
        return y

    def backward(self, gy: torch.Tensor) -> list[torch.Tensor]:
        """gy: dL/d(output) NCHW fp32.  Returns gradients aligned with params()."""
        torch.mul(gy, 1.0 - self.y * self.y, out=self.gp)  # tanh' (utils/models.py:607 act=Tanh)
        grads = torch.empty(self._gsize, device=self.device)
        gbase = grads.data_ptr()
        lib, st, byref = self.lib, ops._stream(), ctypes.byref
        ws, wsn = self.ws.data_ptr(), self.ws.numel()
        main = torch.cuda.current_stream(self.device)
        side_used = False
        if self.side is not None:
            self.side.wait_stream(main)  # `grads` and the forward's activations are ready
            sst = ctypes.c_void_p(self.side.cuda_stream)
        group = self.gen.__dict__.get("_isr_grad_group")
        ddp = _Buckets(self, grads, group, main) if group is not None else None
        red = self.red
        if red is not None:
            rst = ctypes.c_void_p(red.cuda_stream)
            red_used = [False] * RED_RING
            nside = 0
        side_done = red if red is not None else self.side  # where a side-produced segment completes
        for e in self.bwd_launches:
            kind, d = e[0], e[1]
            if kind == "ready":
                if ddp is not None:
                    ddp.ready(d, side_done if (e[2] and self.side is not None) else main)
                continue
            if kind in ("evrec", "evwait") and self.side is None:
                continue
            if kind == "evrec":
                ev = self.events.get(d)
                if ev is None:
                    ev = self.events[d] = torch.cuda.Event()
                ev.record(main)
                continue
            if kind == "evwait":
                self.side.wait_event(self.events[d])
                side_used = True
                continue
            if kind == "conv":
                rc = lib.isr_conv3x3_fwd(byref(d), st)
            elif kind == "bchain":
                rc = d.fn(byref(d.desc), st)
            elif kind == "bnb":
                _, _, go, bo2 = self._conv_goff[e[2]]
                d.dgamma, d.dbeta = gbase + 4 * go, gbase + 4 * bo2
                e[3].acc.zero_()
                rc = lib.isr_bn_bwd_reduce(byref(d), st)
                if rc == 0:
                    rc = lib.isr_bn_bwd_apply(byref(d), st)
            elif kind == "wg3" or kind == "wg9":
                wo, bo = self._conv_goff[e[2]][:2]
                d.dw = gbase + 4 * wo
                d.db = gbase + 4 * bo if bo is not None else None
                if kind == "wg3" and e[3] and red is not None:
                    k = nside % RED_RING
                    nside += 1
                    wsk = self.ws_ring[k]
                    if red_used[k]:
                        self.side.wait_event(self.ev_red[k])  # the slot's previous reduce has read it
                    rc = lib.isr_wgrad3x3_partials(byref(d), wsk.data_ptr(), wsk.numel(), sst)
                    if rc == 0:
                        self.ev_part[k].record(self.side)
                        red.wait_event(self.ev_part[k])
                        rc = lib.isr_wgrad3x3_reduce(byref(d), wsk.data_ptr(), wsk.numel(), rst)
                        self.ev_red[k].record(red)
                        red_used[k] = True
                elif kind == "wg3" and e[3] and self.side is not None:
                    rc = lib.isr_wgrad3x3(byref(d), self.ws_side.data_ptr(), self.ws_side.numel(), sst)
                else:
                    rc = (lib.isr_wgrad3x3 if kind == "wg3" else lib.isr_wgrad9x9)(byref(d), ws, wsn, st)
            elif kind == "wg3g":  # one RDB's weight gradients in one launch (isr_wgrad3x3_group)
                for k, c in enumerate(e[2]):
                    wo, bo = self._conv_goff[c][:2]
                    d[k].dw = gbase + 4 * wo
                    d[k].db = gbase + 4 * bo if bo is not None else None
                if self.side is not None:
                    rc = lib.isr_wgrad3x3_group(d, len(e[2]), self.ws_side.data_ptr(), self.ws_side.numel(), sst)
                else:
                    rc = lib.isr_wgrad3x3_group(d, len(e[2]), ws, wsn, st)
            elif kind == "head":
                rc = lib.isr_head9x9_fwd(byref(d), st)
            else:
                rc = lib.isr_ew_combine(byref(d), st)
            if rc != 0:
                ops.check(rc, f"train backward ({kind})")
        if side_used:
            main.wait_stream(self.side)
            if red is not None:
                main.wait_stream(red)
        if ddp is not None:
            ddp.finish()  # the main stream waits for every bucket, then the mean
        out = []
        for p, off in zip(self._params, self._goff):
            out.append(grads[off:off + p.numel()].view(p.shape))
        return out


def IsrConvDescCopy(d):
    """An independent copy of an isr_conv_desc (ctypes structures assign by value)."""
    c = type(d)()
    ctypes.pointer(c)[0] = d
    return c


# workspaces in the ring of the side stream's split-K partials (train plan with a reduce stream)
RED_RING = 4


def _group_side_wgrads(B: list, lib, skip_final: bool = False) -> list:
    """Runs of consecutive side-stream 3x3 weight gradients (one RDB's five convs: one dense
    buffer, one gradient buffer) become ONE ("wg3g", descriptor array, conv indices, True) entry
    launched through isr_wgrad3x3_group — one grid over all their (co, ci) tile pairs, ~5x fewer
    split-K partials.  A run the library refuses to group stays as separate launches."""
    out, run = [], []

    def flush():
        if len(run) >= 2:
            arr = (_lib.IsrWgradDesc * len(run))(*[r[1] for r in run])
            if lib.isr_wgrad3x3_group_workspace_bytes(arr, len(run)) > 0:
                out.append(("wg3g", arr, [r[2] for r in run], True))
                run.clear()
                return
        out.extend(run)
        run.clear()

    def groupable(e):
        return e[0] == "wg3" and e[3] and not (skip_final and e[1].cout == 64 and e[1].cin == 192)

    for e in B:
        if groupable(e) and len(run) < 5:
            run.append(e)
            continue
        flush()
        if groupable(e):
            run.append(e)
        else:
            out.append(e)
    flush()
    return out


# DDP-style gradient buckets: consecutive backward segments are merged until a bucket holds at
# least this many bytes (xGMI rings are per-link bound: a few MB per call keeps the fixed cost
# per collective small against its transfer time; 47.5 MB of generator gradients -> ~6 buckets)
BUCKET_BYTES = int(float(_os.environ.get("ISR_DDP_BUCKET_MB", "8")) * (1 << 20))


class _Buckets:
    """The data-parallel gradient all-reduce of one backward, overlapped with it (SURVEY.md §8e,
    DDP's bucketed all-reduce): the flat fp32 gradient buffer's segments complete in backward
    order (tail, RRDB nb-1 .. 0, head); consecutive segments merge into buckets of >=
    BUCKET_BYTES, and each bucket is all-reduced on a communication stream as soon as every stream
    that produced one of its segments (main, or the side stream of the RDB weight gradients) has
    enqueued it — an event hand-off, no host synchronisation.  finish() makes the main stream
    wait for every bucket and divides by the world size.  Same sums as one flat all-reduce per
    element (each element is reduced exactly once), so ranks stay bitwise equal."""

    def __init__(self, plan, grads: torch.Tensor, group, main):
        import torch.distributed as dist
        self.dist, self.plan, self.grads, self.main = dist, plan, grads, main
        self.group = None if group is True else group
        self.comm = plan.__dict__.setdefault("_comm_stream", torch.cuda.Stream(grads.device))
        self.lo = self.hi = None
        self.producers = []  # streams that wrote the pending bucket's segments
        self.works = []

    def ready(self, seg_id, stream) -> None:
        lo, hi = self.plan._segments[seg_id]
        if self.hi is None:
            self.lo, self.hi = lo, hi
        else:
            assert hi == self.lo, "gradient segments must complete in descending buffer order"
            self.lo = lo
        if not any(s is stream for s in self.producers):
            self.producers.append(stream)
        if (self.hi - self.lo) * 4 >= BUCKET_BYTES or seg_id == "head":
            # a merged bucket can hold segments of both streams (side-stream RDB weight
            # gradients beside main-stream head/tail ones): wait for every producer
            for s in self.producers:
                ev = torch.cuda.Event()
                ev.record(s)
                self.comm.wait_event(ev)
            with torch.cuda.stream(self.comm):
                self._reduce(self.grads[self.lo:self.hi])
            self.lo = self.hi = None
            self.producers = []

    def _reduce(self, t: torch.Tensor) -> None:
        dist = self.dist
        if dist.get_backend(self.group) == "gloo":  # host-staged (rehearsal on one GPU, tests)
            all_reduce_(t, self.group)
        else:
            self.works.append(dist.all_reduce(t, group=self.group, async_op=True))

    def finish(self) -> None:
        if self.hi is not None:
            raise RuntimeError("gradient buckets: the backward ended with an unreduced segment")
        for w in self.works:
            w.wait()  # the current (main) stream waits for the collective
        self.main.wait_stream(self.comm)
        self.grads.div_(self.dist.get_world_size(self.group))


def _meta_dw(cout: int, cin: int, k: int, dev) -> torch.Tensor:
    """Shape-valid placeholder for descriptor construction; the real dw/db
    pointers are patched per backward call."""
    return _PLACEHOLDER.setdefault((cout, cin, k, str(dev)), torch.empty(cout, cin, k, k, device=dev))


_PLACEHOLDER: dict = {}


class _GeneratorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan, *params):
        ctx.plan = plan
        return plan.forward(x)

    @staticmethod
    def backward(ctx, gy):
        grads = ctx.plan.backward(gy.contiguous().float())
        return (None, None, *grads)


def _device_shared() -> bool:
    """True when several ranks of this job drive one GPU (gloo over CUDA tensors, or more local
    ranks than devices): two persistent-chain grids on one device cannot both be resident, so
    the training plan runs its trunk per conv then."""
    if not (dist.is_available() and dist.is_initialized()):
        return False
    local = int(_os.environ.get("LOCAL_WORLD_SIZE", dist.get_world_size()))
    return dist.get_backend() == "gloo" or local > max(1, torch.cuda.device_count())


def _plan_of(gen: nn.Module):
    """The training plan of a generator (an SRGAN's lives on its res_net, where train_forward runs)."""
    from .models import SRGAN
    if isinstance(gen, SRGAN):
        gen = gen.res_net
    return gen.__dict__.get("_isr_train_plan")


def _grad_group(gen: nn.Module):
    """The process group of the generator's gradient all-reduce (enable_grad_allreduce), or None."""
    from .models import SRGAN
    if isinstance(gen, SRGAN):
        gen = gen.res_net
    return gen.__dict__.get("_isr_grad_group")


def _plan_device(plan) -> torch.device:
    chain = getattr(plan, "chain", None)
    return chain.state.device if chain is not None else plan.device


def verify_chains(gen: nn.Module) -> None:
    """Blocking persistent-chain give-up check of every training forward queued so far on this
    generator (engine.ChainFailed); the trainer calls it at the end of every epoch, before the
    epoch's results (losses, checkpoint) are handed out.  Data parallel: every rank raises when
    any rank's trunk gave up (one all-reduce of the local verdict), so no rank walks on into a
    collective its failed peer will never join.  Every generator rank takes part in that
    all-reduce, also one whose trunk fell back to per-conv launches (it votes 0) and one whose
    check itself failed with another error (it votes 1 and re-raises that error after the
    collective), so a peer never waits in it alone."""
    from .engine import ChainFailed
    plan = _plan_of(gen)
    if plan is None or not hasattr(plan, "chain"):  # no training forward yet / the Denoise plan (no trunk)
        return
    chain = plan.chain
    group = _grad_group(gen)
    if group is None:
        if chain is not None:
            chain.verify()
        return
    err, bad = None, 0
    try:
        if chain is not None:
            chain.verify()
    except ChainFailed:
        bad = 1
    except BaseException as e:  # noqa: BLE001 - re-raised below, after the peers have the vote
        err, bad = e, 1
    t = torch.tensor([bad], dtype=torch.int32, device=_plan_device(plan))
    all_reduce_(t, None if group is True else group)
    if err is not None:
        raise err
    if int(t.item()):
        raise ChainFailed(f"conv chain: a dependency wait gave up on {int(t.item())} rank(s); the "
                          "affected steps were skipped on every rank")


def step_guard_ptr(gen: nn.Module):
    """The trunk give-up guard of the generator's last training forward (engine.ConvChain.guard_ptr),
    or None when it ran without the persistent trunk kernel.

    Data parallel (enable_grad_allreduce): the gradients are already averaged over the ranks when
    the guard is read, so a rank whose trunk gave up has mixed invalid gradients into every peer's.
    The guard is therefore global: each rank's "gave up and not yet reported" flag
    (state[2] != state[3]) is summed over the group on the device and written into a two-word
    guard [sum, 0] that every rank's guarded Adam / EMA kernels read — all ranks skip the step
    together and the replicas stay identical.  Called once per step on every rank (one small
    all-reduce, no host synchronisation with RCCL); a rank whose trunk ran per conv contributes 0
    and still reads the global guard, so ranks never disagree on whether the collective runs."""
    plan = _plan_of(gen)
    if plan is None or not hasattr(plan, "chain"):
        return None
    chain = plan.chain
    group = _grad_group(gen)
    if group is None:
        return chain.guard_ptr if chain is not None else None
    g = plan.__dict__.get("_global_guard")
    if g is None:
        g = plan.__dict__["_global_guard"] = torch.zeros(2, dtype=torch.int32, device=_plan_device(plan))
    if chain is not None:
        flag = (chain.state[2:3] != chain.state[3:4]).to(torch.int32)
    else:
        flag = torch.zeros(1, dtype=torch.int32, device=_plan_device(plan))
    all_reduce_(flag, None if group is True else group)
    g[0:1].copy_(flag)
    return g.data_ptr()


def trunk_done_event(gen: nn.Module):
    """An event recorded on the forward's stream right after its persistent trunk kernel (None
    without one): work that must not run beside that grid may be queued behind it."""
    plan = _plan_of(gen)
    return getattr(plan, "trunk_done", None) if getattr(plan, "chain", None) is not None else None


def get_train_plan(gen: nn.Module, x: torch.Tensor) -> GeneratorTrainPlan:
    n, _, h, w = x.shape
    key = (n, h, w, str(x.device))
    plan = gen.__dict__.get("_isr_train_plan")
    if plan is None or plan.key != key:
        gen.__dict__["_isr_train_plan"] = None
        plan = GeneratorTrainPlan(gen, n, h, w, x.device)
        gen.__dict__["_isr_train_plan"] = plan
    return plan


def train_forward(gen: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """Differentiable generator forward on the HIP path (train mode)."""
    plan = get_train_plan(gen, x)
    plan.pack()
    return _GeneratorFn.apply(x.float().contiguous(), plan, *plan.params())


def enable_grad_allreduce(gen: nn.Module, group=True) -> None:
    """Average the generator's gradients over the process group inside the HIP
    backward (data parallel; `group=True` = the default group, None disables)."""
    from .models import SRGAN
    if isinstance(gen, SRGAN):
        gen = gen.res_net
    gen.__dict__["_isr_grad_group"] = group


def all_reduce_(t: torch.Tensor, group=None) -> None:
    """In-place SUM all-reduce: RCCL on device tensors; with the gloo backend (several
    ranks rehearsing on one GPU, or CPU tests) device tensors are staged through host
    memory, since gloo reduces host buffers."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)


def broadcast_params(params, src: int = 0, group=None) -> None:
    """DDP's initial sync: every parameter from rank `src` as one flat broadcast."""
    import torch.distributed as dist
    ps = [p for p in params]
    if not ps:
        return
    flat = torch.cat([p.detach().reshape(-1) for p in ps])
    if flat.is_cuda and dist.get_backend(group) == "gloo":
        h = flat.cpu()
        dist.broadcast(h, src, group=group)
        flat.copy_(h)
    else:
        dist.broadcast(flat, src, group=group)
    off = 0
    with torch.no_grad():
        for p in ps:
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()


def allreduce_mean(tensors: list, group=None) -> list:
    """Mean of `tensors` over the process group as ONE flat all-reduce (RCCL on the
    GPU, gloo in the CPU tests) — DDP's averaging with a single bucket.  Returns views
    of the reduced flat buffer, one per input tensor."""
    import torch.distributed as dist
    if not tensors:
        return []
    flat = torch.cat([t.reshape(-1) for t in tensors])
    all_reduce_(flat, group)
    flat.div_(dist.get_world_size(group))
    out, off = [], 0
    for t in tensors:
        out.append(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    return out


def allreduce_grads(params, group=None) -> None:
    """Mean of .grad over the group for modules trained outside the HIP plan
    (the discriminator): one flat all-reduce."""
    grads = [p.grad for p in params if p.grad is not None]
    for g, r in zip(grads, allreduce_mean(grads, group)):
        g.copy_(r)
