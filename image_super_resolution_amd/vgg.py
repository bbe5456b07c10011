"""TruncatedVGG19 on libisr — the perceptual-loss feature extractor
(utils/models.py:454-510, used by gen_loss utils/loss.py:7-24).

Same module tree and state_dict keys as the reference (`truncated_vgg19.{idx}.
weight/bias`, torchvision's vgg19.features indices).  The reference downloads
ImageNet weights from torchvision; there is no network here, so the weights
come from a local torchvision-format file when one is given (loaded with
weights_only=True) and are otherwise He-initialised from a fixed seed — the
layer graph, truncation rule and numerics are the reference's either way.

On CUDA tensors the forward runs as a torch.autograd.Function over HIP kernels:
conv3x3 (+bias +ReLU fused, slope 0) and maxpool2 on channel-blocked bf16
buffers; its backward is the input gradient only (the VGG is frozen,
utils/loss.py:9-11): dgrad convs whose epilogue applies ReLU' of the layer
below, and maxpool2 backward with the ReLU' fused.
"""
from __future__ import annotations

import ctypes
import os
import warnings

import torch
from torch import nn

from . import ops
from ._lib import load as _load_lib
from .ops import ActBuffer, round_up, TILE_H, TILE_W

VGG19_CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def vgg19_features() -> list[nn.Module]:
    """torchvision vgg19().features layer list (cfg 'E')."""
    layers, cin = [], 3
    for v in VGG19_CFG:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return layers


def truncate_index(i: int, j: int) -> int:
    """utils/models.py:473-493: index just past the j-th conv after the (i-1)-th maxpool."""
    maxpool_counter = conv_counter = truncate_at = 0
    for layer in vgg19_features():
        truncate_at += 1
        if isinstance(layer, nn.Conv2d):
            conv_counter += 1
        if isinstance(layer, nn.MaxPool2d):
            maxpool_counter += 1
            conv_counter = 0
        if maxpool_counter == i - 1 and conv_counter == j:
            break
    if not (maxpool_counter == i - 1 and conv_counter == j):
        raise ValueError(f"One or both of i={i} and j={j} are not valid choices for the VGG19!")
    return truncate_at


class TruncatedVGG19(nn.Module):
    """utils/models.py:454-510.  `weights`: path to a torchvision vgg19 state_dict
    (`features.N.*` keys) or to a TruncatedVGG19 state_dict; default: the
    ISR_VGG19_WEIGHTS environment variable, else seeded He init."""

    def __init__(self, i, j, beforeActivation=True, weights: str | None = None, seed: int = 0):
        super().__init__()
        truncate_at = truncate_index(i, j)
        pad = 0 if beforeActivation else 1
        self.truncated_vgg19 = nn.Sequential(*vgg19_features()[:truncate_at + pad])
        self.before_act = bool(beforeActivation)
        path = weights or os.environ.get("ISR_VGG19_WEIGHTS")
        if path:
            from .checkpoint import load_checkpoint
            sd = load_checkpoint(path)
            sd = {k.replace("features.", "truncated_vgg19.", 1): v for k, v in sd.items()}
            own = self.state_dict()
            self.load_state_dict({k: sd[k] for k in own}, strict=True)
        else:
            warnings.warn("TruncatedVGG19: no pretrained VGG19 weights available offline; using seeded He init "
                          "(set ISR_VGG19_WEIGHTS to a torchvision vgg19 state_dict file)", stacklevel=2)
            g = torch.Generator().manual_seed(seed)
            for m in self.truncated_vgg19:
                if isinstance(m, nn.Conv2d):
                    fan_in = m.in_channels * 9
                    with torch.no_grad():
                        m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_in) ** 0.5)
                        m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.01)
        for p in self.parameters():
            p.requires_grad = False

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        if not inputs.is_cuda:
            raise RuntimeError("TruncatedVGG19: the HIP feature extractor needs a GPU tensor "
                               "(CPU restatement: oracle/ref_cpu.vgg_truncated, test-only)")
        # inputs that need a gradient get their own plan (activations kept for the
        # backward); the HR pass of calc_contentLoss (no grad) must not overwrite them
        needs_grad = inputs.requires_grad and torch.is_grad_enabled()
        plan = _get_plan(self, inputs, needs_grad)
        return _VGGFn.apply(inputs.float().contiguous(), plan)


class VGGPlan:
    """Buffers, packed weights and descriptors of the truncated VGG for one (n, h, w)."""

    def __init__(self, vgg: TruncatedVGG19, n: int, h: int, w: int, device):
        self.key = (n, h, w, str(device))
        dev = torch.device(device)
        self.device = dev
        self.lib = _load_lib()
        mods = list(vgg.truncated_vgg19)
        # geometry per level: valid (h, w) and computed (ha, wa) with ha_l >= 2 * ha_{l+1}
        levels = 1 + sum(isinstance(m, nn.MaxPool2d) for m in mods)
        hs = [h >> k for k in range(levels)]
        ws = [w >> k for k in range(levels)]
        ha = [0] * levels
        wa = [0] * levels
        for k in range(levels - 1, -1, -1):
            ha[k] = max(round_up(hs[k], TILE_H), 2 * ha[k + 1] if k + 1 < levels else 0)
            wa[k] = max(round_up(ws[k], TILE_W), 2 * wa[k + 1] if k + 1 < levels else 0)
        if min(hs[-1], ws[-1]) < 1 or any(hs[k] % 2 or ws[k] % 2 for k in range(levels - 1)):
            raise ValueError(f"TruncatedVGG19 HIP path needs h, w divisible by {2 ** (levels - 1)}")

        def buf(level, c):
            return ActBuffer.alloc(n, hs[level], ws[level], c, 1, dev, ha=ha[level], wa=wa[level])

        self.x = buf(0, 16)  # 3 input channels, padded to one 16-channel plane
        self.gx32 = buf(0, 32)
        # layer program
        self.steps = []   # ("conv", conv_mod, in_buf, out_buf, relu) | ("pool", in_buf, out_buf, c)
        cur, level, c = self.x, 0, 16
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, nn.Conv2d):
                relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                out = buf(level, m.out_channels)
                self.steps.append(["conv", m, cur, out, relu])
                cur, c = out, m.out_channels
                i += 2 if relu else 1
            elif isinstance(m, nn.MaxPool2d):
                level += 1
                out = buf(level, c)
                self.steps.append(["pool", cur, out, c])
                cur = out
                i += 1
            else:
                raise NotImplementedError(f"VGG layer {type(m).__name__}")
        self.out = cur
        self.out_c = c
        self.out_relu = self.steps[-1][0] == "conv" and self.steps[-1][4]
        # gradient buffers mirror the activations
        self.g = {id(s[3] if s[0] == "conv" else s[2]): None for s in self.steps}
        self._pack(vgg)
        self._build()

    def _pack(self, vgg):
        self.packs = []
        for s in self.steps:
            if s[0] != "conv":
                continue
            m = s[1]
            wt = m.weight.detach().to(self.device, torch.float32)
            b = m.bias.detach().to(self.device, torch.float32).contiguous()
            cin = m.in_channels
            if cin % 16:  # first layer: 3 input channels → one padded plane (forward), 32 (dgrad output)
                w16 = torch.zeros(wt.shape[0], 16, 3, 3, device=self.device)
                w16[:, :cin] = wt
                w32 = torch.zeros(wt.shape[0], 32, 3, 3, device=self.device)
                w32[:, :cin] = wt
                fwd, bwd = ops.pack_conv3x3(w16), ops.pack_conv3x3_dgrad(w32)
            else:
                fwd, bwd = ops.pack_conv3x3(wt), ops.pack_conv3x3_dgrad(wt)
            self.packs.append((fwd, bwd, b))
        self.version = _weights_version(vgg)

    def _build(self):
        F, B = [], []
        lib = self.lib
        pi = 0
        conv_meta = []
        for s in self.steps:
            if s[0] == "conv":
                m, xin, out, relu = s[1], s[2], s[3], s[4]
                fwd, bwd, b = self.packs[pi]
                pi += 1
                cin = xin.c if m.in_channels % 16 else m.in_channels
                F.append((lib.isr_conv3x3_fwd, ops.conv3x3_desc(xin, cin, fwd, b, m.out_channels, out,
                                                                 slope=0.0 if relu else 1.0)))
                conv_meta.append((m, xin, out, relu, bwd))
            else:
                xin, out, c = s[1], s[2], s[3]
                F.append((lib.isr_maxpool2_fwd, ops.pool_desc(xin, out, c)))
        self.fwd_launches = F
        # backward, reverse order.  gbuf[id(activation buffer)] = gradient wrt that activation
        # (already multiplied by the ReLU' of the layer that produced it).
        gb = {}
        n = self.x.n

        def gbuf_like(a: ActBuffer) -> ActBuffer:
            if id(a) not in gb:
                gb[id(a)] = ActBuffer.alloc(n, a.h, a.w, a.c, 1, self.device, ha=a.ha, wa=a.wa)
            return gb[id(a)]

        self.gout = gbuf_like(self.out)
        steps = self.steps
        producer = {}  # activation buffer id → step producing it
        for s in steps:
            producer[id(s[3] if s[0] == "conv" else s[2])] = s
        for k in range(len(steps) - 1, -1, -1):
            s = steps[k]
            if s[0] == "conv":
                m, xin, out, relu = s[1], s[2], s[3], s[4]
                bwd = next(c[4] for c in conv_meta if c[0] is m)
                g_in_out = gb[id(out)]
                if xin is self.x:  # first conv: input gradient, 3 of 32 channels meaningful
                    B.append((lib.isr_conv3x3_fwd, ops.conv3x3_desc(g_in_out, m.out_channels, bwd, None, 32,
                                                                     self.gx32)))
                    continue
                prev = producer[id(xin)]
                gprev = gbuf_like(xin)
                if prev[0] == "conv":  # ReLU' of the conv that produced xin, fused in the epilogue
                    kw = dict(m=xin, mslope=0.0) if prev[4] else {}
                    B.append((lib.isr_conv3x3_fwd, ops.conv3x3_desc(g_in_out, m.out_channels, bwd, None,
                                                                     m.in_channels, gprev, **kw)))
                else:
                    B.append((lib.isr_conv3x3_fwd, ops.conv3x3_desc(g_in_out, m.out_channels, bwd, None,
                                                                     m.in_channels, gprev)))
            else:
                xin, out, c = s[1], s[2], s[3]
                pre = producer[id(xin)]
                relu = pre[0] == "conv" and pre[4]
                B.append((lib.isr_maxpool2_bwd, ops.pool_desc(xin, gb[id(out)], c, gbuf_like(xin),
                                                              mslope=0.0 if relu else 1.0)))
        self.bwd_launches = B
        self.gbufs = gb

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        st = ops._stream()
        ops.nchw_to_blocked(x, self.x)
        for fn, d in self.fwd_launches:
            rc = fn(ctypes.byref(d), st)
            if rc != 0:
                ops.check(rc, "vgg forward")
        o = self.out
        feats = torch.empty(o.n, self.out_c, o.h, o.w, device=self.device)
        return ops.blocked_to_nchw(o, feats)

    def backward(self, gfeat: torch.Tensor) -> torch.Tensor:
        st = ops._stream()
        kw = dict(m=self.out, mslope=0.0) if self.out_relu else {}
        ops.nchw_to_blocked(gfeat.contiguous().float(), self.gout, **kw)
        for fn, d in self.bwd_launches:
            rc = fn(ctypes.byref(d), st)
            if rc != 0:
                ops.check(rc, "vgg backward")
        gx = torch.empty(self.x.n, 3, self.x.h, self.x.w, device=self.device)
        return ops.blocked_to_nchw(self.gx32, gx)


def _weights_version(vgg) -> tuple:
    return tuple((p.data_ptr(), p._version) for p in vgg.parameters())


def _get_plan(vgg: TruncatedVGG19, x: torch.Tensor, needs_grad: bool) -> VGGPlan:
    n, c, h, w = x.shape
    if c != 3:
        raise ValueError("TruncatedVGG19 expects 3-channel input")
    key = (n, h, w, str(x.device), needs_grad)
    plans = vgg.__dict__.setdefault("_isr_plans", {})
    plan = plans.get(key)
    if plan is None or plan.version != _weights_version(vgg):
        plan = VGGPlan(vgg, n, h, w, x.device)
        plans[key] = plan
    return plan


class _VGGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan):
        ctx.plan = plan
        return plan.forward(x)

    @staticmethod
    def backward(ctx, g):
        return ctx.plan.backward(g), None
