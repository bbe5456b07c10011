"""Drop-in mirror of the reference's model classes (utils/models.py).

Same class names, constructor signatures, submodule names and therefore the
same state_dict keys as the reference, so reference checkpoints load with
load_state_dict.  Forward passes on GPU tensors run on libisr's HIP kernels
(engine.py); there is deliberately no CPU compute path in the product — the
CPU restatement used for parity lives in oracle/ and is test-only.
"""
from __future__ import annotations

import math
from copy import deepcopy

import torch
from torch import nn

from . import engine, ops
from .ops import ActBuffer

LEAKY_DEFAULT = 0.01


def autopad(k, p=None, d=1):
    """utils/general.py:40-48."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


def _act(act):
    """Conv's activation rule (utils/models.py:95): True → SiLU, module → a fresh copy, else Identity."""
    if act is True:
        return nn.SiLU()
    if isinstance(act, nn.Module):
        return deepcopy(act)
    return nn.Identity()


def _slope(act: nn.Module) -> float:
    if isinstance(act, nn.Identity):
        return 1.0
    if isinstance(act, nn.LeakyReLU):
        return float(act.negative_slope)
    if isinstance(act, nn.ReLU):
        return 0.0
    raise NotImplementedError(f"activation {type(act).__name__} has no fused HIP epilogue")


def _require_cuda(x: torch.Tensor, who: str):
    if not x.is_cuda:
        raise RuntimeError(f"{who}: image_super_resolution_amd executes on the MI355X HIP kernels only; "
                           f"got a {x.device} tensor (the CPU restatement is oracle/ref_cpu.py, test-only)")


def _no_train(module: nn.Module, who: str):
    if module.training and torch.is_grad_enabled():
        raise NotImplementedError(f"{who}: use image_super_resolution_amd.train (HIP training path) for "
                                  "train-mode autograd; module forward is the inference path")


def _isr_free_state(module: nn.Module) -> dict:
    """Module state without the libisr caches (`_isr_*`: packed weights, launch plans
    holding ctypes descriptors), so deepcopy / pickling (ModelEMA, checkpoints) works
    after a forward; the copy re-packs on its first call."""
    return {k: v for k, v in module.__dict__.items() if not k.startswith("_isr_")}


class Conv(nn.Module):
    """Conv2d(bias=False) + BatchNorm2d + act (utils/models.py:75-111)."""
    store_bn = nn.Identity()

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True, dropout=0.):
        super().__init__()
        if isinstance(d, nn.Module):
            act, d = d, 1
        assert 0 <= dropout <= 1
        pad = autopad(k, p, d) if isinstance(k, int) else [autopad(k[0], p, d), autopad(k[1], p, d)]
        self.conv = nn.Conv2d(c1, c2, k, s, pad, groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2)
        self.drop = nn.Dropout(p=dropout) if dropout > 0. else nn.Identity()
        self.act = _act(act)

    def fuseforward(self):
        if isinstance(self.bn, nn.BatchNorm2d):
            self.store_bn = self.bn
            self.bn = nn.Identity()

    def defuseforward(self):
        if isinstance(self.bn, nn.Identity):
            self.bn = self.store_bn
            self.store_bn = nn.Identity()

    def forward(self, x):
        return _single_conv_forward(self, x)


class ConvWithoutBN(nn.Module):
    """Conv2d(bias=True) + act (utils/models.py:174-199)."""
    store_bn = nn.Identity()

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True, dropout=0.):
        super().__init__()
        if isinstance(d, nn.Module):
            act, d = d, 1
        pad = autopad(k, p, d) if isinstance(k, int) else [autopad(k[0], p, d), autopad(k[1], p, d)]
        self.conv = nn.Conv2d(c1, c2, k, s, pad, groups=g, dilation=d, bias=True)
        self.drop = nn.Dropout(p=dropout) if dropout > 0. else nn.Identity()
        self.act = _act(act)

    def forward(self, x):
        return _single_conv_forward(self, x)


def _conv_sd(m: nn.Module) -> dict:
    return {f"x.{k}": v for k, v in m.state_dict().items()}


def _single_conv_forward(m, x):
    _require_cuda(x, type(m).__name__)
    _no_train(m, type(m).__name__)
    c = m.conv
    if c.kernel_size != (3, 3) or c.stride != (1, 1) or c.groups != 1 or c.dilation != (1, 1):
        raise NotImplementedError("HIP conv path covers the 3x3 stride-1 convs of the SR generator")
    pc = engine._pack3(_conv_sd(m), "x", x.device)
    xb = ActBuffer.from_nchw(x.float(), pad=1)
    yb = ActBuffer.alloc(xb.n, xb.h, xb.w, pc.cout, 1, x.device)
    ops.conv3x3(xb, pc.cin, pc.w, pc.b, pc.cout, yb, slope=_slope(m.act))
    return yb.to_nchw()


class RDB(nn.Module):
    """Residual dense block (utils/models.py:245-271)."""

    def __init__(self, in_channel, growth_channel, kernel_size, act, add_rate=0., use_BN=True):
        super().__init__()
        self.add_rate = add_rate
        C = Conv if use_BN else ConvWithoutBN
        self.conv0 = C(in_channel + growth_channel * 0, growth_channel, kernel_size, 1, None, act=act)
        self.conv1 = C(in_channel + growth_channel * 1, growth_channel, kernel_size, 1, None, act=act)
        self.conv2 = C(in_channel + growth_channel * 2, growth_channel, kernel_size, 1, None, act=act)
        self.conv3 = C(in_channel + growth_channel * 3, growth_channel, kernel_size, 1, None, act=act)
        self.conv = C(in_channel + growth_channel * 4, in_channel, kernel_size, 1, None, act=False)

    def _packed(self, device):
        sd = {f"x.{k}": v for k, v in self.state_dict().items()}
        return [engine._pack3(sd, f"x.{c}", device) for c in ("conv0", "conv1", "conv2", "conv3", "conv")]

    def forward(self, x):
        _require_cuda(x, "RDB")
        _no_train(self, "RDB")
        convs = self._packed(x.device)
        src = ActBuffer.from_nchw(x.float(), pad=1, c_alloc=192)
        dst = ActBuffer.alloc(src.n, src.h, src.w, 64, 1, x.device)
        engine.rdb_forward(convs, src, dst, self.add_rate, slope=_slope(self.conv0.act))
        return dst.to_nchw()


class RRDB(nn.Module):
    """Residual-in-residual dense block (utils/models.py:298-317)."""

    def __init__(self, filters, kernel, act, add_rate=0.2, use_BN=True):
        super().__init__()
        assert 0 < add_rate <= 1, "add must be in range (0, 1]"
        hidden = filters // 2
        self.net = nn.Sequential(*[RDB(filters, hidden, kernel, act, add_rate=add_rate, use_BN=use_BN)
                                   for _ in range(3)])
        self.add_rate = add_rate

    def forward(self, x):
        _require_cuda(x, "RRDB")
        _no_train(self, "RRDB")
        convs = [r._packed(x.device) for r in self.net]
        X = ActBuffer.from_nchw(x.float(), pad=1, c_alloc=192)
        Y = ActBuffer.alloc(X.n, X.h, X.w, 192, 1, x.device)
        Z = ActBuffer.alloc(X.n, X.h, X.w, 192, 1, x.device)
        engine.rrdb_forward(convs, X, Y, Z, self.add_rate, slope=_slope(self.net[0].conv0.act))
        return X.to_nchw(0, 64)


class Scaler(nn.Module):
    """conv3x3 → PixelShuffle → act (utils/models.py:572-589)."""

    def __init__(self, in_channel, out_channel, scale_factor, kernel_size, act):
        super().__init__()
        out_channel = out_channel * (scale_factor ** 2)
        self.net = nn.Sequential(ConvWithoutBN(in_channel, out_channel, kernel_size, 1, None, act=False),
                                 nn.PixelShuffle(scale_factor), _act(act))

    def forward(self, x):
        _require_cuda(x, "Scaler")
        _no_train(self, "Scaler")
        if self.net[1].upscale_factor != 2:
            raise NotImplementedError("HIP Scaler epilogue implements PixelShuffle(2)")
        pc = engine._pack3({f"x.{k}": v for k, v in self.net[0].state_dict().items()}, "x", x.device)
        xb = ActBuffer.from_nchw(x.float(), pad=1)
        yb = ActBuffer.alloc(xb.n, 2 * xb.h, 2 * xb.w, pc.cout // 4, 1, x.device, ha=2 * xb.ha, wa=2 * xb.wa)
        ops.conv3x3(xb, pc.cin, pc.w, pc.b, pc.cout, yb, slope=_slope(self.net[2]), shuffle=2)
        return yb.to_nchw()


class _Generator(nn.Module):
    enchant = False

    def __getstate__(self):
        return _isr_free_state(self)

    def _packed(self, device) -> engine.GeneratorWeights:
        key = (str(device), ops.param_write_epoch()) + tuple((t.data_ptr(), t._version)
                                                             for t in self.state_dict().values())
        cache = self.__dict__.get("_isr_pack")
        if cache is None or cache[0] != key:
            gw = engine.pack_generator(self.state_dict(), enchant=self.enchant, add_rate=self.add_rate,
                                       device=device)
            self.__dict__["_isr_pack"] = (key, gw)
            return gw
        return cache[1]

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        _require_cuda(inputs, type(self).__name__)
        if self.training and torch.is_grad_enabled():
            # differentiable HIP path (forward saves every dense block; backward = libisr
            # dgrad / wgrad kernels), train.py:52-63 / :88-102
            from .train_engine import train_forward
            return train_forward(self, inputs)
        return engine.run_generator(self._packed(inputs.device), inputs.float())


class ResNet(_Generator):
    """RRDB generator with BN (utils/models.py:592-618)."""

    def __init__(self, num_block_resnet=16, add_rate=0.2, scaleRate=2):
        super().__init__()
        stages = scaleRate // 2
        self.add_rate = add_rate
        self.conv0 = ConvWithoutBN(3, 64, 9, 1, None, act=nn.LeakyReLU(0.2))
        self.residual = nn.Sequential(*[RRDB(64, 3, act=nn.LeakyReLU(), add_rate=add_rate)
                                        for _ in range(num_block_resnet)])
        self.conv1 = Conv(64, 64, 3, 1, None, act=False)
        self.scaler = nn.Sequential(*[Scaler(64, 64, 2, 3, nn.LeakyReLU()) for _ in range(stages)])
        self.conv2 = ConvWithoutBN(64, 3, 9, 1, act=nn.Tanh())
        for x in self.modules():
            if hasattr(x, "inplace"):
                x.inplace = True


class EResNet(_Generator):
    """RRDB generator without BN, weights x0.2 at init (utils/models.py:621-650)."""
    enchant = True

    def __init__(self, num_block_resnet=16, add_rate=0.2, scaleRate=2):
        super().__init__()
        stages = scaleRate // 2
        self.add_rate = add_rate
        self.conv0 = ConvWithoutBN(3, 64, 9, 1, None, act=nn.LeakyReLU())
        self.residual = nn.Sequential(*[RRDB(64, 3, act=nn.LeakyReLU(), add_rate=add_rate, use_BN=False)
                                        for _ in range(num_block_resnet)])
        self.conv1 = ConvWithoutBN(64, 64, 3, 1, None, act=False)
        self.scaler = nn.Sequential(*[Scaler(64, 64, 2, 3, nn.LeakyReLU()) for _ in range(stages)])
        self.conv2 = ConvWithoutBN(64, 3, 9, 1, act=nn.Tanh())
        for x in self.modules():
            if isinstance(x, nn.Conv2d):
                x.weight.data *= 0.2
            if hasattr(x, "inplace"):
                x.inplace = True


class SRGAN(nn.Module):
    """Generator wrapper (utils/models.py:653-669): keys under `res_net.`."""

    def __init__(self, deep, add_rate, enchant=False, scaleRate=2):
        super().__init__()
        self.res_net = EResNet(deep, add_rate, scaleRate) if enchant else ResNet(deep, add_rate, scaleRate=scaleRate)

    def init_weight(self, pretrained):
        """utils/models.py:659-665 — loads ckpt['ema'] of a res checkpoint (state_dict or pickled module)."""
        from .checkpoint import load_module_state
        try:
            self.res_net.load_state_dict(load_module_state(pretrained, "ema"))
            print("loaded pre-trained of Resnet")
        except Exception:
            print("Could not load Res checkpoint.")

    def forward(self, inputs):
        return self.res_net(inputs)


class ResidualBlock1(nn.Module):
    """x + Conv(act=False)(Conv(act)(x)), both convs with BN (utils/models.py:202-209)."""

    def __init__(self, in_channel, out_channel, hidden_channel, kernel, act):
        super().__init__()
        self.m = nn.Sequential(Conv(in_channel, hidden_channel, kernel, 1, None, act=act),
                               Conv(hidden_channel, out_channel, kernel, 1, None, act=False))

    def forward(self, inputs):
        _require_cuda(inputs, "ResidualBlock1")
        _no_train(self, "ResidualBlock1")
        c0, c1 = self.m[0].conv, self.m[1].conv
        if c0.kernel_size != (3, 3) or c1.kernel_size != (3, 3) or c1.out_channels != c0.in_channels:
            raise NotImplementedError("HIP ResidualBlock1 covers 3x3 blocks with out_channel == in_channel")
        p0 = engine._pack3(_conv_sd(self.m[0]), "x", inputs.device)
        p1 = engine._pack3(_conv_sd(self.m[1]), "x", inputs.device)
        xb = ActBuffer.from_nchw(inputs.float(), pad=1)
        hb = ActBuffer.alloc(xb.n, xb.h, xb.w, p0.cout, 1, inputs.device)
        yb = ActBuffer.alloc(xb.n, xb.h, xb.w, p1.cout, 1, inputs.device)
        ops.conv3x3(xb, p0.cin, p0.w, p0.b, p0.cout, hb, slope=_slope(self.m[0].act))
        ops.conv3x3(hb, p1.cin, p1.w, p1.b, p1.cout, yb, slope=1.0, r1=xb, s1=1.0)
        return yb.to_nchw()


class Denoise(nn.Module):
    """Same-resolution denoiser (utils/models.py:672-706), trained by
    `train.py --train_denoise` (train.py:204-205).  Inference runs on libisr
    (denoise.py); input height / width must be even, as in the reference."""

    def __init__(self, residual_blocks):
        super().__init__()
        act = nn.LeakyReLU(0.2)
        self.conv0 = nn.Sequential(ConvWithoutBN(3, 64, 9, 1, act=act))
        self.residual_0 = nn.Sequential(*[ResidualBlock1(64, 64, 64, 3, act=act)
                                          for _ in range(residual_blocks // 2)])
        self.residual_conv0 = ConvWithoutBN(64, 256, 3, 2, act=act)
        self.residual_1 = nn.Sequential(*[ResidualBlock1(256, 256, 256, 3, act) for _ in range(2)])
        self.residual_conv1 = nn.Sequential(nn.PixelShuffle(2), nn.LeakyReLU(0.2))
        self.residual_2 = nn.Sequential(*[ResidualBlock1(64, 64, 64, 3, act=act)
                                          for _ in range(residual_blocks // 2)])
        self.conv1 = Conv(64, 64, 3, 1, None, act=False)
        self.conv2 = nn.Sequential(ConvWithoutBN(64, 3, 9, 1, None, act=nn.Tanh()))
        for x in self.modules():
            if hasattr(x, "inplace"):
                x.inplace = True

    def __getstate__(self):
        return _isr_free_state(self)

    def _packed(self, device):
        from .denoise import pack_denoise
        key = (str(device), ops.param_write_epoch()) + tuple((t.data_ptr(), t._version)
                                                             for t in self.state_dict().values())
        cache = self.__dict__.get("_isr_pack")
        if cache is None or cache[0] != key:
            dw = pack_denoise(self.state_dict(), device=device)
            self.__dict__["_isr_pack"] = (key, dw)
            return dw
        return cache[1]

    def forward(self, inputs: torch.Tensor) -> torch.Tensor:
        _require_cuda(inputs, "Denoise")
        if self.training and torch.is_grad_enabled():
            # differentiable HIP path: train-mode BatchNorm, libisr backward (train.py:52-63)
            from .denoise import train_forward
            return train_forward(self, inputs)
        from .denoise import run_denoise
        return run_denoise(self._packed(inputs.device), inputs)


def fuse_conv_and_bn(conv: nn.Conv2d, bn: nn.BatchNorm2d) -> nn.Conv2d:
    """utils/models.py:366-406 — returns a biased Conv2d with BN folded in."""
    fused = nn.Conv2d(conv.in_channels, conv.out_channels, kernel_size=conv.kernel_size, stride=conv.stride,
                      padding=conv.padding, groups=conv.groups, bias=True).to(conv.weight.device)
    fused.requires_grad_(False)
    with torch.no_grad():  # the fused weights are leaves with no autograd history
        s = bn.weight.div(torch.sqrt(bn.eps + bn.running_var))
        fused.weight.copy_(conv.weight * s.view(-1, 1, 1, 1))
        b_conv = torch.zeros(conv.weight.size(0), device=conv.weight.device) if conv.bias is None else conv.bias
        b_bn = bn.bias - bn.weight.mul(bn.running_mean).div(torch.sqrt(bn.running_var + bn.eps))
        fused.bias.copy_(s * b_conv + b_bn)
    return fused


class Normalize(nn.Module):
    """uint8/float → (x/255 - mean)/std (utils/datasets.py:50-71)."""

    def __init__(self, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), max_pixel_value=255., dim=3):
        super().__init__()
        shape = (1, -1, 1, 1) if dim == 4 else (-1, 1, 1)
        self.register_buffer("mean", torch.tensor(list(mean)).view(*shape))
        self.register_buffer("std", torch.tensor(list(std)).view(*shape))
        self.register_buffer("max_pixel_value", torch.tensor(max_pixel_value))

    def forward(self, inputs):
        if inputs.dtype == torch.uint8:
            inputs = inputs.to(self.max_pixel_value.dtype) / self.max_pixel_value
        return (inputs - self.mean) / self.std


class TanhToArrayImage(nn.Module):
    """[-1,1] → uint8 image (utils/models.py:443-451)."""

    def __init__(self, max_pixel_value=255.):
        super().__init__()
        self.register_buffer("max_pixel_value", torch.tensor(max_pixel_value))

    def forward(self, inputs):
        return (((inputs + 1.) / 2.) * self.max_pixel_value).round().to(torch.uint8)


class Model(nn.Module):
    """Inference wrapper (utils/models.py:723-761): fuse/defuse BN, uint8 I/O via init_normalize."""
    mean = None
    std = None

    def __init__(self, model):
        super().__init__()
        self.net = model

    def init_normalize(self, mean, std):
        self.net = nn.Sequential(Normalize(mean, std, dim=4), self.net, TanhToArrayImage())

    def fuse(self):
        for m in self.modules():
            if isinstance(m, Conv) and isinstance(m.bn, nn.BatchNorm2d):
                m.conv = fuse_conv_and_bn(m.conv, m.bn)
                m.fuseforward()
        return self

    def defuse(self):
        for m in self.modules():
            if isinstance(m, Conv):
                m.defuseforward()
        return self

    def forward(self, inputs):
        net = self.net
        if (isinstance(net, nn.Sequential) and len(net) == 3 and isinstance(net[0], Normalize)
                and isinstance(net[2], TanhToArrayImage)):
            gen = net[1].res_net if isinstance(net[1], SRGAN) else net[1]
            if isinstance(gen, _Generator) and inputs.is_cuda:
                _no_train(gen, "Model")
                mean = net[0].mean.flatten().tolist()
                std = net[0].std.flatten().tolist()
                x = inputs if inputs.dtype == torch.uint8 else inputs.float()
                if x.dtype != torch.uint8:
                    # Normalize divides by 255 for uint8 input only (utils/datasets.py:65-71):
                    # float input is taken as already scaled
                    x = (x - net[0].mean) / net[0].std
                return engine.run_generator(gen._packed(inputs.device), x, out_u8=True, mean=mean, std=std)
        return net(inputs)


class ModelEMA:
    """EMA of a model's state_dict (utils/models.py:17-40)."""

    def __init__(self, model: nn.Module, decay=0.9999, tau=2000, updates=0):
        self.ema = deepcopy(model).eval()
        self.updates = updates
        self.decay = lambda x: decay * (1 - math.exp(-x / tau))
        for p in self.ema.parameters():
            p.requires_grad = False

    @torch.no_grad()
    def update(self, model: nn.Module):
        self.updates += 1
        d = self.decay(self.updates)
        msd = model.state_dict()
        ema_f = [v for v in self.ema.state_dict().values() if v.dtype.is_floating_point]
        src_f = [msd[k].detach() for k, v in self.ema.state_dict().items() if v.dtype.is_floating_point]
        # one multi-tensor lerp instead of the reference's per-tensor loop: v = v*d + (1-d)*m
        if ema_f and ema_f[0].is_cuda:
            from .optim import ema_update_
            ema_update_(ema_f, src_f, d)  # HIP multi-tensor kernel (isr_mt_lerp)
        else:
            torch._foreach_mul_(ema_f, d)
            torch._foreach_add_(ema_f, src_f, alpha=1 - d)


def sliding_window(image: torch.Tensor, step, windowSize=None):
    """utils/models.py:709-720 (same as rs.py:16-27)."""
    if windowSize is None:
        windowSize = step
    if isinstance(step, int):
        step = [step] * 2
    step = list(step)
    step[0] = min(image.shape[-2], step[0])
    step[1] = min(image.shape[-1], step[1])
    for y in range(0, image.shape[-2], step[0]):
        for x in range(0, image.shape[-1], step[1]):
            yield step, x, y, image[..., y:y + windowSize, x:x + windowSize]


class Discriminator(nn.Module):
    """SRGAN discriminator (utils/models.py:513-569).  In train mode on the GPU the
    eight conv blocks (incl. the stride-2 ones and train-mode BatchNorm) run on
    libisr (discriminator.py); the adaptive pool and the two Linear layers are
    torch ops.  `use_libisr(False)` (or eval mode) runs the stock modules: at
    [16,3,512,512] the libisr stack is at parity with MIOpen NHWC + find mode
    (8.5-8.8 vs 8.5-9.2 ms fwd+bwd, tools/bench_disc.py), 2 % faster in the full
    SRGAN step, and needs no MIOpen kernel search at start-up."""

    def __init__(self, kernel_size=3, n_channels=64, n_blocks=8, fc_size=1024):
        super().__init__()
        in_channels = 3
        blocks = []
        out_channels = 0
        for i in range(n_blocks):
            out_channels = (n_channels if i == 0 else in_channels * 2) if i % 2 == 0 else in_channels
            stride = 1 if i % 2 == 0 else 2
            if i == 0:
                blocks.append(_TorchConv(in_channels, out_channels, kernel_size, stride, bn=False, slope=0.2))
            else:
                blocks.append(_TorchConv(in_channels, out_channels, kernel_size, stride, bn=True, slope=0.2))
            in_channels = out_channels
        self.conv_blocks = nn.Sequential(*blocks)
        self.adaptive_pool = nn.AdaptiveAvgPool2d((6, 6))
        self.fc1 = nn.Sequential(nn.Linear(out_channels * 6 ** 2, fc_size), nn.LeakyReLU(0.2))
        self.fc2 = nn.Linear(fc_size, 1)

    def use_libisr(self, enable: bool = True) -> "Discriminator":
        self.__dict__["hip"] = bool(enable)
        return self

    def forward(self, inputs):
        b = inputs.size(0)
        if self.training and inputs.is_cuda and self.__dict__.get("hip", True):
            from .discriminator import conv_stack_train
            feat = conv_stack_train(self, inputs)
            out = _adaptive_pool_mm(feat, self.adaptive_pool.output_size)
        else:
            feat = self.conv_blocks(inputs)
            out = self.adaptive_pool(feat)
        return self.fc2(self.fc1(out.reshape(b, -1)))


def _pool_matrix(h: int, w: int, oh: int, ow: int, device) -> torch.Tensor:
    """[h*w, oh*ow] averaging matrix of nn.AdaptiveAvgPool2d((oh, ow)) (window i: rows
    floor(i*h/oh) .. ceil((i+1)*h/oh))."""
    P = torch.zeros(h * w, oh * ow, dtype=torch.float32)
    for i in range(oh):
        r0, r1 = (i * h) // oh, -((-(i + 1) * h) // oh)
        for j in range(ow):
            c0, c1 = (j * w) // ow, -((-(j + 1) * w) // ow)
            v = 1.0 / ((r1 - r0) * (c1 - c0))
            for r in range(r0, r1):
                P[r * w + c0:r * w + c1, i * ow + j] = v
    return P.to(device)


_POOL_MATS: dict = {}


def _adaptive_pool_mm(feat: torch.Tensor, size) -> torch.Tensor:
    """AdaptiveAvgPool2d as one fp32 matmul (utils/models.py:548, :567 — the pooling on the
    discriminator's training path): its backward is the transposed matmul instead of
    ATen's atomic scatter (0.18 ms per call at [16, 512, 32, 32] -> 6x6)."""
    oh, ow = (size, size) if isinstance(size, int) else size
    n, c, h, w = feat.shape
    key = (h, w, oh, ow, str(feat.device))
    P = _POOL_MATS.get(key)
    if P is None:
        P = _POOL_MATS[key] = _pool_matrix(h, w, oh, ow, feat.device)
    with torch.autocast("cuda", enabled=False):
        return (feat.float().reshape(n * c, h * w) @ P).reshape(n, c, oh, ow)


class _TorchConv(nn.Module):
    """Conv / ConvWithoutBN key layout (conv, bn, act) evaluated with stock ops (discriminator only)."""

    def __init__(self, c1, c2, k, s, bn: bool, slope: float):
        super().__init__()
        self.conv = nn.Conv2d(c1, c2, k, s, k // 2, bias=not bn)
        if bn:
            self.bn = nn.BatchNorm2d(c2)
        self.drop = nn.Identity()
        self.act = nn.LeakyReLU(slope, inplace=True)

    def forward(self, x):
        x = self.conv(x)
        if hasattr(self, "bn"):
            x = self.bn(x)
        return self.act(x)
