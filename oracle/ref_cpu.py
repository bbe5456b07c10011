"""ORACLE — test infrastructure only, never shipped or measured.

CPU fp32 restatement of thnak/image_super_resolution's hot path, written from
the reference's behaviour as a functional graph over a state_dict (reference
key names).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module, and only as the checker / the timed CPU baseline.

Pinned against golden vectors produced by running the reference itself in the
survey container (tests/golden/make_golden.py → tests/golden/*.npz; checked by
tests/test_oracle_golden.py).  Citations are file:line in the reference.
"""
from __future__ import annotations

import math
from typing import Iterator

import torch
import torch.nn.functional as F

BN_EPS = 1e-5  # nn.BatchNorm2d default (utils/models.py:93)
LEAKY_DEFAULT = 0.01  # nn.LeakyReLU() default slope (utils/models.py:598, :605, :627)


# --------------------------------------------------------------------- blocks
def conv_unit(sd: dict, prefix: str, x: torch.Tensor, slope: float | None, train_bn: bool = False,
              bn_momentum: float = 0.1) -> torch.Tensor:
    """Conv (utils/models.py:75-111) or ConvWithoutBN (:174-199) forward.

    act(bn(conv(x))) with 'same' padding k//2 (autopad, utils/general.py:40-48);
    BN present iff `{prefix}.bn.weight` is in the state_dict (after Model.fuse
    the BN moves to store_bn and the conv carries the folded bias, :741-751).
    slope=None → Identity (act=False), else LeakyReLU(slope).
    """
    w = sd[f"{prefix}.conv.weight"]
    b = sd.get(f"{prefix}.conv.bias")
    y = F.conv2d(x, w, b, stride=1, padding=w.shape[-1] // 2)
    if f"{prefix}.bn.weight" in sd:
        y = F.batch_norm(y, sd[f"{prefix}.bn.running_mean"], sd[f"{prefix}.bn.running_var"],
                         sd[f"{prefix}.bn.weight"], sd[f"{prefix}.bn.bias"], training=train_bn,
                         momentum=bn_momentum, eps=BN_EPS)
    if slope is not None:
        y = F.leaky_relu(y, slope)
    return y


def rdb(sd: dict, prefix: str, x: torch.Tensor, add_rate: float, train_bn: bool = False) -> torch.Tensor:
    """RDB.forward (utils/models.py:265-271): dense growth-32 block, 5 convs."""
    o0 = conv_unit(sd, f"{prefix}.conv0", x, LEAKY_DEFAULT, train_bn)
    o1 = conv_unit(sd, f"{prefix}.conv1", torch.cat([x, o0], 1), LEAKY_DEFAULT, train_bn)
    o2 = conv_unit(sd, f"{prefix}.conv2", torch.cat([x, o0, o1], 1), LEAKY_DEFAULT, train_bn)
    o3 = conv_unit(sd, f"{prefix}.conv3", torch.cat([x, o0, o1, o2], 1), LEAKY_DEFAULT, train_bn)
    o4 = conv_unit(sd, f"{prefix}.conv", torch.cat([x, o0, o1, o2, o3], 1), None, train_bn)
    return o4 * add_rate + x


def rrdb(sd: dict, prefix: str, x: torch.Tensor, add_rate: float, train_bn: bool = False) -> torch.Tensor:
    """RRDB.forward (utils/models.py:316-317): 3 RDBs, net(x)*add_rate + x."""
    y = x
    for r in range(3):
        y = rdb(sd, f"{prefix}.net.{r}", y, add_rate, train_bn)
    return y * add_rate + x


def scaler(sd: dict, prefix: str, x: torch.Tensor) -> torch.Tensor:
    """Scaler (utils/models.py:572-589): conv3x3 64→256 (+bias) → PixelShuffle(2) → LeakyReLU()."""
    y = conv_unit(sd, f"{prefix}.net.0", x, None)
    return F.leaky_relu(F.pixel_shuffle(y, 2), LEAKY_DEFAULT)


def generator(sd: dict, x: torch.Tensor, *, num_blocks: int, scale: int, enchant: bool = False,
              add_rate: float = 0.2, prefix: str = "", train_bn: bool = False) -> torch.Tensor:
    """ResNet.forward (utils/models.py:592-618) / EResNet.forward (:621-650).

    `scale` is the constructor's scaleRate: scaleRate//2 PixelShuffle(2)
    stages (:595, :624).  conv0 slope 0.2 for ResNet (:596), 0.01 for EResNet
    (:625).  Output in [-1, 1] (tanh, :607).
    """
    p = f"{prefix}." if prefix else ""
    feat = conv_unit(sd, f"{p}conv0", x, LEAKY_DEFAULT if enchant else 0.2, train_bn)
    y = feat
    for i in range(num_blocks):
        y = rrdb(sd, f"{p}residual.{i}", y, add_rate, train_bn)
    y = feat + conv_unit(sd, f"{p}conv1", y, None, train_bn)
    for s in range(scale // 2):
        y = scaler(sd, f"{p}scaler.{s}", y)
    w = sd[f"{p}conv2.conv.weight"]
    return torch.tanh(F.conv2d(y, w, sd[f"{p}conv2.conv.bias"], padding=w.shape[-1] // 2))


def residual_block1(sd: dict, prefix: str, x: torch.Tensor, slope: float = 0.2, train_bn: bool = False) -> torch.Tensor:
    """ResidualBlock1.forward (utils/models.py:202-209): x + Conv(act=False)(Conv(act)(x))."""
    h = conv_unit(sd, f"{prefix}.m.0", x, slope, train_bn)
    return x + conv_unit(sd, f"{prefix}.m.1", h, None, train_bn)


def denoise(sd: dict, x: torch.Tensor, train_bn: bool = False) -> torch.Tensor:
    """Denoise.forward (utils/models.py:695-706); every act is LeakyReLU(0.2) (:676-690).

    conv0 9x9 → residual_0 → residual_conv0 (3x3 stride 2, pad 1, +bias, act)
    → residual_1 (256 ch) → PixelShuffle(2) + act → residual_2 → conv1 + trunk → conv2 9x9 + tanh."""
    def chain(name, y):
        n = len({int(k[len(name) + 1:].split(".")[0]) for k in sd if k.startswith(name + ".")})
        for i in range(n):
            y = residual_block1(sd, f"{name}.{i}", y, train_bn=train_bn)
        return y

    feat = conv_unit(sd, "conv0.0", x, 0.2)
    r = chain("residual_0", feat)
    r = F.leaky_relu(F.conv2d(r, sd["residual_conv0.conv.weight"], sd["residual_conv0.conv.bias"], stride=2,
                              padding=1), 0.2)
    r = chain("residual_1", r)
    r = F.leaky_relu(F.pixel_shuffle(r, 2), 0.2)
    r = chain("residual_2", r)
    y = feat + conv_unit(sd, "conv1", r, None, train_bn)
    w = sd["conv2.0.conv.weight"]
    return torch.tanh(F.conv2d(y, w, sd["conv2.0.conv.bias"], padding=w.shape[-1] // 2))


def count_blocks(sd: dict, prefix: str = "") -> int:
    p = f"{prefix}." if prefix else ""
    idx = {int(k[len(p) + len("residual."):].split(".")[0]) for k in sd if k.startswith(f"{p}residual.")}
    return len(idx)


# --------------------------------------------------------------- inference I/O
def fold_bn(w: torch.Tensor, b: torch.Tensor | None, gamma, beta, mean, var, eps=BN_EPS):
    """fuse_conv_and_bn (utils/models.py:366-406): W' = diag(g/sqrt(var+eps)) W,
    b' = diag(g/sqrt(var+eps)) b + (beta - g*mean/sqrt(var+eps))."""
    s = gamma / torch.sqrt(eps + var)
    w2 = w * s.view(-1, *([1] * (w.dim() - 1)))
    b0 = torch.zeros(w.shape[0]) if b is None else b
    b2 = s * b0 + (beta - gamma * mean / torch.sqrt(var + eps))
    return w2, b2


def fuse_state_dict(sd: dict) -> dict:
    """Model.fuse (utils/models.py:741-751) as a state_dict transform."""
    out = {}
    bn_prefixes = {k[: -len(".bn.weight")] for k in sd if k.endswith(".bn.weight")}
    for k, v in sd.items():
        pre = next((p for p in bn_prefixes if k.startswith(p + ".bn.")), None)
        if pre is not None:
            continue
        out[k] = v
    for p in bn_prefixes:
        w, b = fold_bn(sd[f"{p}.conv.weight"], sd.get(f"{p}.conv.bias"), sd[f"{p}.bn.weight"], sd[f"{p}.bn.bias"],
                       sd[f"{p}.bn.running_mean"], sd[f"{p}.bn.running_var"])
        out[f"{p}.conv.weight"] = w
        out[f"{p}.conv.bias"] = b
    return out


def normalize_u8(img: torch.Tensor, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)) -> torch.Tensor:
    """Normalize.forward (utils/datasets.py:65-71) on uint8 NCHW: /255, -mean, /std."""
    x = img.to(torch.float32) / 255.0
    m = torch.tensor(mean).view(1, -1, 1, 1)
    s = torch.tensor(std).view(1, -1, 1, 1)
    return (x - m) / s


def tanh_to_u8(y: torch.Tensor) -> torch.Tensor:
    """TanhToArrayImage.forward (utils/models.py:448-451): ((y+1)/2*255).round() → uint8."""
    return (((y + 1.0) / 2.0) * 255.0).round().to(torch.uint8)


def model_u8(sd: dict, img: torch.Tensor, **gen_kw) -> torch.Tensor:
    """Model(net).init_normalize(mean, std) (utils/models.py:731-732): uint8 → uint8."""
    return tanh_to_u8(generator(sd, normalize_u8(img), **gen_kw))


# ------------------------------------------------------------ tiled inference
def sliding_window(image: torch.Tensor, step: int) -> Iterator[tuple[list[int], int, int, torch.Tensor]]:
    """rs.py:16-27 — non-overlapping windows, raster order, step clamped to the image."""
    window = step
    st = [min(image.shape[-2], step), min(image.shape[-1], step)]
    for y in range(0, image.shape[-2], st[0]):
        for x in range(0, image.shape[-1], st[1]):
            yield st, x, y, image[..., y:y + window, x:x + window]


def tiled_u8(model, image: torch.Tensor, window: int) -> torch.Tensor:
    """rs.py:78-111 image branch: run `model` (uint8 [1,3,h,w] → uint8) per window
    and paste with the reference's cursor logic."""
    c, h, w = image.shape
    result = None
    image_width = 0
    high, width = 0, 0
    for step, _, _, win in sliding_window(image, window):
        out = model(win.unsqueeze(0))
        r_b, r_c, r_h, r_w = out.shape
        if result is None:
            if step[0] == r_h:
                result = torch.zeros_like(image)
            else:
                sf = r_h / step[0]
                result = torch.zeros([r_c, int(h * sf), int(w * sf)], dtype=torch.uint8)
            _, _, image_width = result.shape
        for frame in out:
            fc, fh, fw = frame.shape
            result[..., high:high + fh, width:width + fw] = frame
            width += fw
            if width >= image_width:
                high += fh
                width = 0
    return result


# ---------------------------------------------------------------- metrics
def psnr(a: torch.Tensor, b: torch.Tensor, peak: float = 2.0) -> float:
    """PSNR in dB on [-1,1] tanh space (peak 2) — SURVEY.md §8d parity metric."""
    mse = torch.mean((a.double() - b.double()) ** 2).item()
    return float("inf") if mse == 0 else 10.0 * math.log10(peak * peak / mse)


def y_channel(img01: torch.Tensor) -> torch.Tensor:
    """BT.601 luma as in Ychannel (utils/datasets.py:159-166), input RGB in [0,1]."""
    r, g, b = img01[:, 0], img01[:, 1], img01[:, 2]
    return (65.481 * r + 128.553 * g + 24.966 * b + 16.0) / 255.0


def psnr_y(a01: torch.Tensor, b01: torch.Tensor, border: int = 4) -> float:
    ya = y_channel(a01)[..., border:-border, border:-border]
    yb = y_channel(b01)[..., border:-border, border:-border]
    return psnr(ya, yb, peak=1.0)


# ----------------------------------------------------------------- losses
def l1_loss(a, b, weight: float = 1.0):
    """L1Loss.forward (utils/loss.py:38-39): sum(weight * mean|a-b|)."""
    return torch.sum(torch.tensor([weight]) * F.l1_loss(a, b))


def vgg19_features_cfg():
    """torchvision vgg19 'E' feature layout: (kind, cin, cout) per layer index."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(("pool", None, None))
        else:
            layers.append(("conv", cin, v))
            layers.append(("relu", None, None))
            cin = v
    return layers


def truncate_index(i: int, j: int) -> int:
    """TruncatedVGG19.__init__ truncation counter (utils/models.py:473-493)."""
    maxpool_counter = conv_counter = truncate_at = 0
    for kind, _, _ in vgg19_features_cfg():
        truncate_at += 1
        if kind == "conv":
            conv_counter += 1
        if kind == "pool":
            maxpool_counter += 1
            conv_counter = 0
        if maxpool_counter == i - 1 and conv_counter == j:
            break
    if not (maxpool_counter == i - 1 and conv_counter == j):
        raise ValueError(f"invalid (i, j) = ({i}, {j}) for VGG19")
    return truncate_at


def vgg_truncated(sd: dict, x: torch.Tensor, i: int = 5, j: int = 4, before_act: bool = False) -> torch.Tensor:
    """TruncatedVGG19.forward (utils/models.py:502-510) over `truncated_vgg19.{idx}.*` keys."""
    n_layers = truncate_index(i, j) + (0 if before_act else 1)
    y = x
    for idx, (kind, _, _) in enumerate(vgg19_features_cfg()[:n_layers]):
        if kind == "conv":
            y = F.conv2d(y, sd[f"truncated_vgg19.{idx}.weight"], sd[f"truncated_vgg19.{idx}.bias"], padding=1)
        elif kind == "relu":
            y = F.relu(y)
        else:
            y = F.max_pool2d(y, 2, 2)
    return y


def content_loss(sd_vgg: dict, sr: torch.Tensor, hr: torch.Tensor, sr_disc: torch.Tensor, beta: float = 1e-3,
                 before_act: bool = False):
    """gen_loss.calc_contentLoss (utils/loss.py:16-24): (perceptual, adversarial, content)."""
    fs = vgg_truncated(sd_vgg, sr, before_act=before_act)
    fh = vgg_truncated(sd_vgg, hr, before_act=before_act).detach()
    content = l1_loss(fs, fh) if before_act else F.mse_loss(fs, fh)
    adv = F.binary_cross_entropy_with_logits(sr_disc, torch.ones_like(sr_disc))
    return content + beta * adv, adv, content


def adv_loss(sr_disc: torch.Tensor, hr_disc: torch.Tensor):
    """gen_loss.calc_advLoss (utils/loss.py:26-29)."""
    return (F.binary_cross_entropy_with_logits(sr_disc, torch.zeros_like(sr_disc))
            + F.binary_cross_entropy_with_logits(hr_disc, torch.ones_like(hr_disc)))


def ema_decay(updates: int, tau: float, decay: float = 0.9999) -> float:
    """ModelEMA.decay (utils/models.py:27)."""
    return decay * (1 - math.exp(-updates / tau))


# ------------------------------------------------------------------ data (LR)
def cv2_resize_linear_u8(img, scale: int):
    """SR_dataset's LR resize (utils/datasets.py:302-303: albumentations.Resize, whose default
    interpolation is cv2.INTER_LINEAR) of a uint8 [..., H, W] array by an integer factor.
    Third-party: albumentations / OpenCV, absent here and unpinned in the reference
    (no requirements file) — restated from OpenCV's uint8 resize: destination pixel d samples
    src = scale*(d + 0.5) - 0.5 with 11-bit fixed-point weights (INTER_RESIZE_COEF_SCALE 2048)
    and rounds the 22-bit product half up; a x2 downscale runs as INTER_AREA (2x2 mean, also
    rounded half up).  At integer factors the weights are 0 / 0.5 / 1, so an even factor
    averages the centre 2x2 of each block, an odd one picks its centre pixel.  Parity
    unpinned (no cv2 to generate golden vectors)."""
    import numpy as np
    a = np.asarray(img).astype(np.int64)
    H, W = a.shape[-2], a.shape[-1]
    h, w = H // scale, W // scale
    if scale % 2:
        c = (scale - 1) // 2
        return a[..., c::scale, c::scale][..., :h, :w].astype(np.uint8)
    c = scale // 2 - 1
    s = (a[..., c::scale, c::scale][..., :h, :w] + a[..., c + 1::scale, c::scale][..., :h, :w]
         + a[..., c::scale, c + 1::scale][..., :h, :w] + a[..., c + 1::scale, c + 1::scale][..., :h, :w])
    return ((s * (1 << 20) + (1 << 21)) >> 22).astype(np.uint8)
