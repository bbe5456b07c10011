"""Generate golden vectors by running the REFERENCE itself (thnak/image_super_resolution).

Runs only where /root/reference exists (the survey container); the GPU box and
the test suite only read the committed .npz outputs.  The reference's missing
third-party modules (torchvision, cv2, albumentations, termcolor) are replaced
by inert stubs — except torchvision.models.vgg19, which is stubbed with a
locally built VGG19 'E' feature stack because ImageNet weights cannot be
downloaded (parity with the real VGG19 weights is therefore unpinned; the
truncation / loss logic is the reference's own).  Every weight comes from
image_super_resolution_amd.weights.synth_state_dict, so tests rebuild the same
weights from (key, shape, seed) instead of storing them.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only-denoise]
"""
from __future__ import annotations

import os
import sys
import types
from pathlib import Path

import numpy as np
import torch
from torch import nn

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent
ROOT = OUT.parents[1]
sys.dont_write_bytecode = True
sys.path.insert(0, str(ROOT))
from image_super_resolution_amd.weights import synth_lr_batch, synth_state_dict, normalize  # noqa: E402


# ------------------------------------------------------------------ stubs
class _Inert:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return self

    def __getattr__(self, n):
        return _Inert()


def _stub(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


def _local_vgg19(weights=None):
    """torchvision vgg19 'E' features built locally (same layer indices)."""
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    m = nn.Module()
    m.features = nn.Sequential(*layers)
    return m


_IO = {}


def install_stubs():
    tv = _stub("torchvision")
    tvt = _stub("torchvision.transforms", InterpolationMode=_Inert(), Lambda=_Inert, Compose=_Inert)
    tv.transforms = tvt
    tvt.functional = _stub("torchvision.transforms.functional", resize=None, InterpolationMode=_Inert())
    tv.io = _stub("torchvision.io", read_image=lambda p, mode=None: _IO["image"].clone(),
                  write_png=lambda t, p: _IO.__setitem__("png", t.clone()),
                  VideoReader=None, ImageReadMode=_Inert())
    tv.models = _stub("torchvision.models", vgg19=_local_vgg19, VGG19_Weights=_Inert())
    _stub("cv2")
    alb = _stub("albumentations")
    alb.pytorch = _stub("albumentations.pytorch", ToTensorV2=_Inert)
    _stub("termcolor", colored=lambda s, *a, **k: s)
    sys.path.insert(0, str(REF))


def load_synth(model: nn.Module, seed: int = 0) -> nn.Module:
    model.load_state_dict(synth_state_dict(model.state_dict(), seed))
    return model


def np32(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


def main():
    if not REF.exists():
        raise SystemExit("reference not present: golden vectors can only be regenerated in the survey container")
    install_stubs()
    import utils.models as M  # reference
    import utils.loss as L  # reference
    import rs as RS  # reference

    torch.manual_seed(0)
    torch.set_grad_enabled(False)

    # 1-3. generator forward, eval (running-stat BN), fp32
    for name, ctor, seed, shape, scale in [
        ("gen_resnet_x4", lambda: M.ResNet(1, 0.2, scaleRate=4), 0, (2, 20, 36), 4),
        ("gen_resnet_x2", lambda: M.ResNet(1, 0.2, scaleRate=2), 1, (1, 32, 32), 2),
        ("gen_eresnet_x4", lambda: M.EResNet(2, 0.2, scaleRate=4), 2, (1, 16, 24), 4),
    ]:
        model = load_synth(ctor().eval(), seed)
        lr, hr = synth_lr_batch(shape[0], shape[1], shape[2], seed=100 + seed, scale=scale)
        x = normalize(lr)
        y = model(x)
        wrapped = M.Model(model)
        wrapped.fuse()
        y_fused = wrapped(x)
        np.savez_compressed(OUT / f"{name}.npz", x=np32(x), y=np32(y), y_fused=np32(y_fused), hr=np32(hr),
                            seed=seed, scale=scale)
        print(name, tuple(y.shape), float((y - y_fused).abs().max()))

    # 4. uint8 Model wrapper (rs.py's TorchScript artifact semantics), fused
    model = load_synth(M.ResNet(1, 0.2, scaleRate=4).eval(), 3)
    wrapped = M.Model(model)
    wrapped.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    wrapped.eval().fuse()
    g = torch.Generator().manual_seed(7)
    img = (torch.rand(1, 3, 24, 40, generator=g) * 255).to(torch.uint8)
    out = wrapped(img.clone())
    np.savez_compressed(OUT / "model_u8.npz", x=img.numpy(), y=out.numpy(), seed=3)
    print("model_u8", tuple(out.shape))

    # 5. rs.py tiled still-image path (runer image branch, rs.py:78-114) with the
    #    reference's own sliding_window + paste cursor; read/write/jit stubbed.
    big = (torch.rand(3, 40, 56, generator=g) * 255).to(torch.uint8)
    _IO["image"] = big
    orig_jit_load = torch.jit.load
    torch.jit.load = lambda *a, **k: wrapped
    try:
        RS.runer(model="model.pt", src="in.png", save_dir="/tmp/_isr_golden_out.png", window_size=16,
                 batch_size=1, worker=0)
    finally:
        torch.jit.load = orig_jit_load
    np.savez_compressed(OUT / "tiled_u8.npz", x=big.numpy(), y=_IO["png"].numpy(), window=16, seed=3)
    print("tiled_u8", tuple(_IO["png"].shape))

    # 6. per-block outputs (for kernel-level localisation)
    blocks = {}
    xb = torch.randn(1, 64, 12, 20, generator=g)
    blocks["x"] = np32(xb)
    conv = load_synth(M.Conv(64, 32, 3, 1, None, act=nn.LeakyReLU()).eval(), 10)
    blocks["conv"] = np32(conv(xb))
    rdb = load_synth(M.RDB(64, 32, 3, nn.LeakyReLU(), add_rate=0.2).eval(), 11)
    blocks["rdb"] = np32(rdb(xb))
    rrdb = load_synth(M.RRDB(64, 3, nn.LeakyReLU(), add_rate=0.2).eval(), 12)
    blocks["rrdb"] = np32(rrdb(xb))
    sc = load_synth(M.Scaler(64, 64, 2, 3, nn.LeakyReLU()).eval(), 13)
    blocks["scaler"] = np32(sc(xb))
    np.savez_compressed(OUT / "blocks.npz", **blocks)
    print("blocks", {k: v.shape for k, v in blocks.items()})

    # 7. one pre-training step's loss and gradients (train.py:52-63 semantics,
    #    fp32 CPU: train-mode BN batch statistics, MSE)
    torch.set_grad_enabled(True)
    model = load_synth(M.ResNet(1, 0.2, scaleRate=2), 4).train()
    lr, hr = synth_lr_batch(2, 16, 16, seed=300, scale=2)
    x = normalize(lr)
    target = hr * 2 - 1  # PIL_to_tanh (utils/datasets.py:96-106)
    pred = model(x)
    loss = nn.MSELoss()(pred, target)
    loss.backward()
    grads = {k: np32(p.grad) for k, p in model.named_parameters() if any(
        s in k for s in ["conv0.conv.weight", "residual.0.net.0.conv0.conv.weight", "residual.0.net.2.conv.bn.weight",
                         "conv1.bn.bias", "scaler.0.net.0.conv.weight", "conv2.conv.weight", "conv2.conv.bias"])}
    stats = {k: np32(v) for k, v in model.state_dict().items() if "running" in k and k.startswith("residual.0.net.0.conv0")}
    np.savez_compressed(OUT / "train_step_x2.npz", x=np32(x), target=np32(target), pred=np32(pred),
                        loss=np32(loss), seed=4, **{"grad:" + k: v for k, v in grads.items()},
                        **{"stat:" + k: v for k, v in stats.items()})
    print("train_step_x2", float(loss.detach()))

    # 8. perceptual + adversarial losses (utils/loss.py) on the locally built VGG19.
    #    Reference quirk: L1Loss(lossweight=1) (utils/loss.py:33-35) wraps an
    #    int64 tensor in nn.Parameter, which torch >= 2.x rejects, so
    #    gen_loss(beforeAct=True) and `train.py --resnet --enchant` crash as
    #    written.  Only for this fixture the default is made the float 1.0 it
    #    was evidently meant to be.
    L.L1Loss.__init__.__defaults__ = (1.0,)
    for before_act in (False, True):
        gl = L.gen_loss(device="cpu", beforeAct=before_act)
        gl.vgg_net.load_state_dict(synth_state_dict(gl.vgg_net.state_dict(), 20))
        sr = torch.randn(2, 3, 32, 32, generator=g, requires_grad=True)
        hr = torch.randn(2, 3, 32, 32, generator=g)
        sr_disc = torch.randn(2, 1, generator=g)
        hr_disc = torch.randn(2, 1, generator=g)
        feats = gl.vgg_net(sr)
        perc, adv, content = gl.calc_contentLoss(sr, hr, sr_disc)
        content.backward()
        d_loss = gl.calc_advLoss(sr_disc, hr_disc)
        np.savez_compressed(OUT / f"loss_vgg_{'pre' if before_act else 'post'}act.npz", sr=np32(sr), hr=np32(hr),
                            sr_disc=np32(sr_disc), hr_disc=np32(hr_disc), feats=np32(feats), perceptual=np32(perc),
                            adversarial=np32(adv), content=np32(content), d_loss=np32(d_loss),
                            grad_sr=np32(sr.grad), seed=20)
        print("loss_vgg", before_act, float(perc.detach()), float(content.detach()), tuple(feats.shape))

    # 9. EMA decay ramp
    ema = M.ModelEMA(nn.Linear(2, 2), tau=2000)
    ups = np.array([1, 10, 100, 1000, 5000])
    np.savez_compressed(OUT / "ema.npz", updates=ups, decay=np.array([ema.decay(int(u)) for u in ups]), tau=2000)
    golden_denoise(M)
    golden_disc(M)
    print("done")


def golden_denoise(M):
    """10. Denoise (utils/models.py:672-706), eval, fp32: the network
    `train.py --train_denoise` trains (train.py:204-205).  residual_blocks=4 →
    2 + 2 + 2 ResidualBlock1; input 40x72 (even, not a tile multiple)."""
    torch.manual_seed(0)
    with torch.no_grad():
        model = load_synth(M.Denoise(4).eval(), 30)
        g = torch.Generator().manual_seed(31)
        x = torch.rand(2, 3, 40, 72, generator=g) * 2 - 1
        y = model(x.clone())
    np.savez_compressed(OUT / "denoise.npz", x=np32(x), y=np32(y), seed=30, residual_blocks=4)
    print("denoise", tuple(y.shape))


def golden_disc(M):
    """11. Discriminator(3, 64, 8, 1024) (utils/models.py:513-569) in train mode, fp32,
    as SRGAN training runs it (train.py:307, :113-126): logits for a [4,3,64,64]
    input, then backward of sum(logits * w) — input gradient, every parameter
    gradient (tensors above 16384 elements: 16384 flattened elements drawn uniformly
    over the WHOLE tensor, sorted, their indices stored as `gidx:{name}` — a sample of
    every output channel and tap, not just the first rows), and the BatchNorm running
    statistics after that forward."""
    torch.manual_seed(0)
    model = load_synth(M.Discriminator(3, 64, 8, 1024), 40).train()
    g = torch.Generator().manual_seed(41)
    x = (torch.randn(4, 3, 64, 64, generator=g)).requires_grad_(True)
    w = torch.randn(4, 1, generator=g)
    with torch.enable_grad():
        y = model(x)
        (y * w).sum().backward()
    out = dict(x=np32(x), w=np32(w), y=np32(y), dx=np32(x.grad), seed=40)
    gs = torch.Generator().manual_seed(42)
    for k, p in model.named_parameters():
        flat = p.grad.flatten()
        if flat.numel() > 16384:
            idx = torch.randperm(flat.numel(), generator=gs)[:16384].sort().values
            out[f"gidx:{k}"] = idx.to(torch.int32).numpy()
            flat = flat[idx]
        out[f"grad:{k}"] = np32(flat)
    for k, b in model.named_buffers():
        if "running" in k:
            out[f"stat:{k}"] = np32(b)
    np.savez_compressed(OUT / "disc.npz", **out)
    print("disc", tuple(y.shape), len(out))


if __name__ == "__main__":
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    only = {"--only-denoise": golden_denoise, "--only-disc": golden_disc}.get(sys.argv[1] if sys.argv[1:] else "")
    if only is not None:  # regenerate just this fixture
        if not REF.exists():
            raise SystemExit("reference not present")
        install_stubs()
        import utils.models as _M  # reference
        only(_M)
    else:
        main()
