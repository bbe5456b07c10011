"""Model-level parity: the HIP path vs the reference's CPU fp32 outputs.

Golden outputs come from the reference itself (tests/golden/make_golden.py);
the oracle (oracle/ref_cpu.py) is pinned to them by test_oracle_golden.py and
is used here for larger/other shapes.  Tolerance (north star): the bf16 HIP
path must stay within 0.01 dB of the fp32 reference's PSNR against the HR
target, and PSNR(HIP vs fp32 reference) >= 40 dB on the [-1, 1] output
(peak 2).  uint8 outputs: |diff| <= 1 LSB on >= 99% of pixels, never > 2.
"""
import numpy as np
import pytest
import torch

from conftest import t
from image_super_resolution_amd import models
from image_super_resolution_amd.weights import synth_state_dict, synth_lr_batch, normalize
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _model(ctor, seed):
    m = ctor()
    m.load_state_dict(synth_state_dict(m.state_dict(), seed))
    return m.eval()


def _check(y_hip, y_ref, hr01):
    p = R.psnr(y_hip, y_ref)
    hr = hr01 * 2 - 1
    dp = abs(R.psnr(y_hip, hr) - R.psnr(y_ref, hr))
    assert p >= 40.0, f"PSNR(HIP vs ref) = {p:.2f} dB"
    assert dp <= 0.01, f"|dPSNR vs HR| = {dp:.4f} dB"
    return p, dp


@pytest.mark.parametrize("name,ctor", [
    ("gen_resnet_x4", lambda: models.ResNet(1, 0.2, scaleRate=4)),
    ("gen_resnet_x2", lambda: models.ResNet(1, 0.2, scaleRate=2)),
    ("gen_eresnet_x4", lambda: models.EResNet(2, 0.2, scaleRate=4)),
])
@torch.no_grad()
def test_generator_vs_reference_golden(golden, name, ctor):
    g = golden(name)
    m = _model(ctor, int(g["seed"])).to(DEV)
    y = m(t(g["x"]).to(DEV)).cpu()
    assert y.shape == g["y"].shape
    _check(y, t(g["y"]), t(g["hr"]))


@torch.no_grad()
def test_fused_model_equivalence(golden):
    g = golden("gen_resnet_x4")
    m = _model(lambda: models.ResNet(1, 0.2, scaleRate=4), int(g["seed"]))
    wrapped = models.Model(m).fuse().to(DEV)
    y = wrapped(t(g["x"]).to(DEV)).cpu()
    _check(y, t(g["y_fused"]), t(g["hr"]))


@torch.no_grad()
def test_model_u8_vs_reference_golden(golden):
    g = golden("model_u8")
    m = _model(lambda: models.ResNet(1, 0.2, scaleRate=4), int(g["seed"]))
    wrapped = models.Model(m)
    wrapped.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    wrapped = wrapped.eval().fuse().to(DEV)
    y = wrapped(t(g["x"]).to(DEV)).cpu()
    assert y.dtype == torch.uint8 and y.shape == g["y"].shape
    d = (y.int() - t(g["y"]).int()).abs()
    assert d.max().item() <= 2 and (d > 1).float().mean().item() < 0.01


@torch.no_grad()
def test_model_float_input_skips_the_255_division(golden):
    """The reference's Normalize divides by 255 only for uint8 input (utils/datasets.py:65-71):
    a float image already in [0, 1] is normalised as is, so it must give the uint8 image's
    output (same normalised values up to fp32 rounding), and a float image in [0, 255] a
    different one."""
    g = golden("model_u8")
    m = _model(lambda: models.ResNet(1, 0.2, scaleRate=4), int(g["seed"]))
    wrapped = models.Model(m)
    wrapped.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    wrapped = wrapped.eval().fuse().to(DEV)
    xu8 = t(g["x"]).to(DEV)
    y_u8 = wrapped(xu8)
    y_f = wrapped(xu8.float() / 255.0)
    assert y_f.dtype == torch.uint8 and y_f.shape == y_u8.shape
    d = (y_f.int() - y_u8.int()).abs()
    assert d.max().item() <= 1 and (d > 0).float().mean().item() < 0.01
    # a [0, 255] float image is NOT divided by 255 (the reference's quirk): a different output
    y_255 = wrapped(xu8.float())
    assert (y_255.int() - y_u8.int()).abs().float().mean().item() > 5.0


@torch.no_grad()
def test_blocks_vs_reference_golden(golden):
    g = golden("blocks")
    x = t(g["x"]).to(DEV)
    cases = [
        ("conv", lambda: models.Conv(64, 32, 3, 1, None, act=torch.nn.LeakyReLU()), 10),
        ("rdb", lambda: models.RDB(64, 32, 3, torch.nn.LeakyReLU(), add_rate=0.2), 11),
        ("rrdb", lambda: models.RRDB(64, 3, torch.nn.LeakyReLU(), add_rate=0.2), 12),
        ("scaler", lambda: models.Scaler(64, 64, 2, 3, torch.nn.LeakyReLU()), 13),
    ]
    for key, ctor, seed in cases:
        y = _model(ctor, seed).to(DEV)(x).cpu()
        ref = t(g[key])
        rel = ((y - ref).norm() / ref.norm()).item()
        assert rel < 1e-2, f"{key}: relative L2 error {rel:.3e}"


@torch.no_grad()
def test_full_depth_generator_vs_oracle():
    """16 RRDBs (the bench model) on a ragged 2x3x36x52 input vs the fp32 oracle."""
    m = _model(lambda: models.ResNet(16, 0.2, scaleRate=4), 5)
    lr, hr = synth_lr_batch(2, 36, 52, seed=77, scale=4)
    x = normalize(lr)
    y = m.to(DEV)(x.to(DEV)).cpu()
    sd = {k: v.float() for k, v in synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), 5).items()}
    ref = R.generator(sd, x, num_blocks=16, scale=4)
    p, dp = _check(y, ref, hr)
    print(f"full-depth PSNR(HIP vs fp32 oracle) = {p:.2f} dB, dPSNR = {dp:.5f} dB")


def _u8_model(seed):
    m = _model(lambda: models.ResNet(1, 0.2, scaleRate=4), seed)
    wrapped = models.Model(m)
    wrapped.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    return wrapped.eval().fuse().to(DEV)


@pytest.mark.parametrize("batch", [1, 4])
@torch.no_grad()
def test_tiled_u8_vs_reference_golden(golden, batch):
    """rs.py image branch (window 16, ragged edges, reference stitch) through the
    HIP tiler: same uint8 tolerance as the single-window path."""
    from image_super_resolution_amd import tiler
    g = golden("tiled_u8")
    runner = tiler.runner_for(_u8_model(int(g["seed"])), DEV)
    up = tiler.TileUpscaler(runner, runner.scale, window=int(g["window"]), halo=0, batch=batch, device=DEV)
    y = up(t(g["x"])).cpu()
    assert y.dtype == torch.uint8 and y.shape == g["y"].shape
    d = (y.int() - t(g["y"]).int()).abs()
    assert d.max().item() <= 2 and (d > 1).float().mean().item() < 0.01


@torch.no_grad()
def test_tiled_halo_reduces_seams():
    """cfg4 halo mode: tiles with context agree with the whole-image run far
    better than the reference's halo-less stitch."""
    from image_super_resolution_amd import tiler
    model = _u8_model(3)
    img = (torch.rand(3, 72, 88, generator=torch.Generator().manual_seed(9)) * 255).to(torch.uint8)
    full = model(img[None].to(DEV))[0].float()
    runner = tiler.runner_for(model, DEV)
    err = {}
    for halo in (0, 8):
        y = tiler.TileUpscaler(runner, 4, window=32, halo=halo, batch=4, device=DEV)(img).float()
        err[halo] = (y - full).abs().mean().item()
    assert err[8] < 0.5 * err[0], err
