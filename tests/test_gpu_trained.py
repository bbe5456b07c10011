"""North-star parity with weights that super-resolve.

The committed ResNet(16, 0.2, x4) in tests/golden/trained_resnet_x4.safetensors was trained by this
repo's own `train.py --resnet` (tools/train_weights.py: pixel MSE, Adam, LinearLR, EMA; reference
train.py:41-67) on synthetic dead-leaves crops (data.leaves_hr_u8).  On held-out tiles of that
distribution the fp32 oracle reaches ~30 dB against HR and beats bicubic upsampling.  In that
regime the bar bites: |PSNR(HIP, HR) - PSNR(ref, HR)| <= 0.01 dB needs PSNR(HIP vs ref) of
roughly 56 dB or more (the synthetic-weights tests sit at a saturated 5 dB output, where any path
that agrees to ~32 dB passes).  Tolerance (north star, written here): 0.01 dB on the [-1, 1]
output (peak 2) and on BT.601 luma with the 4-px border crop (utils/datasets.py:159-166), in
aggregate and for every tile; uint8 path: |diff| <= 2 LSB, > 1 LSB on < 0.1 % of pixels.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from image_super_resolution_amd import checkpoint, models
from image_super_resolution_amd.weights import heldout_tiles
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
WEIGHTS = __import__("pathlib").Path(__file__).parent / "golden" / "trained_resnet_x4.safetensors"
TOL_DB = 0.01
TILES = 4


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


@pytest.fixture(scope="module")
def case():
    sd = checkpoint.load_module_state(WEIGHTS)
    lr, hr = heldout_tiles(TILES, 128, 4, device=DEV)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        ref = R.generator(sd, lr, num_blocks=16, scale=4)
    return sd, lr, hr, ref


def _bicubic(lr):
    m = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
    s = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)
    return F.interpolate(lr * s + m, scale_factor=4, mode="bicubic", align_corners=False).clamp(0, 1)


@torch.no_grad()
def test_trained_weights_super_resolve(case):
    """The weights are a real x4 model: >= 28 dB against HR and better than bicubic."""
    _, lr, hr, ref = case
    p_ref = R.psnr(ref, hr * 2 - 1)
    p_bic = R.psnr(_bicubic(lr) * 2 - 1, hr * 2 - 1)
    print(f"oracle {p_ref:.3f} dB vs bicubic {p_bic:.3f} dB")
    assert p_ref >= 28.0, p_ref
    assert p_ref > p_bic + 0.3, (p_ref, p_bic)


@torch.no_grad()
def test_trained_full_depth_dpsnr(case):
    """16 RRDBs on 128² tiles through the HIP path (the persistent trunk kernel) vs the oracle."""
    sd, lr, hr, ref = case
    net = models.ResNet(16, 0.2, scaleRate=4)
    net.load_state_dict(sd)
    net = net.eval().to(DEV)
    y = net(lr.to(DEV)).float().cpu()
    hr1 = hr * 2 - 1
    agree = R.psnr(y, ref)
    d = abs(R.psnr(y, hr1) - R.psnr(ref, hr1))
    per_tile = [abs(R.psnr(y[i:i + 1], hr1[i:i + 1]) - R.psnr(ref[i:i + 1], hr1[i:i + 1])) for i in range(len(y))]
    to01 = lambda t: (t.clamp(-1, 1) + 1) / 2  # noqa: E731
    dy = abs(R.psnr_y(to01(y), hr) - R.psnr_y(to01(ref), hr))
    print(f"PSNR(HIP vs fp32 oracle) {agree:.2f} dB; dPSNR {d:.5f} dB (worst tile {max(per_tile):.5f}), "
          f"luma {dy:.5f} dB")
    assert d <= TOL_DB and max(per_tile) <= TOL_DB and dy <= TOL_DB
    # the margin the tolerance implies at this model quality (MSE_ref ~ 4e-3): >= ~56 dB agreement
    assert agree >= 10 * math.log10(4 / (4 / 10 ** (R.psnr(ref, hr1) / 10) * (10 ** (TOL_DB / 10) - 1)))


@torch.no_grad()
def test_trained_u8_model(case):
    """The uint8 `Model` wrapper (utils/models.py:723-751: Normalize, fused BN, TanhToArrayImage)."""
    sd, lr, hr, _ = case
    img = (hr[:2] * 255).round().to(torch.uint8)
    img = F.interpolate(img.float(), size=(128, 128), mode="bilinear", align_corners=False)
    img = (img + 0.5).floor().clamp(0, 255).to(torch.uint8)
    net = models.ResNet(16, 0.2, scaleRate=4)
    net.load_state_dict(sd)
    wrapped = models.Model(net)
    wrapped.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    wrapped = wrapped.eval().fuse().to(DEV)
    y = wrapped(img.to(DEV)).cpu()
    ref = R.model_u8(R.fuse_state_dict(sd), img, num_blocks=16, scale=4)
    diff = (y.int() - ref.int()).abs()
    f1, f2 = (diff > 0).float().mean().item(), (diff > 1).float().mean().item()
    print(f"uint8: {f1 * 100:.3f} % of pixels differ by 1 LSB or more, {f2 * 100:.4f} % by 2, max {diff.max().item()}")
    # fp16 storage (round 6): ~1.2e-4 RMS on [-1, 1] is ~0.016 LSB, so only pixels that close to a
    # rounding boundary flip, by one — the round-4 bar (<= 1 LSB) again.  (bf16, ~1e-3 RMS: ~9 % of
    # pixels at 1 LSB and a tail of a few 1e-5 at 2 LSB, profiles/r06_u8_outliers.json.)
    assert diff.max().item() <= 1 and f1 < 0.05
