"""Denoise (utils/models.py:672-706) on libisr vs the reference / oracle.

Golden output from the reference itself (tests/golden/make_golden.py
golden_denoise, pinned to the oracle by test_oracle_golden.py); other shapes
against the oracle (oracle/ref_cpu.denoise).  Tolerance as for the generators
(tests/test_gpu_parity.py): PSNR(HIP vs fp32 reference) >= 40 dB on the [-1, 1]
output, and |dPSNR| <= 0.01 dB against a target (here the noisy input itself,
the identity a denoiser starts from).
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import t
from image_super_resolution_amd import models, ops
from image_super_resolution_amd.ops import ActBuffer
from image_super_resolution_amd.weights import synth_state_dict
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


def _check(y_hip, y_ref, target):
    p = R.psnr(y_hip, y_ref)
    dp = abs(R.psnr(y_hip, target) - R.psnr(y_ref, target))
    assert p >= 40.0, f"PSNR(HIP vs ref) = {p:.2f} dB"
    assert dp <= 0.01, f"|dPSNR vs target| = {dp:.4f} dB"
    return p, dp


@torch.no_grad()
def test_denoise_vs_reference_golden(golden):
    g = golden("denoise")
    m = _model(lambda: models.Denoise(int(g["residual_blocks"])), int(g["seed"])).to(DEV)
    x = t(g["x"])
    y = m(x.to(DEV)).cpu()
    assert y.shape == g["y"].shape
    _check(y, t(g["y"]), x)


@pytest.mark.parametrize("n,h,w,blocks", [(1, 66, 98, 2), (2, 128, 96, 8), (1, 64, 64, 0)])
@torch.no_grad()
def test_denoise_vs_oracle(n, h, w, blocks):
    """Ragged sizes (66x98: odd half-resolution grid 33x49), the default depth's
    structure, and residual_blocks=0 (the stride-2 conv reads conv0's output)."""
    m = _model(lambda: models.Denoise(blocks), 40 + blocks)
    gen = torch.Generator().manual_seed(h * w)
    x = torch.rand(n, 3, h, w, generator=gen) * 2 - 1
    y = m.to(DEV)(x.to(DEV)).cpu()
    ref = R.denoise({k: v.cpu() for k, v in m.state_dict().items()}, x)
    _check(y, ref, x)
    # repeated call on the cached plan is deterministic
    y2 = m(x.to(DEV)).cpu()
    assert torch.equal(y, y2)


@torch.no_grad()
def test_denoise_fused_and_odd_size():
    m = _model(lambda: models.Denoise(2), 50).to(DEV)
    x = torch.rand(1, 3, 32, 48) * 2 - 1
    y = m(x.to(DEV)).cpu()
    wrapped = models.Model(m).fuse()
    yf = wrapped(x.to(DEV)).cpu()
    assert R.psnr(y, yf) >= 40.0
    with pytest.raises(ValueError):
        m(torch.zeros(1, 3, 33, 48, device=DEV))


@torch.no_grad()
def test_pixel_shuffle2_kernel_exact():
    """isr_pixel_shuffle2 == LeakyReLU(0.2)(PixelShuffle(2)(a)) bit-exactly on bf16 data, zeros outside."""
    gen = torch.Generator().manual_seed(3)
    a = torch.randn(2, 256, 20, 27, generator=gen).to(torch.bfloat16).float()
    ab = ActBuffer.from_nchw(a.to(DEV), pad=1)
    yb = ActBuffer.alloc(2, 40, 54, 64, 2, DEV)
    yb.t.fill_(7.0)  # the kernel must overwrite the whole computed region, incl. alignment slack
    p = yb.pad
    yb.t[:, :, :p] = 0
    yb.t[:, :, -p:] = 0
    yb.t[:, :, :, :p] = 0
    yb.t[:, :, :, -p:] = 0
    ops.pixel_shuffle2(yb, ab, 64, slope=0.2)
    ref = F.leaky_relu(F.pixel_shuffle(a, 2), 0.2).to(torch.bfloat16).float()
    assert torch.equal(yb.to_nchw().cpu(), ref)
    assert int((yb.outside_valid() != 0).sum()) == 0


@torch.no_grad()
def test_residual_block1_module():
    blk = _model(lambda: models.ResidualBlock1(64, 64, 64, 3, torch.nn.LeakyReLU(0.2)), 60)
    x = torch.randn(2, 64, 24, 40)
    y = blk.to(DEV)(x.to(DEV)).cpu()
    sd = {f"b.{k}": v.cpu() for k, v in blk.state_dict().items()}
    ref = R.residual_block1(sd, "b", x)
    assert R.psnr(y, ref) >= 40.0


@pytest.mark.parametrize("blocks,n,h,w", [(2, 2, 32, 48), (4, 2, 66, 40), (0, 3, 32, 32)])
def test_denoise_train_step_grads_vs_oracle(blocks, n, h, w):
    """`train.py --train_denoise` step (train.py:52-63: MSE, train-mode BN): every
    parameter gradient of the libisr backward vs fp32 autograd through the oracle.
    Denoise has unscaled residuals and BN on every block, so bf16 activations cost
    5-10 % relative L2 on the deepest gradients; the bar (as tests/test_gpu_disc.py)
    is the error torch's own bf16 autocast makes on the same graph and tensors
    (the reference trains under autocast, train.py:54): hip <= 1.3 x autocast + 0.02,
    cosine >= 0.99.  BN running statistics to 1e-2."""
    m = models.Denoise(blocks)
    m.load_state_dict(synth_state_dict(m.state_dict(), 70 + blocks))
    gen = torch.Generator().manual_seed(5 + h)
    x = torch.rand(n, 3, h, w, generator=gen) * 2 - 1
    target = (x + 0.1 * torch.randn(n, 3, h, w, generator=gen)).clamp(-1, 1)

    def oracle_grads(device, autocast):
        sd = {k: v.detach().clone().float().to(device) for k, v in m.state_dict().items()}
        params = {k: v.requires_grad_(True) for k, v in sd.items()
                  if "running" not in k and "num_batches_tracked" not in k}
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            y = R.denoise(sd, x.to(device), train_bn=True)
        F.mse_loss(y.float(), target.to(device)).backward()
        return sd, y.detach().float().cpu(), {k: p.grad.to(DEV) for k, p in params.items()}

    sd, y_ref, g_ref = oracle_grads("cpu", False)
    _, _, g_amp = oracle_grads(DEV, True)
    m = m.to(DEV).train()
    y = m(x.to(DEV))
    assert R.psnr(y.detach().cpu(), y_ref) >= 40.0
    F.mse_loss(y, target.to(DEV)).backward()
    for name, p in m.named_parameters():
        assert p.grad is not None, name
        r = g_ref[name]
        rel = ((p.grad - r).norm() / r.norm().clamp_min(1e-12)).item()
        rel_amp = ((g_amp[name] - r).norm() / r.norm().clamp_min(1e-12)).item()
        cos = F.cosine_similarity(p.grad.flatten(), r.flatten(), dim=0).item()
        assert rel <= 1.3 * rel_amp + 0.02 and cos >= 0.99, f"{name}: rel {rel:.3e} (autocast {rel_amp:.3e}) cos {cos:.5f}"
    for name, b in m.named_buffers():
        if "running" in name:
            torch.testing.assert_close(b.cpu(), sd[name], rtol=1e-2, atol=1e-3)
        if "num_batches_tracked" in name:
            assert int(b.item()) == 1, name


def test_pixel_unshuffle2_kernel_exact():
    """isr_pixel_unshuffle2 == PixelUnshuffle(2)(a * LeakyReLU'(m)) bit-exactly (the shuffle's input gradient)."""
    gen = torch.Generator().manual_seed(4)
    a = torch.randn(2, 64, 40, 54, generator=gen).to(torch.bfloat16).float()
    mm = torch.randn(2, 64, 40, 54, generator=gen).to(torch.bfloat16).float()
    ab = ActBuffer.from_nchw(a.to(DEV), pad=1)
    mb = ActBuffer.from_nchw(mm.to(DEV), pad=1)
    yb = ActBuffer.alloc(2, 20, 27, 256, 1, DEV)
    ops.pixel_unshuffle2(yb, ab, 256, m=mb, mslope=0.2)
    ref = F.pixel_unshuffle(torch.where(mm > 0, a, a * 0.2), 2).to(torch.bfloat16).float()
    assert torch.equal(yb.to_nchw().cpu(), ref)
    assert int((yb.outside_valid() != 0).sum()) == 0


def test_deepcopy_after_forward():
    """ModelEMA deep-copies the model; libisr caches (ctypes descriptors) must not travel."""
    from copy import deepcopy
    m = _model(lambda: models.Denoise(2), 80).to(DEV)
    x = torch.rand(1, 3, 32, 32, device=DEV) * 2 - 1
    with torch.no_grad():
        y = m(x)
        c = deepcopy(m)
        assert "_isr_pack" in m.__dict__ and "_isr_pack" not in c.__dict__
        assert torch.equal(c(x), y)
    g = _model(lambda: models.ResNet(1, 0.2, scaleRate=2), 81).to(DEV)
    with torch.no_grad():
        yg = g(x)
        assert torch.equal(deepcopy(g)(x), yg)
