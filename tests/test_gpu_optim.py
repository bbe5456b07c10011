"""Multi-tensor optimiser kernels (optim.py / isr_mt_*) vs torch's own
Adam, clip_grad_norm_ and the EMA lerp on the same tensors."""
import copy

import pytest
import torch

from image_super_resolution_amd import models, optim

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [(64, 3, 9, 9), (64,), (32, 64, 3, 3), (7,), (1, 1), (70001,), (256, 64, 3, 3)]
    ps = [torch.randn(s, generator=g).to(DEV).requires_grad_() for s in shapes]
    # one channels_last parameter (the discriminator runs NHWC)
    ps.append(torch.randn(8, 16, 3, 3, generator=g).to(DEV).to(memory_format=torch.channels_last).requires_grad_())
    return ps


def _grads(ps, seed):
    g = torch.Generator().manual_seed(seed)
    for p in ps:
        p.grad = torch.randn(p.shape, generator=g).to(DEV).to(memory_format=torch.channels_last
                                                                if not p.is_contiguous() else torch.contiguous_format)


@pytest.mark.parametrize("wd", [0.0, 1e-2])
def test_fused_adam_matches_torch(wd):
    a = _params(0)
    b = [p.detach().clone().requires_grad_() for p in a]
    oa = optim.FusedAdam(a, lr=1e-3, betas=(0.9, 0.999), weight_decay=wd)
    ob = torch.optim.Adam(b, lr=1e-3, betas=(0.9, 0.999), weight_decay=wd, foreach=False)
    sa = torch.optim.lr_scheduler.LinearLR(oa, 1, 0.01, total_iters=5)
    sb = torch.optim.lr_scheduler.LinearLR(ob, 1, 0.01, total_iters=5)
    for step in range(5):
        _grads(a, step)
        _grads(b, step)
        oa.step(), ob.step(), sa.step(), sb.step()
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, rtol=2e-6, atol=2e-7)
    # state dict round-trips into torch's Adam (checkpoint compatibility)
    st = oa.state_dict()
    oc = torch.optim.Adam(b, lr=1e-3)
    oc.load_state_dict(st)
    assert float(oc.state_dict()["state"][0]["step"]) == 5.0


def test_clip_grad_norm_matches_torch():
    a = _params(1)
    b = [p.detach().clone().requires_grad_() for p in a]
    _grads(a, 7)
    _grads(b, 7)
    for p in a + b:
        p.grad.mul_(3.0)  # total norm well above max_norm → clipping active
    na = optim.clip_grad_norm_(a, 10)
    nb = torch.nn.utils.clip_grad_norm_(b, 10)
    torch.testing.assert_close(na, nb, rtol=1e-5, atol=0)
    for x, y in zip(a, b):
        torch.testing.assert_close(x.grad, y.grad, rtol=1e-5, atol=1e-7)
    # below the threshold: coefficient clamps to 1 (grads unchanged)
    for p in a:
        p.grad.mul_(1e-4)
    before = [p.grad.clone() for p in a]
    optim.clip_grad_norm_(a, 10)
    for x, y in zip(a, before):
        torch.testing.assert_close(x.grad, y, rtol=1e-6, atol=0)


def test_ema_update_matches_reference_formula():
    m = models.ResNet(1, 0.2, scaleRate=2).to(DEV)
    ema = models.ModelEMA(m, tau=10)
    ref = copy.deepcopy(ema.ema.state_dict())
    with torch.no_grad():
        for p in m.parameters():
            p.add_(torch.randn_like(p))
    ema.update(m)
    d = 0.9999 * (1 - __import__("math").exp(-1 / 10))
    msd = m.state_dict()
    for k, v in ema.ema.state_dict().items():
        if v.dtype.is_floating_point:
            torch.testing.assert_close(v, ref[k] * d + (1 - d) * msd[k], rtol=1e-6, atol=1e-7)


def test_eval_repacks_after_hip_optimiser_and_ema_writes():
    """FusedAdam / ema_update_ write parameters through raw pointers (no
    torch `_version` bump); the packed-weight cache must still see the new weights."""
    from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict
    torch.manual_seed(0)
    m = models.EResNet(1, 0.2, scaleRate=2)
    m.load_state_dict(synth_state_dict(m.state_dict(), seed=3))
    m = m.to(DEV).eval()
    lr, _ = synth_lr_batch(1, 16, 16, seed=8, scale=2)
    x = normalize(lr).to(DEV)
    with torch.no_grad():
        y0 = m(x)
    assert y0.abs().max().item() < 0.999  # not saturated: a weight change must show
    params = [p for p in m.parameters()]
    opt = optim.FusedAdam(params, lr=1e-3)
    g = torch.Generator(device=DEV).manual_seed(1)
    for p in params:
        p.grad = torch.randn(p.shape, device=DEV, generator=g)
    opt.step()
    with torch.no_grad():
        y1 = m(x)
        fresh = copy.deepcopy(m)  # no cached pack: packs the stepped weights
        fresh.__dict__.pop("_isr_pack", None)
        yf = fresh(x)
    assert not torch.equal(y0, y1), "eval after an optimiser step reused the stale pack"
    torch.testing.assert_close(y1, yf, rtol=0, atol=0)
    ema = copy.deepcopy(m)
    ema.__dict__.pop("_isr_pack", None)
    with torch.no_grad():
        ye0 = ema(x)
        src = [p.detach().mul(0.9) for p in ema.parameters()]
        optim.ema_update_([p.data for p in ema.parameters()], src, 0.5)
        ye1 = ema(x)
        fresh = copy.deepcopy(ema)
        fresh.__dict__.pop("_isr_pack", None)
        torch.testing.assert_close(ye1, fresh(x), rtol=0, atol=0)
    assert not torch.equal(ye0, ye1)
