"""TruncatedVGG19 + gen_loss on the HIP path vs the reference's own outputs
(tests/golden/loss_vgg_*.npz, produced by utils/loss.py with a seeded local
VGG19 — ImageNet weights are unavailable offline, so parity with those is
unpinned) and vs the fp32 oracle at a multi-tile size.

bf16 activations through 16 convs: features and content loss are compared by
relative L2 error (<= 3%).  The input gradient passes through 16 ReLU masks and
4 maxpool argmaxes decided on bf16 activations; elements whose sign / window
maximum flips between bf16 and fp32 reroute their gradient, so against fp32
autograd only cos >= 0.95 holds (tools/diag_vgg.py: rel 2e-3 without
ReLU/pool, growing with each switch).  The backward kernels themselves are
pinned against autograd of a bf16-emulating torch graph (every activation
rounded to bf16 as the HIP path stores it): rel <= 3%, cos >= 0.999.
"""
import warnings

import pytest
import torch
import torch.nn.functional as F

from conftest import t
from image_super_resolution_amd import loss as L
from image_super_resolution_amd.weights import synth_state_dict
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _gl(before_act, seed):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gl = L.gen_loss(device=DEV, beforeAct=before_act)
    gl.vgg_net.load_state_dict(synth_state_dict(gl.vgg_net.state_dict(), seed))
    return gl


@pytest.mark.parametrize("which", ["postact", "preact"])
def test_gen_loss_vs_reference_golden(golden, which):
    g = golden(f"loss_vgg_{which}")
    gl = _gl(which == "preact", int(g["seed"]))
    sr = t(g["sr"]).to(DEV).requires_grad_(True)
    feats = gl.vgg_net(sr)
    assert _rel(feats.detach().cpu(), t(g["feats"])) < 3e-2
    perc, adv, content = gl.calc_contentLoss(sr, t(g["hr"]).to(DEV), t(g["sr_disc"]).to(DEV))
    content.backward()
    assert abs(content.item() - float(g["content"])) <= 3e-2 * abs(float(g["content"]))
    assert abs(adv.item() - float(g["adversarial"])) <= 1e-5
    gs = sr.grad.cpu()
    ref = t(g["grad_sr"])
    assert F.cosine_similarity(gs.flatten(), ref.flatten(), dim=0).item() >= 0.95
    d = gl.calc_advLoss(t(g["sr_disc"]).to(DEV), t(g["hr_disc"]).to(DEV))
    assert abs(d.item() - float(g["d_loss"])) <= 1e-5


def _bf16_emulated_vgg(vgg, x):
    """torch graph of the truncated VGG with every stored tensor rounded to bf16
    (straight-through in the backward), i.e. the HIP path's storage precision."""
    def rnd(t):
        return t + (t.to(torch.bfloat16).float() - t).detach()
    y = rnd(x)
    for m in vgg.truncated_vgg19:
        if isinstance(m, torch.nn.Conv2d):
            y = F.conv2d(y, m.weight.to(torch.bfloat16).float(), m.bias, padding=1)
            y = rnd(y)
        elif isinstance(m, torch.nn.ReLU):
            y = F.relu(y)
        else:
            y = F.max_pool2d(y, 2, 2)
    return y


@pytest.mark.parametrize("hw", [(32, 32), (64, 96)])
@pytest.mark.parametrize("before_act", [False, True])
def test_vgg_backward_vs_bf16_emulation(hw, before_act):
    gl = _gl(before_act, 21)
    gen = torch.Generator().manual_seed(3)
    sr = torch.randn(2, 3, *hw, generator=gen).to(DEV)
    xr = sr.clone().requires_grad_(True)
    fr = _bf16_emulated_vgg(gl.vgg_net, xr)
    gf = torch.randn(fr.shape, generator=gen).to(DEV)
    fr.backward(gf)
    x = sr.clone().requires_grad_(True)
    f = gl.vgg_net(x)
    f.backward(gf)
    assert _rel(f.detach(), fr.detach()) < 2e-2
    assert _rel(x.grad, xr.grad) < 3e-2
    assert F.cosine_similarity(x.grad.flatten(), xr.grad.flatten(), dim=0).item() >= 0.999


def test_vgg_multitile_vs_oracle():
    gl = _gl(False, 21)
    gen = torch.Generator().manual_seed(3)
    sr = torch.randn(2, 3, 64, 96, generator=gen)
    hr = torch.randn(2, 3, 64, 96, generator=gen)
    sd = {k: v.float() for k, v in gl.vgg_net.state_dict().items()}
    srr = sr.clone().requires_grad_(True)
    fr = R.vgg_truncated(sd, srr)
    F.mse_loss(fr, R.vgg_truncated(sd, hr)).backward()
    x = sr.to(DEV).requires_grad_(True)
    f = gl.vgg_net(x)
    F.mse_loss(f, gl.vgg_net(hr.to(DEV)).detach()).backward()
    assert _rel(f.detach().cpu(), fr.detach()) < 3e-2
    gx, gr = x.grad.cpu(), srr.grad
    assert F.cosine_similarity(gx.flatten(), gr.flatten(), dim=0).item() >= 0.95
