"""Discriminator conv stack on libisr (discriminator.py): stride-2 conv / its input
gradient / weight gradient through the 2x2 phase decomposition vs torch on
bf16-rounded operands, then the whole train-mode D (forward, BN running stats,
parameter and input gradients) vs the stock fp32 modules."""
import copy

import pytest
import torch
import torch.nn.functional as F

from image_super_resolution_amd import discriminator as D, models, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def bf(t):
    return t.to(torch.bfloat16).float()


def _rel(a, b):
    d, n = (a - b).norm().item(), b.norm().item()
    return d / n if n > 0 else d


@pytest.mark.parametrize("cin,cout,h,w", [(64, 64, 32, 64), (128, 256, 16, 32)])
def test_stride2_conv_forward_dgrad_wgrad(cin, cout, h, w):
    g = torch.Generator().manual_seed(cin + cout)
    x = bf(torch.randn(2, cin, h, w, generator=g)).to(DEV)
    W = bf(torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (9 * cin)) ** 0.5).to(DEV)
    # forward: x_sub2 view + phase-expanded weights on taps {0,1}^2
    xb = ops.ActBuffer.alloc(2, h, w, cin, 2, DEV, min_hp=2 * ops.round_up(h // 2, 32) + 4,
                             min_wp=2 * ops.round_up(w // 2, 32) + 4)
    xb.set_nchw(x, 0)
    yb = ops.ActBuffer.alloc(2, h // 2, w // 2, cout, 1, DEV)
    ops.conv3x3(xb, 4 * cin, ops.pack_conv3x3(D.expand_fwd(W)), None, cout, yb, x_sub2=True, taps=1)
    torch.cuda.synchronize()
    ref = F.conv2d(x, W, stride=2, padding=1)
    assert _rel(yb.to_nchw(), ref) < 1e-2
    # input gradient: conv over gy with 4*cin outputs on taps {1,2}^2, PixelShuffle store
    gy = bf(torch.randn(2, cout, h // 2, w // 2, generator=g)).to(DEV)
    gyb = ops.ActBuffer.from_nchw(gy, pad=1)
    gxb = ops.ActBuffer.alloc(2, h, w, cin, 1, DEV, min_hp=2 * gyb.ha + 2, min_wp=2 * gyb.wa + 2)
    ops.conv3x3(gyb, cout, ops.pack_conv3x3(D.expand_dgrad(W)), None, 4 * cin, gxb, shuffle=2, taps=2)
    torch.cuda.synchronize()
    xr = x.clone().requires_grad_()
    Wr = W.clone().requires_grad_()
    F.conv2d(xr, Wr, stride=2, padding=1).backward(gy)
    assert _rel(gxb.to_nchw(), xr.grad) < 1e-2
    # weight gradient on the unshuffled input
    U = ops.ActBuffer.alloc(2, h // 2, w // 2, 4 * cin, 1, DEV)
    cb = cin // 16
    for a in (0, 1):
        for b in (0, 1):
            s = 2 * a + b
            U.t[:, s * cb:(s + 1) * cb, 1:1 + h // 2, 1:1 + w // 2, :] = \
                xb.t[:, :, 2 + a:2 + h:2, 2 + b:2 + w:2, :]
    dwp = torch.empty(cout, 4 * cin, 3, 3, device=DEV)
    ops.wgrad3x3(U, 4 * cin, gyb, cout, dwp, None)
    torch.cuda.synchronize()
    assert _rel(D.gather_wgrad(dwp, cin), Wr.grad) < 1e-3
    # ... and straight from the full-resolution buffer through the x_sub2 view, taps {0,1}^2 only
    dwq = torch.empty(cout, 4 * cin, 3, 3, device=DEV)
    ops.wgrad3x3(xb, 4 * cin, gyb, cout, dwq, None, x_sub2=True, taps=1)
    torch.cuda.synchronize()
    assert _rel(D.gather_wgrad(dwq, cin), Wr.grad) < 1e-3
    # input gradient with the LeakyReLU' mask fused into the PixelShuffle epilogue
    act = bf(torch.randn(2, cin, h, w, generator=g)).to(DEV)
    mb = ops.ActBuffer.alloc(2, h, w, cin, 0, DEV, min_hp=2 * gyb.ha, min_wp=2 * gyb.wa)
    mb.set_nchw(act, 0)
    gmb = ops.ActBuffer.alloc(2, h, w, cin, 1, DEV, min_hp=2 * gyb.ha + 2, min_wp=2 * gyb.wa + 2)
    ops.conv3x3(gyb, cout, ops.pack_conv3x3(D.expand_dgrad(W)), None, 4 * cin, gmb, shuffle=2, taps=2, m=mb,
                mslope=0.2)
    torch.cuda.synchronize()
    assert _rel(gmb.to_nchw(), xr.grad * torch.where(act > 0, 1.0, 0.2)) < 1e-2


def _pair(seed):
    torch.manual_seed(seed)
    hip = models.Discriminator(3, 64, 8, 1024).to(DEV).train()
    ref = copy.deepcopy(hip)
    hip.use_libisr(True)  # stock modules in ref
    return hip, ref


def _run(m, x, w, autocast=False):
    xr = x.clone().requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        o = m(xr)
    (o.float() * w).sum().backward()
    return o.float(), xr.grad, [p.grad for p in m.parameters()]


def test_discriminator_train_step_vs_fp32_modules():
    """Tolerance: a random-init D's gradients are ill-conditioned in bf16 (LeakyReLU
    sign flips compound through 7 BatchNorm backwards: 5-20 % rel L2 vs fp32), so
    the bar is the error torch's own bf16 autocast makes on the same tensors (the
    reference trains D under fp16 autocast): hip <= 1.3 x autocast + 0.02."""
    hip, ref = _pair(0)
    amp = copy.deepcopy(ref)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 3, 128, 128, generator=g).to(DEV)
    w = torch.randn(4, 1, generator=g).to(DEV)
    oh, dxh, gh = _run(hip, x, w)
    orf, dxr, gr = _run(ref, x, w)
    oa, dxa, ga = _run(amp, x, w, autocast=True)
    assert _rel(oh, orf) < 0.03
    assert _rel(dxh, dxr) <= 1.3 * _rel(dxa, dxr) + 0.02
    for (name, _), a, b, c in zip(hip.named_parameters(), gh, gr, ga):
        assert _rel(a, b) <= 1.3 * _rel(c, b) + 0.02, (name, _rel(a, b), _rel(c, b))
    for bh, br in zip(hip.modules(), ref.modules()):
        if isinstance(bh, torch.nn.BatchNorm2d):
            assert _rel(bh.running_mean, br.running_mean) < 2e-2
            assert _rel(bh.running_var, br.running_var) < 2e-2
            assert int(bh.num_batches_tracked) == int(br.num_batches_tracked) == 1


def test_two_live_graphs_use_separate_plans():
    """SRGAN's D(sr.detach()) and D(hr) are both alive at one backward."""
    hip, ref = _pair(1)
    amp = copy.deepcopy(ref)
    g = torch.Generator().manual_seed(6)
    a = torch.randn(2, 3, 64, 64, generator=g).to(DEV)
    b = torch.randn(2, 3, 64, 64, generator=g).to(DEV)
    (hip(a).sum() - hip(b).sum()).backward()
    (ref(a).sum() - ref(b).sum()).backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        la = amp(a).float().sum() - amp(b).float().sum()
    la.backward()
    for ph, pr, pa in zip(hip.parameters(), ref.parameters(), amp.parameters()):
        assert _rel(ph.grad, pr.grad) <= 1.3 * _rel(pa.grad, pr.grad) + 0.02
    plans = next(iter(hip.__dict__["_isr_plans"].values()))
    assert len(plans) == 2 and not any(p.busy for p in plans)


def test_frozen_parameters_skip_weight_gradients():
    """trainer.train_srgan freezes D for the generator-loss forward: the input
    gradient is unchanged and no parameter gradient is produced."""
    from image_super_resolution_amd import trainer
    hip, _ = _pair(2)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, 3, 64, 64, generator=g).to(DEV)
    _, dx_full, _ = _run(hip, x, 1.0)
    hip.zero_grad(set_to_none=True)
    xr = x.clone().requires_grad_()
    with trainer._frozen(hip):
        o = hip(xr)
    assert all(p.requires_grad for p in hip.parameters())
    o.float().sum().backward()
    assert torch.equal(xr.grad, dx_full)
    assert all(p.grad is None for p in hip.parameters())


def _disc_from_golden(g):
    from image_super_resolution_amd.weights import synth_state_dict
    m = models.Discriminator(3, 64, 8, 1024)
    m.load_state_dict(synth_state_dict(m.state_dict(), int(g["seed"])))
    return m.train()


def _grads_vs(g, m, x, w, autocast=False):
    o, dx, grads = _run(m, x, w, autocast)
    names = [k for k, _ in m.named_parameters()]
    out = {}
    for k, gr in zip(names, grads):
        flat = gr.flatten()
        if f"gidx:{k}" in g:  # large tensors: the golden's whole-tensor sample (make_golden.py)
            flat = flat[torch.from_numpy(g[f"gidx:{k}"].astype("int64")).to(flat.device)]
        out[k] = flat
    return o, dx, out


def test_discriminator_vs_reference_golden(golden):
    """pin D to the reference itself (tests/golden/disc.npz, the reference's
    Discriminator(3,64,8,1024) in train mode, utils/models.py:513-569): logits, input
    gradient, parameter gradients and BN running stats of the HIP discriminator vs the
    reference's fp32 outputs.  Bar for gradients: the error torch's own bf16 autocast
    makes against the same golden on the same tensors (the reference trains D under
    fp16 autocast, train.py:91, :114): hip <= 1.3 x autocast + 0.02.  Tensors above 16,384
    elements are compared on 16,384 elements drawn over the whole tensor (every output channel
    and tap of the 512->512 layers), whose indices the golden stores."""
    from conftest import t
    g = golden("disc")
    x, w = t(g["x"]).to(DEV), t(g["w"]).to(DEV)
    hip = _disc_from_golden(g).to(DEV).use_libisr(True)
    amp = _disc_from_golden(g).to(DEV)
    oh, dxh, gh = _grads_vs(g, hip, x, w)
    oa, dxa, ga = _grads_vs(g, amp, x, w, autocast=True)
    y_ref, dx_ref = t(g["y"]).to(DEV), t(g["dx"]).to(DEV)
    assert _rel(oh, y_ref) < 0.03, _rel(oh, y_ref)
    assert _rel(dxh, dx_ref) <= 1.3 * _rel(dxa, dx_ref) + 0.02, (_rel(dxh, dx_ref), _rel(dxa, dx_ref))
    worst = []
    for k in gh:
        ref = t(g[f"grad:{k}"]).to(DEV)
        eh, ea = _rel(gh[k], ref), _rel(ga[k], ref)
        worst.append((eh, ea, k))
        assert eh <= 1.3 * ea + 0.02, (k, eh, ea)
    print("worst D grads (hip, autocast):", sorted(worst, reverse=True)[:3])
    bufs = dict(hip.named_buffers())
    for k in g:
        if k.startswith("stat:"):
            assert _rel(bufs[k[5:]], t(g[k]).to(DEV)) < 2e-2, k


def test_repeated_forward_reuses_activations_exactly(monkeypatch):
    """SRGAN's D step repeats the G step's D(sr) (train.py:104 / :126, D not yet updated): the
    plan reuses its stored activations and replays only the BatchNorm running update.  Outputs,
    running statistics and the following backward must equal two full recomputations; a weight
    change (the D optimiser step) or a new input must recompute."""
    torch.manual_seed(3)
    base = models.Discriminator(3, 64, 8, 1024).to(DEV).train()
    x = torch.rand(2, 3, 64, 64, device=DEV) * 2 - 1

    def run(reuse):
        monkeypatch.setattr(D, "REUSE", reuse)
        m = copy.deepcopy(base)
        m.requires_grad_(False)  # the G step: D frozen, input gradient only; the backward frees the plan
        xg = x.clone().requires_grad_(True)
        o1 = D.conv_stack_train(m, xg)
        o1.sum().backward()
        m.requires_grad_(True)  # the D step: D(sr.detach()) on the same storage
        o2 = D.conv_stack_train(m, xg.detach())
        g = torch.autograd.grad(o2.sum(), next(m.parameters()))[0]
        stats = [(b.running_mean.clone(), b.running_var.clone(), int(b.num_batches_tracked))
                 for b in m.modules() if isinstance(b, torch.nn.BatchNorm2d)]
        with torch.no_grad():  # a weight change must force a recompute
            next(m.parameters()).mul_(0.5)
        o3 = D.conv_stack_train(m, x)
        return o1, o2, g, stats, o3

    r, f = run(True), run(False)
    assert torch.equal(r[0].detach(), f[0].detach()) and torch.equal(r[1].detach(), f[1].detach())
    assert torch.equal(r[2], f[2])
    for (m1, v1, n1), (m2, v2, n2) in zip(r[3], f[3]):
        assert torch.equal(m1, m2) and torch.equal(v1, v2) and n1 == n2
    assert torch.equal(r[4].detach(), f[4].detach())
