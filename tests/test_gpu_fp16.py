"""fp16 storage on the inference path (isr_conv_desc / isr_head_desc / isr_tail_desc /
isr_chain_desc .f16, engine.pack_generator(f16=True), the default since round 6).

Kernel numerics vs a plain PyTorch fp32 reference of the same op, inputs and weights rounded to
fp16 first: what remains is fp32 accumulation order plus one fp16 rounding of the output
(2^-11 relative), so the bar is 8x tighter than the bf16 kernels' (tests/test_gpu_kernels.py):
|err| <= 2e-3 * max(1, |ref|) elementwise and mean error < 2.5e-4.  Then the whole generator:
on the committed trained x2 weights the fp16 plan must agree with the fp32 oracle by >= 70 dB
(the bf16 plan's ~60 dB is what left |dPSNR| at 0.04 dB on cfg5)."""
import ctypes
from pathlib import Path

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
F16 = torch.float16
WEIGHTS_X2 = Path(__file__).parent / "golden" / "trained_resnet_x2.safetensors"


def hf(x):
    return x.to(F16).float()


def close(got, ref, tol=2e-3, mean_tol=2.5e-4):
    err = (got - ref).abs()
    lim = tol * torch.clamp(ref.abs(), min=1.0)
    assert bool((err <= lim).all()), f"max err {err.max().item():.3e} (ref max {ref.abs().max().item():.3e})"
    assert err.mean().item() < mean_tol, f"mean err {err.mean().item():.3e}"


def lrelu(x, s):
    return torch.where(x >= 0, x, x * s)


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _mk(n, c, h, w, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(n, c, h, w, generator=g).to(DEV)


def _w(cout, cin, k, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    s = (1.0 / (cin * k * k)) ** 0.5
    return (torch.rand(cout, cin, k, k, generator=g) * 2 - 1).mul(s * 3 ** 0.5).to(DEV)


@pytest.mark.parametrize("n,cin,cout,h,w", [(1, 64, 32, 16, 32), (2, 160, 32, 33, 65), (2, 192, 64, 18, 40),
                                            (1, 64, 64, 7, 5)])
def test_conv3x3_f16_plain(n, cin, cout, h, w):
    from image_super_resolution_amd import ops
    x = _mk(n, cin, h, w, 1)
    W = _w(cout, cin, 3, 2)
    b = torch.randn(cout, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=1, dtype=F16)
    yb = ops.ActBuffer.alloc(n, h, w, cout, 1, DEV, dtype=F16)
    ops.conv3x3(xb, cin, ops.pack_conv3x3(W, f16=True), b, cout, yb, slope=0.01)
    torch.cuda.synchronize()
    assert yb.t.dtype == F16
    close(yb.to_nchw(), lrelu(F.conv2d(hf(x), hf(W), b, padding=1), 0.01))
    assert yb.outside_valid().float().abs().max().item() == 0.0


def test_conv3x3_f16_rdb_final_fold_and_residuals():
    """The RDB final conv in place over its residual: the folded form (r1 == x, identity activation,
    A = (1/s1) I exact in fp16) and the RRDB double residual (r2), as the trunk runs them."""
    from image_super_resolution_amd import ops
    n, h, w = 2, 24, 40
    buf = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV, dtype=F16)
    x = _mk(n, 192, h, w, 3)
    buf.set_nchw(x, 0)
    W = _w(64, 192, 3, 5)
    b = torch.randn(64, device=DEV) * 0.1
    xin = buf.to_nchw(0, 192)
    dst = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV, dtype=F16)
    ops.conv3x3(buf, 192, ops.pack_conv3x3(W, f16=True), b, 64, dst, slope=1.0, r1=buf, s1=0.2)
    r2buf = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV, dtype=F16)
    r2 = _mk(n, 64, h, w, 6)
    r2buf.set_nchw(r2, 0)
    ops.conv3x3(buf, 192, ops.pack_conv3x3(W, f16=True), b, 64, r2buf, slope=1.0, r1=buf, s1=0.2, r2=r2buf, s2=0.2)
    torch.cuda.synchronize()
    ref1 = F.conv2d(xin, hf(W), b, padding=1) * 0.2 + xin[:, :64]
    close(dst.to_nchw(0, 64), ref1)
    close(r2buf.to_nchw(0, 64), ref1 * 0.2 + hf(r2))


def test_conv3x3_f16_pixel_shuffle_and_dual_output():
    from image_super_resolution_amd import ops
    n, h, w = 2, 20, 36
    x = _mk(n, 64, h, w, 7)
    W = _w(256, 64, 3, 8)
    b = torch.randn(256, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=1, dtype=F16)
    yb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, 64, 4, DEV, ha=2 * xb.ha, wa=2 * xb.wa, dtype=F16)
    ops.conv3x3(xb, 64, ops.pack_conv3x3(W, f16=True), b, 256, yb, slope=0.01, shuffle=2)
    W2 = _w(64, 64, 3, 10)
    y1 = ops.ActBuffer.alloc(n, h, w, 64, 1, DEV, dtype=F16)
    y2 = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV, dtype=F16)
    ops.conv3x3(xb, 64, ops.pack_conv3x3(W2, f16=True), None, 64, y1, slope=1.0, y2=y2)
    torch.cuda.synchronize()
    close(yb.to_nchw(), lrelu(F.pixel_shuffle(F.conv2d(hf(x), hf(W), b, padding=1), 2), 0.01))
    assert yb.outside_valid().float().abs().max().item() == 0.0
    assert torch.equal(y1.to_nchw(), y2.to_nchw(0, 64))
    close(y1.to_nchw(), F.conv2d(hf(x), hf(W2), padding=1))


@pytest.mark.parametrize("u8", [False, True])
def test_head9x9_f16(u8):
    from image_super_resolution_amd import ops
    from image_super_resolution_amd.weights import normalize
    n, h, w = 2, 20, 36
    g = torch.Generator().manual_seed(11)
    img = torch.rand(n, 3, h, w, generator=g).to(DEV)
    if u8:
        x = (img * 255).to(torch.uint8)
        xin = normalize(x.float() / 255.0)
    else:
        x = normalize(img)
        xin = x
    W = _w(64, 3, 9, 12)
    b = torch.randn(64, device=DEV) * 0.1
    y = ops.ActBuffer.alloc(n, h, w, 64, 1, DEV, dtype=F16)
    y2 = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV, dtype=F16)
    ops.head9x9(x, ops.pack_head9x9(W, f16=True), b, y, slope=0.2, y2=y2)
    torch.cuda.synchronize()
    close(y.to_nchw(), lrelu(F.conv2d(hf(xin), hf(W), b, padding=4), 0.2))
    assert torch.equal(y.to_nchw(), y2.to_nchw(0, 64))


@pytest.mark.parametrize("n,h,w", [(2, 40, 72), (3, 96, 64)])
def test_tail9x9_f16_stream_vs_per_tile_and_ref(n, h, w):
    """The production row-streaming tail (variant 5) and its large-image fallback (3) in fp16: bit
    for bit the same sums, and within the fp16 bar of the fp32 reference."""
    from image_super_resolution_amd import _lib, ops
    lib = _lib.load()
    x = _mk(n, 64, h, w, 21) * 0.5
    W = _w(3, 64, 9, 22)
    b = torch.randn(3, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=4, dtype=F16)
    wp = ops.pack_tail9x9(W, f16=True)

    def run(v, dt):
        o = torch.full((n, 3, h, w), 7, device=DEV, dtype=dt)
        d = ops.tail9x9_desc(xb, wp, b, o)
        assert d.f16 == 1
        ops.check(lib.isr_tail9x9_fwd_variant(ctypes.byref(d), v, ops._stream()), f"tail variant {v}")
        torch.cuda.synchronize()
        return o

    ref = torch.tanh(F.conv2d(hf(x), hf(W), b, padding=4))
    for dt in (torch.float32, torch.uint8):
        a = run(5, dt)
        assert torch.equal(run(3, dt), a) and torch.equal(run(0, dt), a)
        if dt == torch.float32:
            close(a, ref, tol=1e-3, mean_tol=1e-4)
        else:
            d = (a.float() - ((ref + 1) / 2 * 255).round()).abs()
            assert d.max().item() <= 1 and (d > 0).float().mean().item() < 0.01


def test_mixed_storage_is_refused():
    """One launch, one storage type: fp16 weights on bf16 activations (or the reverse) raise
    on the host before anything is launched, and the C ABI refuses fp16 backward forms."""
    from image_super_resolution_amd import _lib, ops
    W = _w(64, 64, 3, 1)
    xb = ops.ActBuffer.alloc(1, 16, 32, 64, 1, DEV)
    yh = ops.ActBuffer.alloc(1, 16, 32, 64, 1, DEV, dtype=F16)
    with pytest.raises(TypeError):
        ops.conv3x3_desc(xb, 64, ops.pack_conv3x3(W, f16=True), None, 64, xb)
    with pytest.raises(TypeError):
        ops.conv3x3_desc(xb, 64, ops.pack_conv3x3(W), None, 64, yh)
    xh = ops.ActBuffer.alloc(1, 16, 32, 64, 1, DEV, dtype=F16)
    d = ops.conv3x3_desc(xh, 64, ops.pack_conv3x3(W, f16=True), None, 64, yh)
    d.m = yh.view(0)  # an fp16 backward (LeakyReLU' mask) form: not built
    assert _lib.load().isr_conv3x3_fwd(ctypes.byref(d), ops._stream()) != 0


@torch.no_grad()
def test_trained_x2_generator_fp16_vs_bf16_vs_oracle():
    """The whole ResNet(16, 0.2, x2) forward on the trained weights, chained trunk, fp16 vs bf16
    storage against the fp32 oracle on a held-out crop: fp16 must agree by >= 70 dB and beat bf16
    by >= 10 dB; its |dPSNR| vs HR stays far inside the 0.01 dB bar."""
    from image_super_resolution_amd import checkpoint, engine, models
    from image_super_resolution_amd.weights import heldout_still
    from oracle import ref_cpu as R
    sd = {k: v.float() for k, v in checkpoint.load_module_state(WEIGHTS_X2).items()}
    net = models.ResNet(16, 0.2, scaleRate=2)
    net.load_state_dict(sd)
    lr, hr = heldout_still(96, 128, 2, device="cpu")
    xin = R.normalize_u8(lr[None])
    ref = R.generator(R.fuse_state_dict(sd), xin, num_blocks=16, scale=2)
    hr1 = hr[None].float() / 127.5 - 1
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    dsd = {k: v.to(DEV) for k, v in R.fuse_state_dict(sd).items()}
    x = xin.to(DEV).contiguous()
    res = {}
    for f16 in (True, False):
        gw = engine.pack_generator(dsd, enchant=False, add_rate=0.2, device=DEV, f16=f16)
        assert gw.dtype == (F16 if f16 else torch.bfloat16)
        plan = engine.GeneratorPlan(gw, 1, 96, 128, torch.device(DEV), False, False, mean, std, chain=True)
        assert plan.chain is not None
        y = torch.empty(plan.out_shape, device=DEV)
        plan.run(x, y)
        plan.verify()
        y = y.cpu()
        res[f16] = (R.psnr(y, ref), abs(R.psnr(y, hr1) - R.psnr(ref, hr1)))
        del plan
    print(f"x2 trained, 96x128 crop: fp16 {res[True][0]:.2f} dB (dPSNR {res[True][1]:.5f}), "
          f"bf16 {res[False][0]:.2f} dB (dPSNR {res[False][1]:.5f})")
    assert res[True][0] >= 70.0 and res[True][0] >= res[False][0] + 10.0, res
    assert res[True][1] <= 0.002, res


@torch.no_grad()
def test_plan_keeps_its_packed_weights_alive():
    """A GeneratorPlan's descriptors point into its GeneratorWeights' packed tensors: the plan must
    keep them alive.  Build a bf16 plan, drop every other reference to its weights, pack fp16
    weights of the same shapes (which would reuse the freed blocks) and rerun: the output is
    unchanged (round 6: tools/ab_storage.py's bf16 plan ran on fp16 bits after exactly this)."""
    import gc

    from image_super_resolution_amd import engine, models
    from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict
    sd = {k: v.to(DEV) for k, v in synth_state_dict(models.ResNet(2, 0.2, scaleRate=4).state_dict(), 0).items()}
    x = normalize(synth_lr_batch(2, 32, 32, seed=1)[0]).to(DEV).contiguous()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    plan = engine.GeneratorPlan(engine.pack_generator(sd, enchant=False, device=DEV, f16=False), 2, 32, 32,
                                torch.device(DEV), False, False, mean, std, chain=True)
    y0 = torch.empty(plan.out_shape, device=DEV)
    plan.run(x, y0)
    torch.cuda.synchronize()
    gc.collect()
    others = [engine.pack_generator(sd, enchant=False, device=DEV, f16=True) for _ in range(2)]
    y1 = torch.empty(plan.out_shape, device=DEV)
    plan.run(x, y1)
    plan.verify()
    assert others and torch.isfinite(y1).all() and torch.equal(y0, y1)
