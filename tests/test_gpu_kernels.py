"""HIP kernel numerics vs a plain PyTorch fp32 reference of the same op.

Inputs and weights are rounded to bf16 first (the kernels' storage type), so
the remaining difference is fp32 accumulation order plus one bf16 rounding of
the output: tolerance |err| <= 1.5e-2 * max(1, |ref|) elementwise, and mean
error < 2e-3.
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def bf(x):
    return x.to(torch.bfloat16).float()


def close(got, ref, tol=1.5e-2, mean_tol=2e-3):
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


def _w(cout, cin, k, seed, scale=None):
    g = torch.Generator(device="cpu").manual_seed(seed)
    s = scale if scale is not None else (1.0 / (cin * k * k)) ** 0.5
    return (torch.rand(cout, cin, k, k, generator=g) * 2 - 1).mul(s * 3 ** 0.5).to(DEV)


@pytest.mark.parametrize("n,cin,cout,h,w", [(1, 64, 32, 16, 32), (2, 96, 32, 20, 36), (1, 160, 32, 33, 65),
                                            (2, 192, 64, 18, 40), (1, 64, 64, 7, 5), (1, 64, 128, 16, 32)])
def test_conv3x3_plain(n, cin, cout, h, w):
    from image_super_resolution_amd import ops
    x = _mk(n, cin, h, w, 1)
    W = _w(cout, cin, 3, 2)
    b = torch.randn(cout, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=1)
    yb = ops.ActBuffer.alloc(n, h, w, cout, 1, DEV)
    ops.conv3x3(xb, cin, ops.pack_conv3x3(W), b, cout, yb, slope=0.01)
    torch.cuda.synchronize()
    ref = lrelu(F.conv2d(bf(x), bf(W), b, padding=1), 0.01)
    close(yb.to_nchw(), ref)
    # everything outside the valid region (border + alignment slack) must stay exactly zero
    assert yb.outside_valid().float().abs().max().item() == 0.0


def test_conv3x3_dense_slice_and_residuals():
    """Growth conv into a channel slice + RDB/RRDB double-residual epilogue."""
    from image_super_resolution_amd import ops
    n, h, w = 2, 24, 40
    buf = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV)
    x = _mk(n, 96, h, w, 3)
    buf.set_nchw(x, 0)
    before = buf.t.clone()
    W = _w(32, 96, 3, 4)
    b = torch.randn(32, device=DEV) * 0.1
    ops.conv3x3(buf, 96, ops.pack_conv3x3(W), b, 32, buf, y_coff=96, slope=0.01)
    torch.cuda.synchronize()
    ref = lrelu(F.conv2d(bf(x), bf(W), b, padding=1), 0.01)
    close(buf.to_nchw(96, 128), ref)
    # channel blocks outside the written slice [96, 128) are untouched
    assert torch.equal(buf.t[:, :6], before[:, :6]) and torch.equal(buf.t[:, 8:], before[:, 8:])

    # final conv: y = ((conv + b) * 0.2 + r1) * 0.2 + r2, written in place over r2
    W2 = _w(64, 192, 3, 5)
    b2 = torch.randn(64, device=DEV) * 0.1
    xin = bf(buf.to_nchw(0, 192))
    r2buf = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV)
    r2 = _mk(n, 64, h, w, 6)
    r2buf.set_nchw(r2, 0)
    ops.conv3x3(buf, 192, ops.pack_conv3x3(W2), b2, 64, r2buf, slope=1.0, r1=buf, s1=0.2, r2=r2buf, s2=0.2)
    torch.cuda.synchronize()
    ref = ((F.conv2d(xin, bf(W2), b2, padding=1)) * 0.2 + xin[:, :64]) * 0.2 + bf(r2)
    close(r2buf.to_nchw(0, 64), ref)


def test_conv3x3_pixel_shuffle():
    from image_super_resolution_amd import ops
    n, h, w = 2, 20, 36
    x = _mk(n, 64, h, w, 7)
    W = _w(256, 64, 3, 8)
    b = torch.randn(256, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=1)
    yb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, 64, 4, DEV, ha=2 * xb.ha, wa=2 * xb.wa)
    ops.conv3x3(xb, 64, ops.pack_conv3x3(W), b, 256, yb, slope=0.01, shuffle=2)
    torch.cuda.synchronize()
    ref = lrelu(F.pixel_shuffle(F.conv2d(bf(x), bf(W), b, padding=1), 2), 0.01)
    close(yb.to_nchw(), ref)
    assert yb.outside_valid().float().abs().max().item() == 0.0


def test_conv3x3_dual_output():
    from image_super_resolution_amd import ops
    x = _mk(1, 64, 16, 32, 9)
    W = _w(64, 64, 3, 10)
    xb = ops.ActBuffer.from_nchw(x, pad=1)
    y1 = ops.ActBuffer.alloc(1, 16, 32, 64, 1, DEV)
    y2 = ops.ActBuffer.alloc(1, 16, 32, 192, 1, DEV)
    ops.conv3x3(xb, 64, ops.pack_conv3x3(W), None, 64, y1, slope=1.0, y2=y2)
    torch.cuda.synchronize()
    assert torch.equal(y1.to_nchw(), y2.to_nchw(0, 64))
    close(y1.to_nchw(), F.conv2d(bf(x), bf(W), padding=1))


@pytest.mark.parametrize("u8", [False, True])
def test_head9x9(u8):
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
    y = ops.ActBuffer.alloc(n, h, w, 64, 1, DEV)
    y2 = ops.ActBuffer.alloc(n, h, w, 192, 1, DEV)
    ops.head9x9(x, ops.pack_head9x9(W), b, y, slope=0.2, y2=y2)
    torch.cuda.synchronize()
    ref = lrelu(F.conv2d(bf(xin), bf(W), b, padding=4), 0.2)
    close(y.to_nchw(), ref)
    assert torch.equal(y.to_nchw(), y2.to_nchw(0, 64))


@pytest.mark.parametrize("u8", [False, True])
def test_tail9x9(u8):
    from image_super_resolution_amd import ops
    n, h, w = 2, 40, 72
    x = _mk(n, 64, h, w, 13) * 0.5
    W = _w(3, 64, 9, 14)
    b = torch.randn(3, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=4)
    out = torch.empty(n, 3, h, w, device=DEV, dtype=torch.uint8 if u8 else torch.float32)
    ops.tail9x9(xb, ops.pack_tail9x9(W), b, out)
    torch.cuda.synchronize()
    ref = torch.tanh(F.conv2d(bf(x), bf(W), b, padding=4))
    if u8:
        ref8 = (((ref + 1) / 2) * 255).round()
        d = (out.float() - ref8).abs()
        assert d.max().item() <= 1 and (d > 0).float().mean().item() < 0.02
    else:
        close(out, ref, tol=5e-3, mean_tol=5e-4)


@pytest.mark.parametrize("n,h,w", [(2, 40, 72), (5, 128, 160), (3, 96, 64), (2, 300, 96)])
def test_tail9x9_persistent_vs_per_tile(n, h, w):
    """The production row-streaming tail (variant 5, 8 waves; segment heights 16 / 128 / 32 / 16
    here) vs the 8-row per-tile kernel (variant 3, its large-image fallback): the same sums in the
    same order, so bit-identical, and run-to-run bit equality.  With the tuning library
    (ISR_LIB=.../libisr_tuning.so) also the A/B forms: the 16-row per-tile kernel (1), the
    persistent kernel (2), the 4-wave walk (4) and the lane-streaming walk (6)."""
    import ctypes
    import os
    from image_super_resolution_amd import ops, _lib
    lib = _lib.load()
    tuning = "tuning" in os.environ.get("ISR_LIB", "")
    x = _mk(n, 64, h, w, 21) * 0.5
    W = _w(3, 64, 9, 22)
    b = torch.randn(3, device=DEV) * 0.1
    xb = ops.ActBuffer.from_nchw(x, pad=4)
    wp = ops.pack_tail9x9(W)

    def run(v, dt, fill=None):
        o = torch.empty(n, 3, h, w, device=DEV, dtype=dt) if fill is None else \
            torch.full((n, 3, h, w), fill, device=DEV, dtype=dt)
        d = ops.tail9x9_desc(xb, wp, b, o)
        ops.check(lib.isr_tail9x9_fwd_variant(ctypes.byref(d), v, ops._stream()), f"tail variant {v}")
        torch.cuda.synchronize()
        return o

    for dt in (torch.float32, torch.uint8):
        a = run(3, dt)
        p0, p1 = run(5, dt, fill=7), run(5, dt, fill=7)
        assert torch.equal(p0, a) and torch.equal(p1, a)
        assert torch.equal(run(0, dt, fill=7), a)  # variant 0 = the production choice
        if tuning:
            for v in (1, 4, 6):
                assert torch.equal(run(v, dt, fill=7), a), v
            q0, q1 = run(2, dt), run(2, dt)  # persistent: its own order, run-to-run equal
            assert torch.equal(q0, q1)
            if dt == torch.float32:
                assert (a - q0).abs().max().item() < 1e-5
            else:
                dd = (a.float() - q0.float()).abs()
                assert dd.max().item() <= 1 and (dd > 0).float().mean().item() < 1e-3


def test_bad_descriptor_raises():
    from image_super_resolution_amd import ops, _lib
    x = ops.ActBuffer.alloc(1, 16, 32, 48, 1, DEV)
    y = ops.ActBuffer.alloc(1, 16, 32, 64, 1, DEV)
    with pytest.raises(_lib.IsrError, match="multiple of 16"):  # cin 40: not a whole K-step
        ops.conv3x3(x, 40, torch.zeros(10, dtype=torch.bfloat16, device=DEV), None, 64, y)
    with pytest.raises(_lib.IsrError, match="multiple of 32"):  # cout 48: not a whole MFMA tile
        ops.conv3x3(x, 48, torch.zeros(10, dtype=torch.bfloat16, device=DEV), None, 48, y)


def test_conv3x3_backward_epilogue_mask_and_limited_residual():
    """dgrad-style launch: r1 added to the first r1_cn channels only, LeakyReLU'
    mask (from a forward activation buffer) on channels >= m_c0."""
    from image_super_resolution_amd import ops
    n, h, w, cin, cout = 2, 20, 36, 64, 192
    x = _mk(n, cin, h, w, 21)
    W = _w(cout, cin, 3, 22)
    r = _mk(n, cout, h, w, 23)
    act = _mk(n, cout, h, w, 24)
    xb = ops.ActBuffer.from_nchw(x, pad=1)
    rb = ops.ActBuffer.from_nchw(r, pad=1)
    mb = ops.ActBuffer.from_nchw(act, pad=1)
    yb = ops.ActBuffer.alloc(n, h, w, cout, 1, DEV)
    ops.conv3x3(xb, cin, ops.pack_conv3x3(W), None, cout, yb, r1=rb, r1_cn=64, m=mb, m_c0=160, mslope=0.01)
    torch.cuda.synchronize()
    ref = F.conv2d(bf(x), bf(W), padding=1)
    ref[:, :64] += bf(r)[:, :64]
    ref[:, 160:] *= torch.where(bf(act)[:, 160:] > 0, 1.0, 0.01)
    close(yb.to_nchw(), ref)
    assert yb.outside_valid().float().abs().max().item() == 0.0


def test_conv3x3_in_place_accumulate_with_mask():
    """RDB dgrad step: G[0:cout] += conv(G[cin slot]) in place, last 32 channels masked."""
    from image_super_resolution_amd import ops
    n, h, w = 1, 18, 40
    g = _mk(n, 192, h, w, 31)
    act = _mk(n, 192, h, w, 32)
    gb = ops.ActBuffer.from_nchw(g, pad=1)
    mb = ops.ActBuffer.from_nchw(act, pad=1)
    W = _w(160, 32, 3, 33)
    ops.conv3x3(gb, 32, ops.pack_conv3x3(W), None, 160, gb, x_coff=160, r1=gb, m=mb, m_c0=128, mslope=0.2)
    torch.cuda.synchronize()
    ref = F.conv2d(bf(g)[:, 160:], bf(W), padding=1) + bf(g)[:, :160]
    ref[:, 128:] *= torch.where(bf(act)[:, 128:160] > 0, 1.0, 0.2)
    close(gb.to_nchw(0, 160), ref)
    assert torch.equal(gb.to_nchw(160, 192), bf(g)[:, 160:])


@pytest.mark.parametrize("h,w", [(16, 32), (20, 36), (40, 24)])
def test_conv3x3_x_sub2_is_pixel_unshuffle(h, w):
    """Input read as PixelShuffle(2)ᵀ of a 2h x 2w buffer (scaler backward)."""
    from image_super_resolution_amd import ops
    n, cs, cout = 2, 64, 64
    g = _mk(n, cs, 2 * h, 2 * w, 41)
    Wu = _w(cout, 4 * cs, 3, 42)  # weights over pixel_unshuffle channel order 4c + 2i + j
    lr = ops.ActBuffer.alloc(n, h, w, cout, 1, DEV)
    gb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, cs, 2, DEV, ha=2 * lr.ha, wa=2 * lr.wa)
    gb.set_nchw(g, 0)
    Wk = Wu.view(cout, cs, 4, 3, 3).transpose(1, 2).reshape(cout, 4 * cs, 3, 3).contiguous()
    ops.conv3x3(gb, 4 * cs, ops.pack_conv3x3(Wk), None, cout, lr, x_sub2=True)
    torch.cuda.synchronize()
    ref = F.conv2d(F.pixel_unshuffle(bf(g), 2), bf(Wu), padding=1)
    close(lr.to_nchw(), ref)


def _wgrad_ref(x, g, scale=1.0):
    """autograd reference: dW, db of y = conv2d(x, W, b, padding=1) for upstream grad g."""
    cin, cout = x.shape[1], g.shape[1]
    W = torch.zeros(cout, cin, 3, 3, device=DEV, requires_grad=True)
    b = torch.zeros(cout, device=DEV, requires_grad=True)
    y = F.conv2d(x, W, b, padding=1)
    y.backward(g)
    return W.grad * scale, b.grad * scale


def _close_rel(got, ref, tol=2e-2):
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < tol, f"relative L2 error {rel:.3e}"
    lim = tol * ref.abs().max().item()
    assert (got - ref).abs().max().item() <= lim * 2, f"max err {(got - ref).abs().max().item():.3e}"


@pytest.mark.parametrize("n,cin,cout,h,w,splits", [(2, 64, 32, 20, 36, 0), (1, 96, 32, 33, 65, 0),
                                                   (2, 192, 64, 18, 40, 0), (1, 64, 64, 7, 5, 3),
                                                   (2, 32, 160, 16, 32, 0), (1, 64, 192, 24, 24, 1),
                                                   (1, 192, 64, 20, 36, 5), (1, 160, 32, 9, 70, 0)])
def test_wgrad3x3(n, cin, cout, h, w, splits):
    from image_super_resolution_amd import ops
    x = bf(_mk(n, cin, h, w, 51))
    g = bf(_mk(n, cout, h, w, 52))
    xb = ops.ActBuffer.from_nchw(x, pad=1)
    gb = ops.ActBuffer.from_nchw(g, pad=1)
    dw = torch.empty(cout, cin, 3, 3, device=DEV)
    db = torch.empty(cout, device=DEV)
    ops.wgrad3x3(xb, cin, gb, cout, dw, db, scale=0.5, splits=splits)
    torch.cuda.synchronize()
    rw, rb = _wgrad_ref(x, g, 0.5)
    _close_rel(dw, rw, 1e-3)
    _close_rel(db, rb, 1e-3)


def test_wgrad3x3_dense_slices_and_sub2():
    """wgrad reading channel slices of a dense buffer, and the Scaler's
    PixelShuffle'd gradient (g_sub2) with reference channel order."""
    from image_super_resolution_amd import ops
    n, h, w = 2, 20, 24
    dense = _mk(n, 192, h, w, 61)
    db_ = ops.ActBuffer.from_nchw(dense, pad=1)
    dw = torch.empty(32, 128, 3, 3, device=DEV)
    ops.wgrad3x3(db_, 128, db_, 32, dw, None, g_coff=160)
    torch.cuda.synchronize()
    rw, _ = _wgrad_ref(bf(dense)[:, :128], bf(dense)[:, 160:192])
    _close_rel(dw, rw, 1e-3)
    # Scaler: y = shuffle(conv(x)); grad wrt conv output = pixel_unshuffle(g_hr)
    x = bf(_mk(n, 64, h, w, 62))
    ghr = bf(_mk(n, 64, 2 * h, 2 * w, 63))
    xb = ops.ActBuffer.from_nchw(x, pad=1)
    gb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, 64, 2, DEV, ha=2 * xb.ha, wa=2 * xb.wa)
    gb.set_nchw(ghr, 0)
    dw = torch.empty(256, 64, 3, 3, device=DEV)
    dbias = torch.empty(256, device=DEV)
    ops.wgrad3x3(xb, 64, gb, 256, dw, dbias, g_sub2=True)
    torch.cuda.synchronize()
    rw, rb = _wgrad_ref(x, F.pixel_unshuffle(ghr, 2))
    _close_rel(dw, rw, 1e-3)
    _close_rel(dbias, rb, 1e-3)


@pytest.mark.parametrize("n,h,w", [(2, 20, 36), (1, 33, 40)])
def test_wgrad3x3_group_rdb_vs_autograd(n, h, w):
    """isr_wgrad3x3_group: an RDB's five weight gradients in one launch (dense buffer D =
    [x | o0 | o1 | o2 | o3], gradient buffer E = [g_out | g_3 | g_2 | g_1 | g_0]) vs autograd,
    and vs the five separate isr_wgrad3x3 launches (same sums, other split-K partition)."""
    import ctypes
    from image_super_resolution_amd import _lib, ops
    lib = _lib.load()
    D = bf(_mk(n, 192, h, w, 81))
    E = bf(_mk(n, 192, h, w, 82))
    Db, Eb = ops.ActBuffer.from_nchw(D, pad=1), ops.ActBuffer.from_nchw(E, pad=1)
    shapes = [(192, 64, 0, 0.04), (64 + 32 * 3, 32, 64, 1.0), (64 + 32 * 2, 32, 96, 1.0), (64 + 32, 32, 128, 1.0),
              (64, 32, 160, 1.0)]  # (cin, cout, g_coff, scale): final conv, growth 3 .. 0
    outs, descs = [], []
    for cin, cout, gco, sc in shapes:
        dw = torch.empty(cout, cin, 3, 3, device=DEV)
        db = torch.empty(cout, device=DEV)
        outs.append((dw, db))
        descs.append(ops.wgrad3x3_desc(Db, cin, Eb, cout, dw, db, g_coff=gco, scale=sc))
    arr = (_lib.IsrWgradDesc * 5)(*descs)
    nbytes = lib.isr_wgrad3x3_group_workspace_bytes(arr, 5)
    assert nbytes > 0
    ws = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.isr_wgrad3x3_group(arr, 5, ws.data_ptr(), ws.numel(), st) == 0
    assert lib.isr_wgrad3x3_group(arr, 5, ws.data_ptr(), nbytes - 4, st) != 0  # short workspace refused
    torch.cuda.synchronize()
    for (cin, cout, gco, sc), (dw, db) in zip(shapes, outs):
        rw, rb = _wgrad_ref(D[:, :cin], E[:, gco:gco + cout], sc)
        _close_rel(dw, rw, 1e-3)
        _close_rel(db, rb, 1e-3)
        dw1, db1 = torch.empty_like(dw), torch.empty_like(db)
        ops.wgrad3x3(Db, cin, Eb, cout, dw1, db1, g_coff=gco, scale=sc)
        torch.cuda.synchronize()
        torch.testing.assert_close(dw, dw1, rtol=1e-5, atol=1e-5 * dw1.abs().max().item())
    # the member-major block order (ISR_WGRAD_GROUP_ORDER=0) gives the same bits as the default
    # split-major one: same blocks, same partials, same reduce
    old = os.environ.get("ISR_WGRAD_GROUP_ORDER")
    os.environ["ISR_WGRAD_GROUP_ORDER"] = "0"
    try:
        ref = [(dw.clone(), db.clone()) for dw, db in outs]
        for dw, db in outs:
            dw.fill_(float("nan"))
            db.fill_(float("nan"))
        assert lib.isr_wgrad3x3_group(arr, 5, ws.data_ptr(), ws.numel(), st) == 0
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("ISR_WGRAD_GROUP_ORDER")
        else:
            os.environ["ISR_WGRAD_GROUP_ORDER"] = old
    for (dw, db), (rw, rb) in zip(outs, ref):
        assert torch.equal(dw, rw) and torch.equal(db, rb)
    # a member on another computed grid (ha) is refused
    Ds = ops.ActBuffer.from_nchw(bf(_mk(n, 64, h + 64, w, 83)), pad=1)  # another computed extent
    bad = list(descs)
    bad[4] = ops.wgrad3x3_desc(Ds, 64, Eb, 32, outs[4][0], None, g_coff=160)
    arr2 = (_lib.IsrWgradDesc * 5)(*bad)
    assert lib.isr_wgrad3x3_group_workspace_bytes(arr2, 5) == 0


# every production form of the weight gradient (wgrad3x3.hip pick_default<1>) — ha is always a
# multiple of ISR_TILE_H = 32 (the ABI validates it), so the 4- and 2-row fallbacks of that pick
# are unreachable; `kind`: plain, g_sub2 (the Scaler: gradient read through PixelShuffle(2)),
# x_sub2 taps=1 (the discriminator's stride-2 convs on the phase decomposition)
WGRAD_FORMS = [
    (64, 32, "plain"),     # row sweep WG::RS (8-row stages, 2 waves per kernel column)
    (128, 32, "plain"),    # row sweep
    (64, 64, "plain"),     # row sweep, two cout tiles
    (96, 32, "plain"),     # cin % 64 == 32: 4-row stages, asm reads (WG::AR)
    (160, 32, "plain"),    # the same form at cin 160
    (192, 64, "plain"),    # RDB final conv: 64 x 96 ci-split tile, asm reads without read-ahead (AR 2)
    (128, 128, "plain"),   # discriminator wide form, 128 ci per block
    (128, 256, "plain"),   # the same, two 128-cout tiles
    (64, 128, "plain"),    # discriminator wide form, 64 ci per block
    (64, 256, "g_sub2"),   # Scaler weight gradient (row sweep on the PixelShuffle'd gradient)
    (256, 64, "x_sub2"),   # stride-2 phase conv, wide taps=1 form
    (256, 32, "x_sub2"),   # stride-2 phase conv, 32-cout taps=1 form (4 waves)
]


@pytest.mark.parametrize("cin,cout,kind", WGRAD_FORMS)
def test_wgrad3x3_asm_read_forms_bitwise(cin, cout, kind):
    """The production forms read LDS through inline asm with hand-counted lgkmcnt waits (row sweep
    WG::RS, asm-read kernel-row forms WG::AR); variant 16 runs the same tiles, split counts and MFMA
    order with compiler-visible LDS reads.  dW / db must be bit-identical — a fragment read before
    its wait, a compiler copy of an asm destination or an SMEM load under a counted wait would show
    here as a difference (the static side is tools/check_lds_waits.py in the build)."""
    import ctypes
    from image_super_resolution_amd import _lib, ops
    lib = _lib.load()
    n, h, w = 2, 40, 72
    if kind == "plain":
        xb = ops.ActBuffer.from_nchw(bf(_mk(n, cin, h, w, 91)), pad=1)
        gb = ops.ActBuffer.from_nchw(bf(_mk(n, cout, h, w, 92)), pad=1)
        kw = {}
    elif kind == "g_sub2":  # x at LR, the gradient of the 64-channel PixelShuffle output at 2x
        xb = ops.ActBuffer.from_nchw(bf(_mk(n, cin, h, w, 91)), pad=1)
        gb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, cout // 4, 2, DEV, ha=2 * xb.ha, wa=2 * xb.wa)
        gb.set_nchw(bf(_mk(n, cout // 4, 2 * h, 2 * w, 92)), 0)
        kw = dict(g_sub2=True)
    else:  # x at 2x with cin / 4 channels, read as PixelUnshuffle(2); the gradient at LR
        gb = ops.ActBuffer.from_nchw(bf(_mk(n, cout, h, w, 92)), pad=1)
        xb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, cin // 4, 2, DEV, ha=2 * gb.ha, wa=2 * gb.wa)
        xb.set_nchw(bf(_mk(n, cin // 4, 2 * h, 2 * w, 91)), 0)
        kw = dict(x_sub2=True, taps=1)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = []
    for v in (0, 16):
        dw = torch.full((cout, cin, 3, 3), float("nan"), device=DEV)
        db = None if kind == "x_sub2" else torch.full((cout,), float("nan"), device=DEV)
        d = ops.wgrad3x3_desc(xb, cin, gb, cout, dw, db, scale=0.25, **kw)
        nb = lib.isr_wgrad3x3_variant_workspace_bytes(ctypes.byref(d), v)
        assert nb > 0
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        assert lib.isr_wgrad3x3_variant(ctypes.byref(d), v, ws.data_ptr(), nb, st) == 0
        torch.cuda.synchronize()
        res.append((dw, db))
    taps = slice(0, 2) if kind == "x_sub2" else slice(0, 3)
    assert torch.isfinite(res[0][0][..., taps, taps]).all()
    assert torch.equal(res[0][0][..., taps, taps], res[1][0][..., taps, taps])
    if res[0][1] is not None:
        assert torch.equal(res[0][1], res[1][1])
    if kind == "plain":
        rw, _ = _wgrad_ref(xb.to_nchw(0, cin), gb.to_nchw(0, cout), 0.25)
        _close_rel(res[0][0], rw, 1e-3)
    # the round-1..4 tile forms are tuning-build only: a production library refuses them
    if "tuning" not in os.environ.get("ISR_LIB", ""):
        d = ops.wgrad3x3_desc(xb, cin, gb, cout, res[0][0], res[0][1], **kw)
        assert lib.isr_wgrad3x3_variant_workspace_bytes(ctypes.byref(d), 5) == 0


def test_wgrad3x3_group_asm_reads_bitwise():
    """The grouped RDB launch (row sweep, asm reads) against its compiler-read form of the same
    tiles and splits (isr_wgrad3x3_group_variant 1): bit-identical, on a 4x-cfg3-shaped RDB."""
    import ctypes
    from image_super_resolution_amd import _lib, ops
    lib = _lib.load()
    n, h, w = 2, 40, 72
    Db = ops.ActBuffer.from_nchw(bf(_mk(n, 192, h, w, 81)), pad=1)
    Eb = ops.ActBuffer.from_nchw(bf(_mk(n, 192, h, w, 82)), pad=1)
    shapes = [(192, 64, 0, 0.04), (160, 32, 64, 1.0), (128, 32, 96, 1.0), (96, 32, 128, 1.0), (64, 32, 160, 1.0)]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = []
    for v in (0, 1):
        outs = [(torch.full((co, ci, 3, 3), float("nan"), device=DEV), torch.full((co,), float("nan"), device=DEV))
                for ci, co, _, _ in shapes]
        arr = (_lib.IsrWgradDesc * 5)(*[ops.wgrad3x3_desc(Db, ci, Eb, co, dw, db, g_coff=gco, scale=sc)
                                         for (ci, co, gco, sc), (dw, db) in zip(shapes, outs)])
        nbytes = lib.isr_wgrad3x3_group_workspace_bytes(arr, 5)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
        assert lib.isr_wgrad3x3_group_variant(arr, 5, v, ws.data_ptr(), nbytes, st) == 0
        torch.cuda.synchronize()
        res.append(outs)
    for (a, b), (c, d) in zip(res[0], res[1]):
        assert torch.isfinite(a).all() and torch.equal(a, c) and torch.equal(b, d)


def test_wgrad3x3_partials_then_reduce_equals_one_call():
    """isr_wgrad3x3_partials + isr_wgrad3x3_reduce (the reduce on another stream) == isr_wgrad3x3,
    bit for bit (same partition, same summation order)."""
    import ctypes
    from image_super_resolution_amd import _lib, ops
    lib = _lib.load()
    x, g = bf(_mk(2, 128, 24, 40, 91)), bf(_mk(2, 32, 24, 40, 92))
    xb, gb = ops.ActBuffer.from_nchw(x, pad=1), ops.ActBuffer.from_nchw(g, pad=1)
    dw0, dw1 = torch.empty(32, 128, 3, 3, device=DEV), torch.empty(32, 128, 3, 3, device=DEV)
    ops.wgrad3x3(xb, 128, gb, 32, dw0)
    d = ops.wgrad3x3_desc(xb, 128, gb, 32, dw1)
    nbytes = lib.isr_wgrad3x3_workspace_bytes(ctypes.byref(d))
    ws = torch.empty(nbytes, dtype=torch.uint8, device=DEV)
    s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream()
    assert lib.isr_wgrad3x3_partials(ctypes.byref(d), ws.data_ptr(), nbytes, ctypes.c_void_p(s1.cuda_stream)) == 0
    s2.wait_stream(s1)
    assert lib.isr_wgrad3x3_reduce(ctypes.byref(d), ws.data_ptr(), nbytes, ctypes.c_void_p(s2.cuda_stream)) == 0
    torch.cuda.synchronize()
    assert torch.equal(dw0, dw1)


def test_dgrad_via_transposed_pack():
    """Input gradient = conv3x3 with the dgrad-packed weights (incl. scale and the
    Scaler's x_sub2 order) vs autograd."""
    from image_super_resolution_amd import ops
    n, h, w = 2, 20, 36
    for cin, cout, sub2 in [(64, 32, False), (32, 160, False), (192, 64, False), (64, 256, True)]:
        x = _mk(n, cin, h, w, 71).requires_grad_(True)
        W = _w(cout, cin, 3, 72)
        y = F.conv2d(x, bf(W), padding=1)
        gy = bf(_mk(n, cout, h, w, 73))
        if sub2:
            ghr = bf(_mk(n, cout // 4, 2 * h, 2 * w, 74))
            gy = F.pixel_unshuffle(ghr, 2)
        y.backward(gy)
        wp = ops.pack_conv3x3_dgrad(W, scale=0.25, sub2=sub2)
        out = ops.ActBuffer.alloc(n, h, w, cin, 1, DEV)
        if sub2:
            gb = ops.ActBuffer.alloc(n, 2 * h, 2 * w, cout // 4, 2, DEV, ha=2 * out.ha, wa=2 * out.wa)
            gb.set_nchw(ghr, 0)
        else:
            gb = ops.ActBuffer.from_nchw(gy, pad=1)
        ops.conv3x3(gb, cout, wp, None, cin, out, x_sub2=sub2)
        torch.cuda.synchronize()
        close(out.to_nchw(), x.grad * 0.25)


def _wgrad9_ref(inp, gout, cin, cout):
    W = torch.zeros(cout, cin, 9, 9, device=DEV, requires_grad=True)
    b = torch.zeros(cout, device=DEV, requires_grad=True)
    F.conv2d(inp, W, b, padding=4).backward(gout)
    return W.grad, b.grad


@pytest.mark.parametrize("n,h,w", [(2, 20, 36), (1, 64, 64), (3, 7, 70)])
def test_wgrad9x9_tail_and_head(n, h, w):
    from image_super_resolution_amd import ops
    # tail conv2: 64 → 3 on the HR grid
    U = bf(_mk(n, 64, h, w, 81))
    gp = bf(_mk(n, 3, h, w, 82))
    ub = ops.ActBuffer.from_nchw(U, pad=4)
    dw = torch.empty(3, 64, 9, 9, device=DEV)
    db = torch.empty(3, device=DEV)
    ops.wgrad9x9(gp.contiguous(), ub, dw, db, head=False, scale=2.0)
    torch.cuda.synchronize()
    rw, rb = _wgrad9_ref(U, gp, 64, 3)
    _close_rel(dw, rw * 2, 1e-3)
    _close_rel(db, rb * 2, 1e-3)
    # head conv0: 3 → 64 on the LR grid
    X = bf(_mk(n, 3, h, w, 83))
    gq = bf(_mk(n, 64, h, w, 84))
    qb = ops.ActBuffer.from_nchw(gq, pad=1)
    dw = torch.empty(64, 3, 9, 9, device=DEV)
    db = torch.empty(64, device=DEV)
    ops.wgrad9x9(X.contiguous(), qb, dw, db, head=True)
    torch.cuda.synchronize()
    rw, rb = _wgrad9_ref(X, gq, 3, 64)
    _close_rel(dw, rw, 1e-3)
    _close_rel(db, rb, 1e-3)


def test_tail_dgrad_via_head_kernel_with_mask():
    """Input gradient of the 9x9 tail conv (64 → 3) = head kernel with rotated,
    transposed weights, masked by LeakyReLU'(last Scaler output)."""
    from image_super_resolution_amd import ops
    n, h, w = 2, 40, 72
    U = _mk(n, 64, h, w, 91).requires_grad_(True)
    W2 = _w(3, 64, 9, 92)
    gp = bf(_mk(n, 3, h, w, 93))
    F.conv2d(U, bf(W2), padding=4).backward(gp)
    act = _mk(n, 64, h, w, 94)
    mb = ops.ActBuffer.from_nchw(act, pad=1)
    Wt = W2.flip(2, 3).transpose(0, 1).contiguous()  # [64][3][9][9]
    out = ops.ActBuffer.alloc(n, h, w, 64, 2, DEV)
    ops.head9x9(gp.contiguous(), ops.pack_head9x9(Wt), None, out, slope=1.0, m=mb, mslope=0.01)
    torch.cuda.synchronize()
    ref = U.grad * torch.where(bf(act) > 0, 1.0, 0.01)
    close(out.to_nchw(), ref)


@pytest.mark.parametrize("n,c,h,w,slope", [(2, 32, 20, 36, 0.01), (4, 64, 16, 32, 1.0), (1, 32, 7, 45, 0.01)])
def test_batchnorm_train_forward_backward(n, c, h, w, slope):
    """Train-mode BatchNorm2d kernels vs F.batch_norm(training=True) + autograd."""
    from image_super_resolution_amd import ops
    z = bf(_mk(n, c, h, w, 101) * 0.7 + 0.3)
    bn = torch.nn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(c, device=DEV) + 0.5)
        bn.bias.copy_(torch.randn(c, device=DEV) * 0.1)
        bn.running_mean.copy_(torch.randn(c, device=DEV) * 0.1)
        bn.running_var.copy_(torch.rand(c, device=DEV) + 0.5)
    rm, rv = bn.running_mean.clone(), bn.running_var.clone()
    r = bf(_mk(n, c, h, w, 102))
    zb = ops.ActBuffer.from_nchw(z, pad=1)
    rb = ops.ActBuffer.from_nchw(r, pad=1)
    yb = ops.ActBuffer.alloc(n, h, w, c, 1, DEV)
    st = ops.BNState(c, DEV)
    ops.bn_forward(ops.bn_desc(zb, yb, c, st, bn, slope=slope, r1=rb, s1=0.2, s2=0.5), st)
    torch.cuda.synchronize()
    zr = z.clone().requires_grad_(True)
    w_ = bn.weight.detach().clone().requires_grad_(True)
    b_ = bn.bias.detach().clone().requires_grad_(True)
    pre = F.batch_norm(zr, rm, rv, w_, b_, training=True, momentum=0.1, eps=1e-5)
    ref = (lrelu(pre, slope) * 0.2 + r) * 0.5
    close(yb.to_nchw(), ref)
    assert yb.outside_valid().float().abs().max().item() == 0.0
    torch.testing.assert_close(bn.running_mean, rm, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn.running_var, rv, rtol=1e-4, atol=1e-5)
    # backward of the BN output (pre-activation gradient g), scaled
    g = bf(_mk(n, c, h, w, 103))
    pre.backward(g * 0.25)
    gb = ops.ActBuffer.from_nchw(g, pad=1)
    dzb = ops.ActBuffer.alloc(n, h, w, c, 1, DEV)
    dgam = torch.empty(c, device=DEV)
    dbet = torch.empty(c, device=DEV)
    ops.bn_backward(ops.bn_desc(zb, gb, c, st, bn, dz=dzb, dgamma=dgam, dbeta=dbet, gscale=0.25), st)
    torch.cuda.synchronize()
    close(dzb.to_nchw(), zr.grad)
    torch.testing.assert_close(dgam, w_.grad, rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(dbet, b_.grad, rtol=2e-3, atol=2e-3)
    assert torch.equal(gb.to_nchw(), g)  # dz went to its own buffer
