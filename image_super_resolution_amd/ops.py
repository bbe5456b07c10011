"""Thin host wrappers over the libisr C-ABI.

PyTorch is plumbing here: it allocates device memory and supplies the current
HIP stream; every byte of compute happens in libisr.so.  All functions require
CUDA (HIP) tensors and raise otherwise.
"""
from __future__ import annotations

import os as _os

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import IsrConvDesc, IsrConvertDesc, IsrEwDesc, IsrHeadDesc, IsrPoolDesc, IsrTailDesc, IsrView, IsrWgrad9Desc, IsrWgradDesc, TILE_H, TILE_W, check


# Bumped whenever a libisr kernel writes parameters in place (FusedAdam.step,
# ema_update_).  Raw-pointer writes do not bump torch's tensor `_version`, so the
# packed-weight caches (models._Generator._packed, Denoise._packed) key on this too.
_PARAM_EPOCH = [0]


def param_write_epoch() -> int:
    return _PARAM_EPOCH[0]


def bump_param_epoch() -> None:
    _PARAM_EPOCH[0] += 1


def round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


def _stream() -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _require_gpu(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(f"{what}: image_super_resolution_amd runs on the MI355X HIP path only "
                           f"(got a {t.device} tensor); the CPU restatement lives in oracle/ for tests")


@dataclass
class ActBuffer:
    """Channel-blocked activation buffer [n][c/16][ha+2p][wa+2p][16], zero border p.

    Storage is bf16 (training: the per-conv forward and backward) or fp16 (the inference
    forward, isr_conv_desc.f16 — 3 more mantissa bits at the same MFMA rate and footprint;
    the generator's activations stay far inside fp16 range).

    Each 16-channel block is a contiguous plane, so a conv K-chunk reads whole
    cache lines.  (h, w) is the valid image size, (ha, wa) the tile-aligned
    computed extent.  Kernels keep every position outside (h, w) at exactly
    zero, so the border and alignment slack act as the conv's zero padding.
    """
    t: torch.Tensor
    n: int
    h: int
    w: int
    ha: int
    wa: int
    pad: int

    @staticmethod
    def alloc(n: int, h: int, w: int, c: int, pad: int, device, ha: int | None = None,
              wa: int | None = None, min_hp: int = 0, min_wp: int = 0,
              dtype: torch.dtype = torch.bfloat16) -> "ActBuffer":
        """min_hp / min_wp: extra zero rows / columns below / right of the computed
        region (a stride-2 consumer reads 2*ha_out + 2*pad rows of its input)."""
        if dtype not in (torch.bfloat16, torch.float16):
            raise TypeError(f"ActBuffer storage must be bfloat16 or float16, got {dtype}")
        if c % 16:
            raise ValueError(f"ActBuffer channels must be a multiple of 16, got {c}")
        ha = round_up(h, TILE_H) if ha is None else ha
        wa = round_up(w, TILE_W) if wa is None else wa
        hp, wp = max(ha + 2 * pad, min_hp), max(wa + 2 * pad, min_wp)
        t = torch.zeros((n, c // 16, hp, wp, 16), dtype=dtype, device=device)
        return ActBuffer(t, n, h, w, ha, wa, pad)

    @property
    def c(self) -> int:
        return self.t.shape[1] * 16

    @property
    def f16(self) -> int:
        """1 for fp16 storage (the descriptors' f16 field), 0 for bf16."""
        return int(self.t.dtype == torch.float16)

    def view(self, coff: int = 0) -> IsrView:
        return IsrView(self.t.data_ptr(), self.t.shape[2], self.t.shape[3], self.c, self.pad, coff)

    def interior(self, c0: int = 0, c1: int | None = None) -> torch.Tensor:
        """Valid region as an [n, c, h, w] strided view (for tests / debugging)."""
        p = self.pad
        v = self.t[:, :, p:p + self.h, p:p + self.w, :]  # n, c16, h, w, 16
        v = v.permute(0, 1, 4, 2, 3).reshape(self.n, self.c, self.h, self.w)
        return v[:, c0:c1]

    def set_nchw(self, x: torch.Tensor, c0: int = 0) -> None:
        """Write NCHW x into channels [c0, c0 + x.shape[1]) of the valid region."""
        n, c, h, w = x.shape
        if c % 16 or c0 % 16 or (h, w) != (self.h, self.w):
            raise ValueError("set_nchw: channel block / shape mismatch")
        p = self.pad
        self.t[:, c0 // 16:(c0 + c) // 16, p:p + h, p:p + w, :] = (
            x.reshape(n, c // 16, 16, h, w).permute(0, 1, 3, 4, 2).to(self.t.dtype))

    def outside_valid(self) -> torch.Tensor:
        """Every element outside the valid h x w region (border + alignment slack)."""
        mask = torch.ones(self.t.shape, dtype=torch.bool, device=self.t.device)
        p = self.pad
        mask[:, :, p:p + self.h, p:p + self.w, :] = False
        return self.t[mask]

    @staticmethod
    def from_nchw(x: torch.Tensor, pad: int = 1, c_alloc: int | None = None,
                  dtype: torch.dtype = torch.bfloat16) -> "ActBuffer":
        n, c, h, w = x.shape
        buf = ActBuffer.alloc(n, h, w, c_alloc or c, pad, x.device, dtype=dtype)
        buf.set_nchw(x, 0)
        return buf

    def to_nchw(self, c0: int = 0, c1: int | None = None) -> torch.Tensor:
        return self.interior(c0, c1).float().contiguous()


_NULL_VIEW = IsrView(None, 0, 0, 0, 0, 0)


# ---------------------------------------------------------------- packing
def _wdtype(f16: bool) -> torch.dtype:
    return torch.float16 if f16 else torch.bfloat16


def pack_conv3x3(w: torch.Tensor, out: torch.Tensor | None = None, f16: bool = False) -> torch.Tensor:
    """fp32 OIHW [cout, cin, 3, 3] device weights → packed bf16 (fp16 with `f16`: the
    inference forward, isr_pack_conv3x3_f16) kernel layout."""
    _require_gpu(w, "pack_conv3x3")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    n = lib.isr_conv3x3_packed_bytes(cout, cin) // 2
    dt = _wdtype(f16)
    if out is None:
        out = torch.empty(n, dtype=dt, device=w.device)
    elif out.numel() != n or out.dtype != dt:
        raise ValueError("pack_conv3x3: bad output buffer")
    fn = lib.isr_pack_conv3x3_f16 if f16 else lib.isr_pack_conv3x3
    check(fn(w.data_ptr(), out.data_ptr(), cout, cin, _stream()), "isr_pack_conv3x3")
    return out


def pack_conv3x3_dgrad(w: torch.Tensor, scale: float = 1.0, sub2: bool = False,
                       out: torch.Tensor | None = None) -> torch.Tensor:
    """Layer weights [cout, cin, 3, 3] → packed weights of the input-gradient conv
    cout → cin (180°-rotated, times `scale`; `sub2` = PixelShuffle channel order)."""
    _require_gpu(w, "pack_conv3x3_dgrad")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    n = lib.isr_conv3x3_packed_bytes(cin, cout) // 2
    if out is None:
        out = torch.empty(n, dtype=torch.bfloat16, device=w.device)
    elif out.numel() != n or out.dtype != torch.bfloat16:
        raise ValueError("pack_conv3x3_dgrad: bad output buffer")
    check(lib.isr_pack_conv3x3_dgrad(w.data_ptr(), out.data_ptr(), cout, cin, scale, int(sub2), _stream()),
          "isr_pack_conv3x3_dgrad")
    return out


def pack_batch_table(items, device) -> tuple[torch.Tensor, int]:
    """Device table of isr_pack_item for isr_pack_conv3x3_batch.  items: tuples
    (w fp32 [cout,cin,3,3], out packed bf16, cout, cin, dgrad, sub2, scale) or, for a
    dgrad window (isr.h isr_pack_item), (w [cout,src_cin,3,3], out, cout, cin, 1, 0, scale,
    src_n0, src_cin, out_elem_offset) with out_elem_offset the block's bf16 element offset
    inside `out`; the tensors must stay alive and in place (parameters, packed buffers)."""
    import struct
    raw = bytearray()
    lib = _lib.load()
    for it in items:
        w, out, cout, cin, dgrad, sub2, scale = it[:7]
        n0, scin, eoff = (it[7], it[8], it[9]) if len(it) > 7 else (0, 0, 0)
        _require_gpu(w, "pack_conv3x3_batch")
        wshape = (cout, scin if scin else cin, 3, 3)
        if w.dtype != torch.float32 or not w.is_contiguous() or tuple(w.shape) != wshape:
            raise ValueError(f"pack_conv3x3_batch: weights must be contiguous fp32 {list(wshape)}")
        if cin % 16 or cout % 32 or (dgrad and (cin % 32 or cout % 16)):
            raise ValueError(f"pack_conv3x3_batch: unsupported shape cout={cout} cin={cin}")
        if scin and (not dgrad or sub2 or n0 < 0 or n0 + cin > scin):
            raise ValueError("pack_conv3x3_batch: bad dgrad window")
        if out.dtype != torch.bfloat16 or out.numel() < eoff + lib.isr_conv3x3_packed_bytes(cout, cin) // 2:
            raise ValueError("pack_conv3x3_batch: bad output buffer")
        raw += struct.pack("<QQiiiifiii", w.data_ptr(), out.data_ptr() + 2 * eoff, cout, cin, int(dgrad), int(sub2),
                           float(scale), int(n0), int(scin), 0)
    table = torch.frombuffer(raw, dtype=torch.uint8).to(device)
    return table, len(items)


def pack_batch(table: tuple[torch.Tensor, int]) -> None:
    t, n = table
    check(_lib.load().isr_pack_conv3x3_batch(t.data_ptr(), n, _stream()), "isr_pack_conv3x3_batch")


def pack_head9x9(w: torch.Tensor, out: torch.Tensor | None = None, f16: bool = False) -> torch.Tensor:
    _require_gpu(w, "pack_head9x9")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    n = lib.isr_head9x9_packed_bytes(cout, cin) // 2
    dt = _wdtype(f16)
    if out is None:
        out = torch.empty(n, dtype=dt, device=w.device)
    elif out.numel() != n or out.dtype != dt:
        raise ValueError("pack_head9x9: bad output buffer")
    fn = lib.isr_pack_head9x9_f16 if f16 else lib.isr_pack_head9x9
    check(fn(w.data_ptr(), out.data_ptr(), cout, cin, _stream()), "isr_pack_head9x9")
    return out


def pack_tail9x9(w: torch.Tensor, out: torch.Tensor | None = None, f16: bool = False) -> torch.Tensor:
    _require_gpu(w, "pack_tail9x9")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    n = lib.isr_tail9x9_packed_bytes(cout, cin) // 2
    dt = _wdtype(f16)
    if out is None:
        out = torch.empty(n, dtype=dt, device=w.device)
    elif out.numel() != n or out.dtype != dt:
        raise ValueError("pack_tail9x9: bad output buffer")
    fn = lib.isr_pack_tail9x9_f16 if f16 else lib.isr_pack_tail9x9
    check(fn(w.data_ptr(), out.data_ptr(), cout, cin, _stream()), "isr_pack_tail9x9")
    return out


# ---------------------------------------------------------------- launches
def conv3x3_desc(x: ActBuffer, cin: int, wpack: torch.Tensor, bias: torch.Tensor | None, cout: int,
                 y: ActBuffer, *, x_coff: int = 0, y_coff: int = 0, slope: float = 1.0,
                 r1: ActBuffer | None = None, r1_coff: int = 0, s1: float = 1.0,
                 r2: ActBuffer | None = None, r2_coff: int = 0, s2: float = 1.0,
                 y2: ActBuffer | None = None, y2_coff: int = 0, shuffle: int = 1,
                 m: ActBuffer | None = None, m_coff: int | None = None, mslope: float = 1.0, m_c0: int = 0,
                 r1_cn: int = 0, x_sub2: bool = False, taps: int = 0) -> IsrConvDesc:
    """Descriptor for y[..., y_coff:y_coff+cout] = epilogue(conv3x3(x[..., x_coff:x_coff+cin])).

    Backward extensions: `m` (read at channel m_coff, default y_coff) masks output
    channels >= m_c0 with LeakyReLU'(m) of slope `mslope`; `r1_cn` limits r1 to the
    first r1_cn output channels; `x_sub2` reads x (2h x 2w grid) as PixelShuffle(2)ᵀ;
    `taps` 1 / 2 restricts the conv to kernel taps {0,1}² / {1,2}² (stride-2 convs, see isr.h)."""
    d = IsrConvDesc()
    d.n, d.h, d.w, d.ha, d.wa = x.n, x.h, x.w, x.ha, x.wa
    d.cin, d.cout = cin, cout
    d.x = x.view(x_coff)
    d.y = y.view(y_coff)
    d.y2 = y2.view(y2_coff) if y2 is not None else _NULL_VIEW
    d.r1 = r1.view(r1_coff) if r1 is not None else _NULL_VIEW
    d.r2 = r2.view(r2_coff) if r2 is not None else _NULL_VIEW
    d.wpack = wpack.data_ptr()
    d.bias = bias.data_ptr() if bias is not None else None
    d.slope, d.s1, d.s2, d.shuffle = slope, s1, s2, shuffle
    if x_sub2:
        d.n, d.h, d.w, d.ha, d.wa = y.n, y.h, y.w, y.ha, y.wa
    d.m = m.view(y_coff if m_coff is None else m_coff) if m is not None else _NULL_VIEW
    d.mslope, d.m_c0, d.r1_cn, d.x_sub2 = mslope, m_c0, r1_cn, int(bool(x_sub2))
    d.taps = taps
    d.f16 = _same_storage("conv3x3", wpack, x, y, y2, r1, r2, m)
    return d


def _same_storage(what: str, wpack: torch.Tensor, *bufs) -> int:
    """The descriptor's f16 flag: every activation buffer and the packed weights of one launch
    share one storage type (bf16 or fp16)."""
    dts = {b.t.dtype for b in bufs if b is not None}
    if len(dts) != 1 or wpack.dtype not in dts:
        raise TypeError(f"{what}: mixed storage types {sorted(map(str, dts | {wpack.dtype}))}")
    return int(wpack.dtype == torch.float16)


def launch_conv3x3(d: IsrConvDesc) -> None:
    check(_lib.load().isr_conv3x3_fwd(ctypes.byref(d), _stream()), "isr_conv3x3_fwd")


def conv3x3(x: ActBuffer, cin: int, wpack: torch.Tensor, bias: torch.Tensor | None, cout: int,
            y: ActBuffer, **kw) -> None:
    """y[..., y_coff:y_coff+cout] = epilogue(conv3x3(x[..., x_coff:x_coff+cin]))."""
    launch_conv3x3(conv3x3_desc(x, cin, wpack, bias, cout, y, **kw))


def head9x9_desc(x: torch.Tensor, wpack: torch.Tensor, bias: torch.Tensor | None, y: ActBuffer, *,
                 slope: float, y2: ActBuffer | None = None, y2_coff: int = 0,
                 mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                 m: ActBuffer | None = None, mslope: float = 1.0) -> IsrHeadDesc:
    _require_gpu(x, "head9x9")
    if not x.is_contiguous():
        raise ValueError("head9x9: input must be contiguous NCHW")
    d = IsrHeadDesc()
    d.n, d.h, d.w, d.ha, d.wa = y.n, y.h, y.w, y.ha, y.wa
    d.cout = 64
    d.x = x.data_ptr()
    if x.dtype == torch.uint8:
        d.x_u8 = 1
    elif x.dtype == torch.float32:
        d.x_u8 = 0
    else:
        raise TypeError(f"head9x9: input must be float32 or uint8, got {x.dtype}")
    for i in range(3):
        d.mean[i] = float(mean[i])
        d.inv_std[i] = 1.0 / float(std[i])
    d.y = y.view(0)
    d.y2 = y2.view(y2_coff) if y2 is not None else _NULL_VIEW
    d.wpack = wpack.data_ptr()
    d.bias = bias.data_ptr() if bias is not None else None
    d.slope = slope
    d.m = m.view(0) if m is not None else _NULL_VIEW
    d.mslope = mslope
    d.f16 = _same_storage("head9x9", wpack, y, y2, m)
    return d


def launch_head9x9(d: IsrHeadDesc) -> None:
    check(_lib.load().isr_head9x9_fwd(ctypes.byref(d), _stream()), "isr_head9x9_fwd")


def head9x9(x: torch.Tensor, wpack: torch.Tensor, bias: torch.Tensor | None, y: ActBuffer, **kw) -> None:
    """9x9 head conv on an NCHW fp32 (normalised) or uint8 (raw) image."""
    launch_head9x9(head9x9_desc(x.contiguous(), wpack, bias, y, **kw))


def tail9x9_desc(x: ActBuffer, wpack: torch.Tensor, bias: torch.Tensor | None, out: torch.Tensor) -> IsrTailDesc:
    _require_gpu(out, "tail9x9")
    if out.dtype not in (torch.float32, torch.uint8) or not out.is_contiguous():
        raise TypeError("tail9x9: out must be a contiguous float32 or uint8 tensor")
    if tuple(out.shape) != (x.n, 3, x.h, x.w):
        raise ValueError(f"tail9x9: out shape {tuple(out.shape)} != {(x.n, 3, x.h, x.w)}")
    d = IsrTailDesc()
    d.n, d.h, d.w, d.ha, d.wa = x.n, x.h, x.w, x.ha, x.wa
    d.cin = 64
    d.x = x.view(0)
    d.wpack = wpack.data_ptr()
    d.bias = bias.data_ptr() if bias is not None else None
    d.y = out.data_ptr()
    d.y_u8 = 1 if out.dtype == torch.uint8 else 0
    d.f16 = _same_storage("tail9x9", wpack, x)
    return d


def launch_tail9x9(d: IsrTailDesc) -> None:
    check(_lib.load().isr_tail9x9_fwd(ctypes.byref(d), _stream()), "isr_tail9x9_fwd")


def tail9x9(x: ActBuffer, wpack: torch.Tensor, bias: torch.Tensor | None, out: torch.Tensor) -> None:
    """out (NCHW [n,3,h,w], fp32 or uint8) = tanh(conv9x9(x) + bias) (→ uint8 image)."""
    launch_tail9x9(tail9x9_desc(x, wpack, bias, out))


# ---------------------------------------------------------------- backward
class Workspace:
    """Grow-only device scratch for split-K partial sums (the library never allocates)."""

    def __init__(self):
        self.t = None

    def get(self, nbytes: int, device) -> torch.Tensor:
        if self.t is None or self.t.numel() < nbytes or self.t.device != torch.device(device):
            self.t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
        return self.t


_WS = Workspace()


def wgrad3x3_desc(x: ActBuffer, cin: int, g: ActBuffer, cout: int, dw: torch.Tensor, db: torch.Tensor | None = None,
                  *, x_coff: int = 0, g_coff: int = 0, scale: float = 1.0, g_sub2: bool = False,
                  splits: int = 0, x_sub2: bool = False, taps: int = 0) -> IsrWgradDesc:
    """dw[cout, cin, 3, 3] = scale * sum g ⊗ shifted x (fp32, overwritten); db[cout] likewise.
    `x_sub2`: x (2h x 2w grid) is read as PixelShuffle(2)ᵀ (cin = 4 x its channels);
    `taps=1`: only taps {0,1}² are computed (stride-2 phase convs)."""
    if dw.dtype != torch.float32 or not dw.is_contiguous() or tuple(dw.shape) != (cout, cin, 3, 3):
        raise ValueError("wgrad3x3: dw must be contiguous fp32 [cout, cin, 3, 3]")
    if db is not None and (db.dtype != torch.float32 or not db.is_contiguous() or db.numel() != cout):
        raise ValueError("wgrad3x3: db must be contiguous fp32 [cout]")
    d = IsrWgradDesc()
    grid = g if x_sub2 else x
    d.n, d.h, d.w, d.ha, d.wa = grid.n, grid.h, grid.w, grid.ha, grid.wa
    d.cin, d.cout = cin, cout
    d.x_sub2, d.taps = int(bool(x_sub2)), taps
    d.x = x.view(x_coff)
    d.g = g.view(g_coff)
    d.g_sub2 = int(bool(g_sub2))
    d.scale = scale
    d.dw = dw.data_ptr()
    d.db = db.data_ptr() if db is not None else None
    d.splits = splits
    return d


_WGRAD_VARIANT = int(_os.environ.get("ISR_WGRAD_VARIANT", "0"))  # A/B only (isr_wgrad3x3_variant)


def launch_wgrad3x3(d: IsrWgradDesc, device) -> None:
    lib = _lib.load()
    if _WGRAD_VARIANT:
        nbytes = lib.isr_wgrad3x3_variant_workspace_bytes(ctypes.byref(d), _WGRAD_VARIANT)
        ws = _WS.get(max(nbytes, 16), device)
        check(lib.isr_wgrad3x3_variant(ctypes.byref(d), _WGRAD_VARIANT, ws.data_ptr(), ws.numel(), _stream()),
              "isr_wgrad3x3_variant")
        return
    nbytes = lib.isr_wgrad3x3_workspace_bytes(ctypes.byref(d))
    if nbytes == 0:
        check(lib.isr_wgrad3x3(ctypes.byref(d), None, 0, _stream()), "isr_wgrad3x3")
        return
    ws = _WS.get(nbytes, device)
    check(lib.isr_wgrad3x3(ctypes.byref(d), ws.data_ptr(), ws.numel(), _stream()), "isr_wgrad3x3")


def wgrad3x3(x: ActBuffer, cin: int, g: ActBuffer, cout: int, dw: torch.Tensor, db: torch.Tensor | None = None,
             **kw) -> None:
    launch_wgrad3x3(wgrad3x3_desc(x, cin, g, cout, dw, db, **kw), x.t.device)


def wgrad9x9_desc(p: torch.Tensor, q: ActBuffer, dw: torch.Tensor, db: torch.Tensor | None = None, *, head: bool,
                  scale: float = 1.0, splits: int = 0) -> IsrWgrad9Desc:
    """9x9 conv weight gradient (see include/isr.h isr_wgrad9_desc)."""
    _require_gpu(p, "wgrad9x9")
    if p.dtype != torch.float32 or not p.is_contiguous() or p.dim() != 4 or p.shape[1] != 3:
        raise ValueError("wgrad9x9: p must be contiguous fp32 [n, 3, h, w]")
    shape = (64, 3, 9, 9) if head else (3, 64, 9, 9)
    if dw.dtype != torch.float32 or not dw.is_contiguous() or tuple(dw.shape) != shape:
        raise ValueError(f"wgrad9x9: dw must be contiguous fp32 {shape}")
    if db is not None and (db.dtype != torch.float32 or not db.is_contiguous() or db.numel() != shape[0]):
        raise ValueError("wgrad9x9: bad db")
    if tuple(p.shape[2:]) != (q.h, q.w) or p.shape[0] != q.n:
        raise ValueError("wgrad9x9: p / q grids differ")
    d = IsrWgrad9Desc()
    d.n, d.h, d.w, d.ha, d.wa = q.n, q.h, q.w, q.ha, q.wa
    d.head = int(bool(head))
    d.p = p.data_ptr()
    d.q = q.view(0)
    d.scale = scale
    d.dw = dw.data_ptr()
    d.db = db.data_ptr() if db is not None else None
    d.splits = splits
    return d


def launch_wgrad9x9(d: IsrWgrad9Desc, device) -> None:
    lib = _lib.load()
    nbytes = lib.isr_wgrad9x9_workspace_bytes(ctypes.byref(d))
    if nbytes == 0:
        check(lib.isr_wgrad9x9(ctypes.byref(d), None, 0, _stream()), "isr_wgrad9x9")
        return
    ws = _WS.get(nbytes, device)
    check(lib.isr_wgrad9x9(ctypes.byref(d), ws.data_ptr(), ws.numel(), _stream()), "isr_wgrad9x9")


def wgrad9x9(p: torch.Tensor, q: ActBuffer, dw: torch.Tensor, db: torch.Tensor | None = None, **kw) -> None:
    launch_wgrad9x9(wgrad9x9_desc(p, q, dw, db, **kw), p.device)


def ew_combine_desc(y: ActBuffer, a: ActBuffer, c: int, *, sa: float = 1.0, b: ActBuffer | None = None,
                    sb: float = 1.0, m: ActBuffer | None = None, mslope: float = 1.0,
                    y_coff: int = 0, a_coff: int = 0, b_coff: int = 0, m_coff: int = 0) -> IsrEwDesc:
    """y = (a*sa + b*sb) * LeakyReLU'(m) over c channels (zero outside the valid region)."""
    d = IsrEwDesc()
    d.n, d.h, d.w, d.ha, d.wa, d.c = y.n, y.h, y.w, y.ha, y.wa, c
    d.y, d.a = y.view(y_coff), a.view(a_coff)
    d.b = b.view(b_coff) if b is not None else _NULL_VIEW
    d.m = m.view(m_coff) if m is not None else _NULL_VIEW
    d.sa, d.sb, d.mslope = sa, sb, mslope
    return d


def ew_combine(y: ActBuffer, a: ActBuffer, c: int, **kw) -> None:
    check(_lib.load().isr_ew_combine(ctypes.byref(ew_combine_desc(y, a, c, **kw)), _stream()), "isr_ew_combine")


def pixel_shuffle2_desc(y: ActBuffer, a: ActBuffer, c: int, *, slope: float = 1.0, sa: float = 1.0) -> IsrEwDesc:
    """y[0:c] (grid 2h x 2w) = LeakyReLU_slope(sa * PixelShuffle(2)(a[0:4c]))."""
    d = IsrEwDesc()
    d.n, d.h, d.w, d.ha, d.wa, d.c = y.n, y.h, y.w, y.ha, y.wa, c
    d.y, d.a, d.b, d.m = y.view(0), a.view(0), _NULL_VIEW, _NULL_VIEW
    d.sa, d.sb, d.mslope = sa, 0.0, slope
    return d


def pixel_unshuffle2_desc(y: ActBuffer, a: ActBuffer, c: int, *, m: ActBuffer | None = None, mslope: float = 1.0,
                          sa: float = 1.0) -> IsrEwDesc:
    """y[0:c] (grid h x w) = PixelShuffle(2)ᵀ(sa * a[0:c/4] * LeakyReLU'(m)) — a, m on the 2h x 2w grid."""
    d = IsrEwDesc()
    d.n, d.h, d.w, d.ha, d.wa, d.c = y.n, y.h, y.w, y.ha, y.wa, c
    d.y, d.a, d.b = y.view(0), a.view(0), _NULL_VIEW
    d.m = m.view(0) if m is not None else _NULL_VIEW
    d.sa, d.sb, d.mslope = sa, 0.0, mslope
    return d


def pixel_unshuffle2(y: ActBuffer, a: ActBuffer, c: int, **kw) -> None:
    check(_lib.load().isr_pixel_unshuffle2(ctypes.byref(pixel_unshuffle2_desc(y, a, c, **kw)), _stream()),
          "isr_pixel_unshuffle2")


def pixel_shuffle2(y: ActBuffer, a: ActBuffer, c: int, **kw) -> None:
    check(_lib.load().isr_pixel_shuffle2(ctypes.byref(pixel_shuffle2_desc(y, a, c, **kw)), _stream()),
          "isr_pixel_shuffle2")


def convert_desc(nchw: torch.Tensor, v: ActBuffer, *, v_coff: int = 0, scale: torch.Tensor | None = None,
                 shift: torch.Tensor | None = None, m: ActBuffer | None = None, mslope: float = 1.0,
                 m_coff: int = 0) -> IsrConvertDesc:
    _require_gpu(nchw, "convert")
    if nchw.dtype != torch.float32 or not nchw.is_contiguous() or nchw.dim() != 4:
        raise ValueError("convert: nchw must be contiguous fp32 [n, c, h, w]")
    n, c, h, w = nchw.shape
    if (n, h, w) != (v.n, v.h, v.w):
        raise ValueError(f"convert: grid mismatch {tuple(nchw.shape)} vs buffer {(v.n, v.h, v.w)}")
    d = IsrConvertDesc()
    d.n, d.h, d.w, d.ha, d.wa, d.c = n, h, w, v.ha, v.wa, c
    d.nchw = nchw.data_ptr()
    d.v = v.view(v_coff)
    d.scale = scale.data_ptr() if scale is not None else None
    d.shift = shift.data_ptr() if shift is not None else None
    d.m = m.view(m_coff) if m is not None else _NULL_VIEW
    d.mslope = mslope
    return d


def nchw_to_blocked(nchw: torch.Tensor, v: ActBuffer, **kw) -> None:
    check(_lib.load().isr_nchw_to_blocked(ctypes.byref(convert_desc(nchw, v, **kw)), _stream()), "isr_nchw_to_blocked")


def blocked_to_nchw(v: ActBuffer, out: torch.Tensor, **kw) -> torch.Tensor:
    check(_lib.load().isr_blocked_to_nchw(ctypes.byref(convert_desc(out, v, **kw)), _stream()), "isr_blocked_to_nchw")
    return out


def pool_desc(x: ActBuffer, y: ActBuffer, c: int, g: ActBuffer | None = None, mslope: float = 0.0) -> IsrPoolDesc:
    if (y.h, y.w) != (x.h // 2, x.w // 2) or y.ha * 2 > x.ha or y.wa * 2 > x.wa:
        raise ValueError("maxpool2: output grid must be (h/2, w/2) with 2*ha_out within the input buffer")
    d = IsrPoolDesc()
    d.n, d.h, d.w, d.c, d.hao, d.wao = x.n, x.h, x.w, c, y.ha, y.wa
    d.x, d.y = x.view(0), y.view(0)
    d.g = g.view(0) if g is not None else _NULL_VIEW
    d.mslope = mslope
    return d


def maxpool2_fwd(x: ActBuffer, y: ActBuffer, c: int) -> None:
    check(_lib.load().isr_maxpool2_fwd(ctypes.byref(pool_desc(x, y, c)), _stream()), "isr_maxpool2_fwd")


def maxpool2_bwd(x: ActBuffer, gy: ActBuffer, gx: ActBuffer, c: int, mslope: float = 0.0) -> None:
    check(_lib.load().isr_maxpool2_bwd(ctypes.byref(pool_desc(x, gy, c, gx, mslope)), _stream()), "isr_maxpool2_bwd")


# ---------------------------------------------------------------- BatchNorm (train mode)
class BNState:
    """Per-layer scratch of the train-mode BatchNorm kernels: double accumulators
    acc[2][c] and the saved (mean, invstd)[2][c]."""

    def __init__(self, c: int, device):
        self.c = c
        self.acc = torch.zeros(2 * c, dtype=torch.float64, device=device)
        self.save = torch.zeros(2 * c, dtype=torch.float32, device=device)


def bn_desc(z: ActBuffer, y: ActBuffer, c: int, st: BNState, bn: "torch.nn.BatchNorm2d", *, z_coff: int = 0,
            y_coff: int = 0, slope: float = 1.0, r1: ActBuffer | None = None, r1_coff: int = 0, s1: float = 1.0,
            r2: ActBuffer | None = None, r2_coff: int = 0, s2: float = 1.0, dz: ActBuffer | None = None,
            dz_coff: int = 0, dgamma: torch.Tensor | None = None, dbeta: torch.Tensor | None = None,
            gscale: float = 1.0, update_running: bool = True) -> _lib.IsrBnDesc:
    d = _lib.IsrBnDesc()
    d.n, d.h, d.w, d.ha, d.wa, d.c = z.n, z.h, z.w, z.ha, z.wa, c
    d.z, d.y = z.view(z_coff), y.view(y_coff)
    d.r1 = r1.view(r1_coff) if r1 is not None else _NULL_VIEW
    d.r2 = r2.view(r2_coff) if r2 is not None else _NULL_VIEW
    d.dz = dz.view(dz_coff) if dz is not None else _NULL_VIEW
    d.s1, d.s2, d.slope = s1, s2, slope
    d.gamma, d.beta = bn.weight.data_ptr(), bn.bias.data_ptr()
    if update_running and bn.running_mean is not None:
        d.running_mean, d.running_var = bn.running_mean.data_ptr(), bn.running_var.data_ptr()
    d.momentum = float(bn.momentum if bn.momentum is not None else 0.1)
    d.eps = float(bn.eps)
    d.acc, d.save = st.acc.data_ptr(), st.save.data_ptr()
    d.dgamma = dgamma.data_ptr() if dgamma is not None else None
    d.dbeta = dbeta.data_ptr() if dbeta is not None else None
    d.gscale = gscale
    return d


def bn_forward(d: _lib.IsrBnDesc, st: BNState) -> None:
    lib, s = _lib.load(), _stream()
    st.acc.zero_()
    check(lib.isr_bn_stats(ctypes.byref(d), s), "isr_bn_stats")
    check(lib.isr_bn_finalize(ctypes.byref(d), s), "isr_bn_finalize")
    check(lib.isr_bn_apply(ctypes.byref(d), s), "isr_bn_apply")


def bn_backward(d: _lib.IsrBnDesc, st: BNState) -> None:
    lib, s = _lib.load(), _stream()
    st.acc.zero_()
    check(lib.isr_bn_bwd_reduce(ctypes.byref(d), s), "isr_bn_bwd_reduce")
    check(lib.isr_bn_bwd_apply(ctypes.byref(d), s), "isr_bn_bwd_apply")
