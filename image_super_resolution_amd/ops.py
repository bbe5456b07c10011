"""Thin host wrappers over the libisr C-ABI.

PyTorch is plumbing here: it allocates device memory and supplies the current
HIP stream; every byte of compute happens in libisr.so.  All functions require
CUDA (HIP) tensors and raise otherwise.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import IsrConvDesc, IsrHeadDesc, IsrTailDesc, IsrView, TILE_H, TILE_W, check


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
    """Channel-blocked bf16 activation buffer [n][c/16][ha+2p][wa+2p][16], zero border p.

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
              wa: int | None = None) -> "ActBuffer":
        if c % 16:
            raise ValueError(f"ActBuffer channels must be a multiple of 16, got {c}")
        ha = round_up(h, TILE_H) if ha is None else ha
        wa = round_up(w, TILE_W) if wa is None else wa
        t = torch.zeros((n, c // 16, ha + 2 * pad, wa + 2 * pad, 16), dtype=torch.bfloat16, device=device)
        return ActBuffer(t, n, h, w, ha, wa, pad)

    @property
    def c(self) -> int:
        return self.t.shape[1] * 16

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
            x.reshape(n, c // 16, 16, h, w).permute(0, 1, 3, 4, 2).to(torch.bfloat16))

    def outside_valid(self) -> torch.Tensor:
        """Every element outside the valid h x w region (border + alignment slack)."""
        mask = torch.ones(self.t.shape, dtype=torch.bool, device=self.t.device)
        p = self.pad
        mask[:, :, p:p + self.h, p:p + self.w, :] = False
        return self.t[mask]

    @staticmethod
    def from_nchw(x: torch.Tensor, pad: int = 1, c_alloc: int | None = None) -> "ActBuffer":
        n, c, h, w = x.shape
        buf = ActBuffer.alloc(n, h, w, c_alloc or c, pad, x.device)
        buf.set_nchw(x, 0)
        return buf

    def to_nchw(self, c0: int = 0, c1: int | None = None) -> torch.Tensor:
        return self.interior(c0, c1).float().contiguous()


_NULL_VIEW = IsrView(None, 0, 0, 0, 0, 0)


# ---------------------------------------------------------------- packing
def pack_conv3x3(w: torch.Tensor) -> torch.Tensor:
    """fp32 OIHW [cout, cin, 3, 3] device weights → packed bf16 kernel layout."""
    _require_gpu(w, "pack_conv3x3")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    out = torch.empty(lib.isr_conv3x3_packed_bytes(cout, cin) // 2, dtype=torch.bfloat16, device=w.device)
    check(lib.isr_pack_conv3x3(w.data_ptr(), out.data_ptr(), cout, cin, _stream()), "isr_pack_conv3x3")
    return out


def pack_head9x9(w: torch.Tensor) -> torch.Tensor:
    _require_gpu(w, "pack_head9x9")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    out = torch.empty(lib.isr_head9x9_packed_bytes(cout, cin) // 2, dtype=torch.bfloat16, device=w.device)
    check(lib.isr_pack_head9x9(w.data_ptr(), out.data_ptr(), cout, cin, _stream()), "isr_pack_head9x9")
    return out


def pack_tail9x9(w: torch.Tensor) -> torch.Tensor:
    _require_gpu(w, "pack_tail9x9")
    lib = _lib.load()
    cout, cin = w.shape[:2]
    w = w.detach().float().contiguous()
    out = torch.empty(lib.isr_tail9x9_packed_bytes(cout, cin) // 2, dtype=torch.bfloat16, device=w.device)
    check(lib.isr_pack_tail9x9(w.data_ptr(), out.data_ptr(), cout, cin, _stream()), "isr_pack_tail9x9")
    return out


# ---------------------------------------------------------------- launches
def conv3x3_desc(x: ActBuffer, cin: int, wpack: torch.Tensor, bias: torch.Tensor | None, cout: int,
                 y: ActBuffer, *, x_coff: int = 0, y_coff: int = 0, slope: float = 1.0,
                 r1: ActBuffer | None = None, r1_coff: int = 0, s1: float = 1.0,
                 r2: ActBuffer | None = None, r2_coff: int = 0, s2: float = 1.0,
                 y2: ActBuffer | None = None, y2_coff: int = 0, shuffle: int = 1,
                 m: ActBuffer | None = None, m_coff: int | None = None, mslope: float = 1.0, m_c0: int = 0,
                 r1_cn: int = 0, x_sub2: bool = False) -> IsrConvDesc:
    """Descriptor for y[..., y_coff:y_coff+cout] = epilogue(conv3x3(x[..., x_coff:x_coff+cin])).

    Backward extensions: `m` (read at channel m_coff, default y_coff) masks output
    channels >= m_c0 with LeakyReLU'(m) of slope `mslope`; `r1_cn` limits r1 to the
    first r1_cn output channels; `x_sub2` reads x (2h x 2w grid) as PixelShuffle(2)ᵀ."""
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
    return d


def launch_conv3x3(d: IsrConvDesc) -> None:
    check(_lib.load().isr_conv3x3_fwd(ctypes.byref(d), _stream()), "isr_conv3x3_fwd")


def conv3x3(x: ActBuffer, cin: int, wpack: torch.Tensor, bias: torch.Tensor | None, cout: int,
            y: ActBuffer, **kw) -> None:
    """y[..., y_coff:y_coff+cout] = epilogue(conv3x3(x[..., x_coff:x_coff+cin]))."""
    launch_conv3x3(conv3x3_desc(x, cin, wpack, bias, cout, y, **kw))


def head9x9_desc(x: torch.Tensor, wpack: torch.Tensor, bias: torch.Tensor | None, y: ActBuffer, *,
                 slope: float, y2: ActBuffer | None = None, y2_coff: int = 0,
                 mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)) -> IsrHeadDesc:
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
    return d


def launch_tail9x9(d: IsrTailDesc) -> None:
    check(_lib.load().isr_tail9x9_fwd(ctypes.byref(d), _stream()), "isr_tail9x9_fwd")


def tail9x9(x: ActBuffer, wpack: torch.Tensor, bias: torch.Tensor | None, out: torch.Tensor) -> None:
    """out (NCHW [n,3,h,w], fp32 or uint8) = tanh(conv9x9(x) + bias) (→ uint8 image)."""
    launch_tail9x9(tail9x9_desc(x, wpack, bias, out))
