"""ctypes binding of libisr.so (include/isr.h).

This module only mirrors the C structs and loads the library; it holds no
compute.  A missing or unloadable library raises immediately: there is no
fallback path.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int32, c_size_t, c_void_p
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libisr.so"

TILE_H = 32  # ISR_TILE_H
TILE_W = 32  # ISR_TILE_W


class IsrView(ctypes.Structure):
    _fields_ = [("data", c_void_p), ("hp", c_int32), ("wp", c_int32), ("cs", c_int32),
                ("pad", c_int32), ("coff", c_int32)]


class IsrConvDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32),
                ("cin", c_int32), ("cout", c_int32),
                ("x", IsrView), ("y", IsrView), ("y2", IsrView), ("r1", IsrView), ("r2", IsrView),
                ("wpack", c_void_p), ("bias", c_void_p),
                ("slope", c_float), ("s1", c_float), ("s2", c_float), ("shuffle", c_int32),
                ("m", IsrView), ("mslope", c_float), ("m_c0", c_int32), ("r1_cn", c_int32), ("x_sub2", c_int32),
                ("taps", c_int32), ("f16", c_int32)]


class IsrChainDesc(ctypes.Structure):
    _fields_ = [("layers", c_void_p), ("kinds", c_void_p), ("nl", c_int32), ("n", c_int32), ("ha", c_int32),
                ("wa", c_int32), ("state", c_void_p), ("acquire", c_int32), ("f16", c_int32)]


class IsrHeadDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32),
                ("cout", c_int32), ("x", c_void_p), ("x_u8", c_int32),
                ("mean", c_float * 3), ("inv_std", c_float * 3),
                ("y", IsrView), ("y2", IsrView), ("wpack", c_void_p), ("bias", c_void_p), ("slope", c_float),
                ("m", IsrView), ("mslope", c_float), ("f16", c_int32)]


class IsrTailDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32),
                ("cin", c_int32), ("x", IsrView), ("wpack", c_void_p), ("bias", c_void_p),
                ("y", c_void_p), ("y_u8", c_int32), ("f16", c_int32)]


class IsrWgradDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32),
                ("cin", c_int32), ("cout", c_int32), ("x", IsrView), ("g", IsrView), ("g_sub2", c_int32),
                ("scale", c_float), ("dw", c_void_p), ("db", c_void_p), ("splits", c_int32),
                ("x_sub2", c_int32), ("taps", c_int32)]


class IsrWgrad9Desc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32),
                ("head", c_int32), ("p", c_void_p), ("q", IsrView), ("scale", c_float),
                ("dw", c_void_p), ("db", c_void_p), ("splits", c_int32)]


class IsrEwDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32), ("c", c_int32),
                ("y", IsrView), ("a", IsrView), ("b", IsrView), ("m", IsrView),
                ("sa", c_float), ("sb", c_float), ("mslope", c_float)]


class IsrSrTransformDesc(ctypes.Structure):
    _fields_ = [("crops", c_void_p), ("hr", c_void_p), ("lr", c_void_p), ("n", c_int32), ("t", c_int32),
                ("scale", c_int32), ("hr_norm", c_int32), ("mean", c_float * 3), ("std", c_float * 3)]


class IsrConvertDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32), ("c", c_int32),
                ("nchw", c_void_p), ("v", IsrView), ("scale", c_void_p), ("shift", c_void_p),
                ("m", IsrView), ("mslope", c_float), ("f16", c_int32)]


class IsrPoolDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("c", c_int32), ("hao", c_int32), ("wao", c_int32),
                ("x", IsrView), ("y", IsrView), ("g", IsrView), ("mslope", c_float)]


class IsrBnDesc(ctypes.Structure):
    _fields_ = [("n", c_int32), ("h", c_int32), ("w", c_int32), ("ha", c_int32), ("wa", c_int32), ("c", c_int32),
                ("z", IsrView), ("y", IsrView), ("r1", IsrView), ("r2", IsrView), ("dz", IsrView),
                ("s1", c_float), ("s2", c_float), ("slope", c_float),
                ("gamma", c_void_p), ("beta", c_void_p), ("running_mean", c_void_p), ("running_var", c_void_p),
                ("momentum", c_float), ("eps", c_float), ("acc", c_void_p), ("save", c_void_p),
                ("dgamma", c_void_p), ("dbeta", c_void_p), ("gscale", c_float)]


class IsrAdamArgs(ctypes.Structure):
    _fields_ = [("step", c_float), ("beta1", c_float), ("beta2", c_float), ("eps", c_float),
                ("weight_decay", c_float), ("bc2_sqrt", c_float)]


MT_TENSOR_BYTES = 40  # isr_mt_tensor: 4 pointers + int64
MT_CHUNK_BYTES = 16   # isr_mt_chunk: int32 t, int32 len, int64 start


# Every symbol include/isr.h declares, with its ctypes signature.
SIGNATURES = {
    "isr_conv3x3_packed_bytes": (c_size_t, [c_int32, c_int32]),
    "isr_pack_conv3x3": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "isr_pack_conv3x3_batch": (c_int32, [c_void_p, c_int32, c_void_p]),
    "isr_pack_conv3x3_dgrad": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_float, c_int32, c_void_p]),
    "isr_wgrad3x3_workspace_bytes": (c_size_t, [POINTER(IsrWgradDesc)]),
    "isr_wgrad3x3": (c_int32, [POINTER(IsrWgradDesc), c_void_p, c_size_t, c_void_p]),
    "isr_wgrad3x3_partials": (c_int32, [POINTER(IsrWgradDesc), c_void_p, c_size_t, c_void_p]),
    "isr_wgrad3x3_group_workspace_bytes": (c_size_t, [POINTER(IsrWgradDesc), c_int32]),
    "isr_wgrad3x3_group": (c_int32, [POINTER(IsrWgradDesc), c_int32, c_void_p, c_size_t, c_void_p]),
    "isr_wgrad3x3_group_variant": (c_int32, [POINTER(IsrWgradDesc), c_int32, c_int32, c_void_p, c_size_t, c_void_p]),
    "isr_wgrad3x3_reduce": (c_int32, [POINTER(IsrWgradDesc), c_void_p, c_size_t, c_void_p]),
    "isr_wgrad3x3_variant_workspace_bytes": (c_size_t, [POINTER(IsrWgradDesc), c_int32]),
    "isr_wgrad3x3_variant": (c_int32, [POINTER(IsrWgradDesc), c_int32, c_void_p, c_size_t, c_void_p]),
    "isr_wgrad9x9_workspace_bytes": (c_size_t, [POINTER(IsrWgrad9Desc)]),
    "isr_wgrad9x9": (c_int32, [POINTER(IsrWgrad9Desc), c_void_p, c_size_t, c_void_p]),
    "isr_ew_combine": (c_int32, [POINTER(IsrEwDesc), c_void_p]),
    "isr_pixel_shuffle2": (c_int32, [POINTER(IsrEwDesc), c_void_p]),
    "isr_sr_transform": (c_int32, [POINTER(IsrSrTransformDesc), c_void_p]),
    "isr_pixel_unshuffle2": (c_int32, [POINTER(IsrEwDesc), c_void_p]),
    "isr_bn_stats": (c_int32, [POINTER(IsrBnDesc), c_void_p]),
    "isr_bn_finalize": (c_int32, [POINTER(IsrBnDesc), c_void_p]),
    "isr_bn_apply": (c_int32, [POINTER(IsrBnDesc), c_void_p]),
    "isr_bn_bwd_reduce": (c_int32, [POINTER(IsrBnDesc), c_void_p]),
    "isr_bn_bwd_apply": (c_int32, [POINTER(IsrBnDesc), c_void_p]),
    "isr_nchw_to_blocked": (c_int32, [POINTER(IsrConvertDesc), c_void_p]),
    "isr_blocked_to_nchw": (c_int32, [POINTER(IsrConvertDesc), c_void_p]),
    "isr_maxpool2_fwd": (c_int32, [POINTER(IsrPoolDesc), c_void_p]),
    "isr_maxpool2_bwd": (c_int32, [POINTER(IsrPoolDesc), c_void_p]),
    "isr_head9x9_packed_bytes": (c_size_t, [c_int32, c_int32]),
    "isr_pack_head9x9": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "isr_tail9x9_packed_bytes": (c_size_t, [c_int32, c_int32]),
    "isr_pack_tail9x9": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "isr_pack_conv3x3_f16": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "isr_pack_head9x9_f16": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "isr_pack_tail9x9_f16": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "isr_conv3x3_fwd": (c_int32, [POINTER(IsrConvDesc), c_void_p]),
    "isr_conv3x3_fwd_variant": (c_int32, [POINTER(IsrConvDesc), c_int32, c_void_p]),
    "isr_tuning_conv_stamps": (c_int32, [c_void_p]),
    "isr_tuning_tail_stamps": (c_int32, [c_void_p]),
    "isr_tuning_chain_knobs": (c_int32, [c_int32, c_int32, c_int32, c_int32]),
    "isr_conv3x3_check": (c_int32, [POINTER(IsrConvDesc)]),
    "isr_conv_chain_state_words": (c_size_t, [c_int32, c_int32, c_int32]),
    "isr_conv_chain": (c_int32, [POINTER(IsrChainDesc), c_void_p]),
    "isr_conv_chain_variant": (c_int32, [POINTER(IsrChainDesc), c_int32, c_void_p]),
    "isr_tuning_trunk_stamps": (c_int32, [c_void_p]),
    "isr_tuning_trunk_knobs": (c_int32, [c_int32, c_int32, c_int32, c_int32]),
    "isr_tuning_trunk_item_stamps": (c_int32, [c_void_p]),
    "isr_head9x9_fwd": (c_int32, [POINTER(IsrHeadDesc), c_void_p]),
    "isr_tail9x9_fwd": (c_int32, [POINTER(IsrTailDesc), c_void_p]),
    "isr_tail9x9_fwd_variant": (c_int32, [POINTER(IsrTailDesc), c_int32, c_void_p]),
    "isr_mt_adam": (c_int32, [c_void_p, c_void_p, c_int32, POINTER(IsrAdamArgs), c_void_p, c_void_p]),
    "isr_mt_sumsq": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "isr_clip_coef": (c_int32, [c_void_p, c_int32, c_float, c_void_p, c_void_p]),
    "isr_mt_scale": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p]),
    "isr_mt_lerp": (c_int32, [c_void_p, c_void_p, c_int32, c_float, c_void_p]),
    "isr_mt_adam_guarded": (c_int32, [c_void_p, c_void_p, c_int32, POINTER(IsrAdamArgs), c_void_p, c_void_p,
                                      c_void_p]),
    "isr_mt_lerp_guarded": (c_int32, [c_void_p, c_void_p, c_int32, c_float, c_void_p, c_void_p]),
    "isr_last_error": (ctypes.c_char_p, []),
    "isr_version": (c_int32, []),
}

_lib = None


class IsrError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libisr.so (built by image_super_resolution_amd._build / __graft_entry__.build)."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("ISR_LIB", LIB_PATH))
    if not path.exists():
        raise IsrError(f"libisr.so not found at {path}; run `python -m image_super_resolution_amd._build` "
                       "(or __graft_entry__.build()) first — there is no non-HIP fallback")
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().isr_last_error().decode(errors="replace")
        raise IsrError(f"{what} failed ({rc}): {msg}")
