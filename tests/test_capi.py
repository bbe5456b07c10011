"""C-ABI checks that need no GPU: libisr.so loads, exports every symbol
include/isr.h declares, the ctypes mirrors match the C struct layouts (probed
with gcc), and descriptor validation rejects bad input before any launch."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

from conftest import ROOT
from image_super_resolution_amd import _lib

HEADER = ROOT / "include" / "isr.h"


def declared_functions():
    txt = HEADER.read_text()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(isr_[a-z0-9_]+)\s*\(", txt)))


def test_all_header_symbols_exported(built_lib):
    names = declared_functions()
    assert len(names) >= 12
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (isr_[a-z0-9_]+)\b", nm))
    missing = [n for n in names if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    # and the ctypes binding knows every one of them
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "isr.h"
#define F(s, m) printf(#s "." #m " %zu\n", offsetof(s, m))
#define S(s) printf(#s " %zu\n", sizeof(s))
int main(void) {
  printf("isr_view %zu\nisr_conv_desc %zu\nisr_head_desc %zu\nisr_tail_desc %zu\n",
         sizeof(isr_view), sizeof(isr_conv_desc), sizeof(isr_head_desc), sizeof(isr_tail_desc));
  F(isr_view, coff); F(isr_conv_desc, x); F(isr_conv_desc, r2); F(isr_conv_desc, wpack);
  F(isr_conv_desc, bias); F(isr_conv_desc, slope); F(isr_conv_desc, shuffle);
  F(isr_head_desc, x); F(isr_head_desc, x_u8); F(isr_head_desc, inv_std); F(isr_head_desc, y);
  F(isr_head_desc, slope); F(isr_tail_desc, x); F(isr_tail_desc, y); F(isr_tail_desc, y_u8);
  S(isr_chain_desc); F(isr_chain_desc, kinds); F(isr_chain_desc, nl); F(isr_chain_desc, wa);
  F(isr_chain_desc, state); F(isr_chain_desc, acquire);
  S(isr_pack_item); F(isr_pack_item, scale); F(isr_pack_item, src_n0); F(isr_pack_item, src_cin);
  return 0;
}
"""


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), str(src), "-o", str(exe)], check=True)
    c = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines())
    py = {"isr_view": ctypes.sizeof(_lib.IsrView), "isr_conv_desc": ctypes.sizeof(_lib.IsrConvDesc),
          "isr_head_desc": ctypes.sizeof(_lib.IsrHeadDesc), "isr_tail_desc": ctypes.sizeof(_lib.IsrTailDesc),
          "isr_chain_desc": ctypes.sizeof(_lib.IsrChainDesc)}
    for k, v in py.items():
        assert int(c[k]) == v, k
    # isr_pack_item is written by ops.pack_batch_table with struct "<QQiiiifiii"
    assert int(c["isr_pack_item"]) == 48
    assert (int(c["isr_pack_item.scale"]), int(c["isr_pack_item.src_n0"]), int(c["isr_pack_item.src_cin"])) == (32, 36, 40)
    cls = {"isr_view": _lib.IsrView, "isr_conv_desc": _lib.IsrConvDesc, "isr_head_desc": _lib.IsrHeadDesc,
           "isr_tail_desc": _lib.IsrTailDesc, "isr_chain_desc": _lib.IsrChainDesc}
    for key, val in c.items():
        if "." in key and not key.startswith("isr_pack_item"):
            s, m = key.split(".")
            assert getattr(cls[s], m).offset == int(val), key


def test_validation_rejects_without_touching_gpu(built_lib):
    lib = built_lib
    assert lib.isr_version() >= 1
    assert lib.isr_conv3x3_fwd(None, None) == -1
    assert b"null descriptor" in lib.isr_last_error()
    d = _lib.IsrConvDesc()
    d.n, d.h, d.w, d.ha, d.wa, d.cin, d.cout = 1, 16, 32, 32, 32, 40, 64
    assert lib.isr_conv3x3_fwd(ctypes.byref(d), None) == -2
    assert b"multiple of 16" in lib.isr_last_error()
    d.cin = 64
    d.ha = 16  # not tile aligned (ISR_TILE_H = 32)
    assert lib.isr_conv3x3_fwd(ctypes.byref(d), None) == -1
    d.ha = 32
    assert lib.isr_conv3x3_fwd(ctypes.byref(d), None) == -1  # null weights / views
    assert lib.isr_head9x9_fwd(None, None) == -1
    assert lib.isr_tail9x9_fwd(None, None) == -1
    assert lib.isr_pack_conv3x3(None, None, 64, 64, None) == -1
    assert lib.isr_pack_tail9x9(ctypes.c_void_p(16), ctypes.c_void_p(16), 4, 64, None) == -2


def test_packed_sizes(built_lib):
    lib = built_lib
    assert lib.isr_conv3x3_packed_bytes(64, 192) == 64 * 192 * 9 * 2
    assert lib.isr_head9x9_packed_bytes(64, 3) == 9 * 3 * 64 * 16 * 2
    assert lib.isr_tail9x9_packed_bytes(3, 64) == 9 * 2 * 2 * 32 * 32


def test_product_path_refuses_cpu_tensors():
    import torch
    from image_super_resolution_amd import models
    m = models.ResNet(1, 0.2, scaleRate=2).eval()
    with pytest.raises(RuntimeError, match="HIP"):
        with torch.no_grad():
            m(torch.zeros(1, 3, 16, 16))
