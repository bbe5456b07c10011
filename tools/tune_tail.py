#!/usr/bin/env python3
"""A/B the tail9x9 kernels (isr_tail9x9_fwd_variant) on the 4x generator's tail:
16 x 64ch x 512² bf16 → 16 x 3 x 512² (fp32 and uint8 out), interleaved rounds."""
from __future__ import annotations

import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, ops  # noqa: E402

lib = _lib.load()
VS = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,0").split(",")]
n, s = 16, 512
g = torch.Generator().manual_seed(0)
xb = ops.ActBuffer.alloc(n, s, s, 64, 4, "cuda")
xb.set_nchw((torch.randn(n, 64, s, s, generator=g) * 0.5).cuda(), 0)
wp = ops.pack_tail9x9((torch.randn(3, 64, 9, 9, generator=g) * 0.02).cuda())
b = torch.zeros(3, device="cuda")
flops = 2.0 * n * s * s * 3 * 64 * 81
for dt in (torch.float32,):
    out = torch.empty(n, 3, s, s, device="cuda", dtype=dt)
    d = ops.tail9x9_desc(xb, wp, b, out)
    st = ops._stream()
    res = {v: [] for v in VS}
    for _ in range(7):
        for v in res:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.check(lib.isr_tail9x9_fwd_variant(ctypes.byref(d), v, st), "tail")
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(json.dumps({"out": str(dt), **{f"v{v}_us": round(statistics.median(t), 1) for v, t in res.items()},
                      "in_bytes": xb.t.numel() * 2, **{f"v{v}_in_GBps": round(xb.t.numel() * 2 / statistics.median(t) / 1e3, 1)
                                                       for v, t in res.items()}}))
