#!/usr/bin/env python3
"""Per-wave timeline of the row-streaming tail (tail variant 36 = 4 with stamps; tuning
build: ISR_LIB=.../libisr_tuning.so).  One launch at 16 x 64ch x 512² -> fp32: prints the
launch span, the block lifetime, and per wave the share of the summed top-of-group wait
(DMA + barrier) and of the loop body, in microseconds.  usage: python tools/tail_timeline.py
"""
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
n, s = 16, 512
g = torch.Generator().manual_seed(0)
xb = ops.ActBuffer.alloc(n, s, s, 64, 4, "cuda")
xb.set_nchw((torch.randn(n, 64, s, s, generator=g) * 0.5).cuda(), 0)
wp = ops.pack_tail9x9((torch.randn(3, 64, 9, 9, generator=g) * 0.02).cuda())
b = torch.zeros(3, device="cuda")
out = torch.empty(n, 3, s, s, device="cuda")
d = ops.tail9x9_desc(xb, wp, b, out)
st = ops._stream()
blocks = n * (s // 32) * (s // 128)
buf = torch.zeros(blocks * 4 * 4, dtype=torch.int64, device="cuda")
for _ in range(3):
    ops.check(lib.isr_tail9x9_fwd_variant(ctypes.byref(d), 4, st), "tail")
ops.check(lib.isr_tuning_tail_stamps(ctypes.c_void_p(buf.data_ptr())), "stamps")
ops.check(lib.isr_tail9x9_fwd_variant(ctypes.byref(d), 36, st), "tail stamped")
torch.cuda.synchronize()
ops.check(lib.isr_tuning_tail_stamps(None), "stamps off")
v = buf.view(blocks, 4, 4).cpu().double() / 100.0  # 100 MHz ticks -> us
entry, exit_, wait, loop = v[..., 0], v[..., 1], v[..., 2], v[..., 3]
t0 = entry.min().item()
life = (exit_ - entry).flatten().tolist()
res = {"blocks": blocks, "span_us": round(exit_.max().item() - t0, 1),
       "block_life_us": {"median": round(statistics.median(life), 2), "min": round(min(life), 2), "max": round(max(life), 2)},
       "wait_us_median": round(statistics.median(wait.flatten().tolist()), 2),
       "loop_us_median": round(statistics.median(loop.flatten().tolist()), 2),
       "entry_skew_first256_us": round((entry[:256].max() - entry[:256].min()).item(), 2)}
starts = sorted(entry[:, 0].tolist())
res["start_quartiles_us"] = [round(starts[int(q * (blocks - 1))] - t0, 1) for q in (0, 0.25, 0.5, 0.75, 1.0)]
print(json.dumps(res))
