#!/usr/bin/env python3
"""Per-block timeline of conv3x3 launches (tuning build: ISR_LIB=.../libisr_tuning.so).

For each shape, one launch at N=16 128² with per-block s_memrealtime stamps
(entry, first chunk landed, main loop done, epilogue done) and the CU / XCD ids:
prints the launch's span, start skew, and the distribution of prologue / main loop
/ epilogue durations, in microseconds.  usage: python tools/conv_timeline.py
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, ops  # noqa: E402


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def main():
    lib = _lib.load()
    dev = "cuda"
    n, s = 16, 128
    for cin, cout in [(64, 32), (160, 32), (192, 64)]:
        g = torch.Generator().manual_seed(cin)
        src = ops.ActBuffer.alloc(n, s, s, 192, 1, dev)
        src.set_nchw(torch.randn(n, cin, s, s, generator=g).to(dev), 0)
        w = (torch.rand(cout, cin, 3, 3, generator=g) * 2 - 1).mul((3.0 / (cin * 9)) ** 0.5).to(dev)
        b = torch.randn(cout, generator=g).mul(0.1).to(dev)
        wp = ops.pack_conv3x3(w)
        if cout == 32:
            d = ops.conv3x3_desc(src, cin, wp, b, cout, src, y_coff=cin, slope=0.01)
        else:
            dst = ops.ActBuffer.alloc(n, s, s, 192, 1, dev)
            d = ops.conv3x3_desc(src, cin, wp, b, cout, dst, slope=1.0, r1=src, s1=0.2)
        blocks = (d.wa // 32) * (d.ha // 16) * n * (cout // (64 if cout % 64 == 0 else 32))
        st = torch.zeros(blocks * 8, dtype=torch.int64, device=dev)
        for _ in range(5):
            lib.isr_conv3x3_fwd(ctypes.byref(d), ops._stream())
        torch.cuda.synchronize()
        _lib.check(lib.isr_tuning_conv_stamps(ctypes.c_void_p(st.data_ptr())), "stamps")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.isr_conv3x3_fwd(ctypes.byref(d), ops._stream())
        e1.record()
        torch.cuda.synchronize()
        _lib.check(lib.isr_tuning_conv_stamps(None), "stamps off")
        a = st.view(blocks, 8).cpu()
        t0 = a[:, 0].min().item()
        us = lambda x: x / 100.0  # 100 MHz ticks → µs
        start = [us(v - t0) for v in a[:, 0].tolist()]
        pro = [us(x) for x in (a[:, 1] - a[:, 0]).tolist()]
        main_ = [us(x) for x in (a[:, 2] - a[:, 1]).tolist()]
        epi = [us(x) for x in (a[:, 3] - a[:, 2]).tolist()]
        end = [us(v - t0) for v in a[:, 3].tolist()]
        xcc = a[:, 7].tolist()
        hw = a[:, 6].tolist()
        cu_ids = {(int(x) & 0xF, (int(h) >> 8) & 0xF, (int(h) >> 13) & 0x3) for x, h in zip(xcc, hw)}
        row = {"cin": cin, "cout": cout, "blocks": blocks, "event_us": round(e0.elapsed_time(e1) * 1e3, 2),
               "span_us": round(max(end), 2), "start_p50/p100": [round(pct(start, .5), 2), round(max(start), 2)]}
        for name, v in (("prologue", pro), ("main", main_), ("epilogue", epi), ("end", end)):
            row[name] = [round(pct(v, q), 2) for q in (0.0, 0.1, 0.5, 0.9, 1.0)]
        row["distinct_cu_slots"] = len(cu_ids)
        # the two blocks sharing a CU: is the earlier-dispatched one faster (wave age wins issue)?
        by_cu = {}
        for i, (x, h) in enumerate(zip(xcc, hw)):
            by_cu.setdefault((int(x) & 0xF, int(h) & 0xFF00), []).append(i)
        first, second, gap = [], [], []
        for idx in by_cu.values():
            if len(idx) == 2:
                a_, b_ = sorted(idx, key=lambda i: start[i])
                first.append(end[a_])
                second.append(end[b_])
                gap.append(start[b_] - start[a_])
        if first:
            row["end_first_slot_p50"] = round(pct(first, .5), 2)
            row["end_second_slot_p50"] = round(pct(second, .5), 2)
            row["second_later_frac"] = round(sum(b > a for a, b in zip(first, second)) / len(first), 3)
        per_xcd = {}
        for i, x in enumerate(xcc):
            per_xcd.setdefault(int(x) & 0xF, []).append(end[i])
        row["end_p50_by_xcd"] = {k: round(pct(v, .5), 2) for k, v in sorted(per_xcd.items())}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
