#!/usr/bin/env python3
"""A/B the wgrad3x3 kernel variants (isr_wgrad3x3_variant) on the generator's
training shapes (N=16, 128² LR): interleaved rounds in one process; each variant's
dW is checked against variant 1 (relative L2)."""
from __future__ import annotations

import argparse
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--hw", type=int, default=128)
    ap.add_argument("--variants", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--splits", default="", help="variant:splits pairs, e.g. 0:128,0:256 (split-K override)")
    args = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    n, s = args.n, args.hw
    shapes = [(64, 32, False), (96, 32, False), (128, 32, False), (160, 32, False), (192, 64, False),
              (64, 64, False), (64, 256, True)]
    vs = [int(v) for v in args.variants.split(",")]
    # (variant, splits) configurations: splits 0 = the library's own choice
    cfgs = [(v, 0) for v in vs] + [tuple(int(q) for q in c.split(":")) for c in args.splits.split(",") if c]
    for cin, cout, sub2 in shapes:
        g = torch.Generator().manual_seed(cin + cout)
        x = ops.ActBuffer.alloc(n, s, s, 192, 1, dev)
        x.set_nchw(torch.randn(n, cin, s, s, generator=g).to(dev), 0)
        if sub2:
            gb = ops.ActBuffer.alloc(n, 2 * s, 2 * s, 64, 2, dev, ha=2 * x.ha, wa=2 * x.wa)
            gb.set_nchw(torch.randn(n, 64, 2 * s, 2 * s, generator=g).to(dev), 0)
        else:
            gb = ops.ActBuffer.alloc(n, s, s, max(64, cout), 1, dev)
            gb.set_nchw(torch.randn(n, cout, s, s, generator=g).to(dev), 0)
        dw = torch.empty(cout, cin, 3, 3, device=dev)
        db = torch.empty(cout, device=dev)
        d = ops.wgrad3x3_desc(x, cin, gb, cout, dw, db, g_sub2=sub2)
        st = ops._stream()
        res, ok = {}, []
        for v, sp in cfgs:
            d.splits = sp
            nb = lib.isr_wgrad3x3_variant_workspace_bytes(ctypes.byref(d), v)
            ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=dev)
            rc = lib.isr_wgrad3x3_variant(ctypes.byref(d), v, ws.data_ptr(), ws.numel(), st)
            if rc == 0:
                torch.cuda.synchronize()
                res[(v, sp)] = (dw.clone(), db.clone(), ws)
                ok.append((v, sp))
        times = {v: [] for v in ok}
        for _ in range(args.rounds):
            for v in ok:
                ws = res[v][2]
                d.splits = v[1]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    lib.isr_wgrad3x3_variant(ctypes.byref(d), v[0], ws.data_ptr(), ws.numel(), st)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps * 1e3)
        flops = 2.0 * n * s * s * 9 * cin * cout * (4 if sub2 else 1)
        row = {"cin": cin, "cout": cout, "sub2": sub2}
        base = res[ok[0]][0]
        for v in ok:
            us = statistics.median(times[v])
            tag = f"v{v[0]}" + (f"s{v[1]}" if v[1] else "")
            row[f"{tag}_us"] = round(us, 1)
            row[f"{tag}_tf"] = round(flops / us / 1e6, 0)
            row[f"{tag}_rel"] = float(((res[v][0] - base).norm() / base.norm()).item())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
