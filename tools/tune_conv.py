#!/usr/bin/env python3
"""A/B the conv3x3 kernel variants on every conv shape of the 4x RRDB generator.

Runs all variants interleaved in one process (cdna_hip_programming.md §5.4
rule 24), on random data, and checks each variant's output against variant 0.
Usage (GPU box):  python tools/tune_conv.py [--n 16] [--hw 128] [--rounds 5]
"""
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="", help="comma list of CINxCOUT shapes, e.g. 160x32,192x64")
    ap.add_argument("--final-r1-only", action="store_true", help="192->64 with r1 only (RDB 1/2 final conv)")
    args = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    n, hw = args.n, args.hw
    variants = [int(v) for v in args.variants.split(",")]
    shapes = [(64, 32, 1, hw), (96, 32, 1, hw), (128, 32, 1, hw), (160, 32, 1, hw), (192, 64, 1, hw),
              (64, 64, 1, hw), (64, 256, 2, hw), (64, 256, 2, 2 * hw),
              # long-K shapes: fixed per-block latency amortised → main-loop throughput
              (512, 32, 1, hw), (512, 64, 1, hw),
              # backward (dgrad) shapes of the growth convs: cin' = 32, cout' = layer cin
              (32, 64, 1, hw), (32, 96, 1, hw), (32, 128, 1, hw), (32, 160, 1, hw)]
    if args.only:
        keep = {tuple(int(v) for v in s.split("x")) for s in args.only.split(",")}
        shapes = [s for s in shapes if (s[0], s[1]) in keep]
    results = []
    for cin, cout, shuffle, s in shapes:
        g = torch.Generator().manual_seed(cin + cout)
        src = ops.ActBuffer.alloc(n, s, s, max(192, cin + 32), 1, dev)
        src.set_nchw(torch.randn(n, cin, s, s, generator=g).to(dev), 0)
        w = (torch.rand(cout, cin, 3, 3, generator=g) * 2 - 1).mul((3.0 / (cin * 9)) ** 0.5).to(dev)
        b = torch.randn(cout, generator=g).mul(0.1).to(dev)
        wp = ops.pack_conv3x3(w)
        if shuffle == 2:
            dst = ops.ActBuffer.alloc(n, 2 * s, 2 * s, cout // 4, 1, dev, ha=2 * src.ha, wa=2 * src.wa)
            kw = dict(slope=0.01, shuffle=2)
        elif cout == 32:
            dst = src
            kw = dict(y_coff=cin, slope=0.01)
        else:
            dst = ops.ActBuffer.alloc(n, s, s, 192, 1, dev)
            kw = dict(slope=1.0) if cin != 192 else (dict(slope=1.0, r1=src, s1=0.2) if args.final_r1_only
                                                       else dict(slope=1.0, r1=src, s1=0.2, r2=src, s2=0.2))
        d = ops.conv3x3_desc(src, cin, wp, b, cout, dst, **kw)
        stream = ops._stream()
        outs = {}
        ok = []
        for v in variants:
            rc = lib.isr_conv3x3_fwd_variant(ctypes.byref(d), v, stream)
            if rc == 0:
                ok.append(v)
                torch.cuda.synchronize()
                sl = dst.t[:, cin // 16:cin // 16 + 2] if (cout == 32) else dst.t
                outs[v] = sl.float().clone()
        times = {v: [] for v in ok}
        for _ in range(args.rounds):
            for v in ok:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    lib.isr_conv3x3_fwd_variant(ctypes.byref(d), v, stream)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / args.reps * 1e3)
        flops = 2.0 * n * s * s * 9 * cin * cout
        row = {"cin": cin, "cout": cout, "shuffle": shuffle, "hw": s}
        base = outs[ok[0]]
        for v in ok:
            us = statistics.median(times[v])
            err = (outs[v] - base).abs().max().item()
            row[f"v{v}_us"] = round(us, 2)
            row[f"v{v}_tflops"] = round(flops / us / 1e6, 1)
            row[f"v{v}_maxdiff"] = err
        results.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(results, indent=1))


if __name__ == "__main__":
    main()
