#!/usr/bin/env python3
"""Does running independent sub-batches of one conv on several HIP streams overlap
their prologue/epilogue phases?  Times conv shapes as 1 stream x batch N vs
S streams x batch N/S (same total work), per kernel variant."""
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--streams", default="1,2,4")
    args = ap.parse_args()
    lib = _lib.load()
    dev = "cuda"
    n, s = args.n, args.hw
    for cin, cout in [(64, 32), (160, 32), (192, 64)]:
        g = torch.Generator().manual_seed(cin)
        w = (torch.rand(cout, cin, 3, 3, generator=g) * 2 - 1).mul((3.0 / (cin * 9)) ** 0.5).to(dev)
        b = torch.randn(cout, generator=g).mul(0.1).to(dev)
        wp = ops.pack_conv3x3(w)
        row = {"cin": cin, "cout": cout}
        for S in [int(v) for v in args.streams.split(",")]:
            m = n // S
            srcs, dsts, descs = [], [], []
            for j in range(S):
                src = ops.ActBuffer.alloc(m, s, s, 192, 1, dev)
                src.set_nchw(torch.randn(m, cin, s, s, generator=g).to(dev), 0)
                if cout == 32:
                    dst, kw = src, dict(y_coff=cin, slope=0.01)
                else:
                    dst = ops.ActBuffer.alloc(m, s, s, 192, 1, dev)
                    kw = dict(slope=1.0, r1=src, s1=0.2, r2=src, s2=0.2)
                srcs.append(src), dsts.append(dst)
                descs.append(ops.conv3x3_desc(src, cin, wp, b, cout, dst, **kw))
            streams = [torch.cuda.Stream() for _ in range(S)]
            sp = [ctypes.c_void_p(st.cuda_stream) for st in streams]
            for v in [int(x) for x in args.variants.split(",")]:
                ts = []
                for _ in range(3):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for st in streams:
                        st.wait_stream(torch.cuda.current_stream())
                    for _ in range(args.reps):
                        for j in range(S):
                            lib.isr_conv3x3_fwd_variant(ctypes.byref(descs[j]), v, sp[j])
                    for st in streams:
                        torch.cuda.current_stream().wait_stream(st)
                    e1.record()
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1) / args.reps * 1e3)
                row[f"S{S}_v{v}_us"] = round(statistics.median(ts), 2)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
