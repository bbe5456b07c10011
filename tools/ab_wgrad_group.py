"""Time the grouped RDB weight-gradient launch (isr_wgrad3x3_group) at the cfg3 shape and dump its
dW / db, so tile configurations (tuning build, ISR_WGRAD_GROUP_CFG, read once per process) can be
compared for time and for bit-identity across processes.

usage: ISR_LIB=.../libisr_tuning.so ISR_WGRAD_GROUP_CFG=8 python tools/ab_wgrad_group.py --dump /tmp/a.pt
       python tools/ab_wgrad_group.py --compare /tmp/a.pt /tmp/b.pt
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--hw", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dump", default="")
    ap.add_argument("--compare", nargs=2, default=None)
    a = ap.parse_args()
    if a.compare:
        x, y = (torch.load(p, weights_only=True) for p in a.compare)
        same = all(torch.equal(x[k], y[k]) for k in x)
        diff = max((x[k] - y[k]).abs().max().item() for k in x)
        print(json.dumps({"bitwise": same, "max_abs_diff": diff}))
        return
    from image_super_resolution_amd import _lib, ops
    lib = _lib.load()
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(81)
    D = (torch.randn(a.n, 192, a.hw, a.hw, generator=g) * 0.5).to(dev, torch.bfloat16).float()
    E = (torch.randn(a.n, 192, a.hw, a.hw, generator=g) * 0.5).to(dev, torch.bfloat16).float()
    Db, Eb = ops.ActBuffer.from_nchw(D, pad=1), ops.ActBuffer.from_nchw(E, pad=1)
    shapes = [(192, 64, 0, 0.04), (160, 32, 64, 1.0), (128, 32, 96, 1.0), (96, 32, 128, 1.0), (64, 32, 160, 1.0)]
    outs, descs = [], []
    for cin, cout, gco, sc in shapes:
        dw = torch.empty(cout, cin, 3, 3, device=dev)
        db = torch.empty(cout, device=dev)
        outs.append((dw, db))
        descs.append(ops.wgrad3x3_desc(Db, cin, Eb, cout, dw, db, g_coff=gco, scale=sc))
    arr = (_lib.IsrWgradDesc * 5)(*descs)
    nbytes = lib.isr_wgrad3x3_group_workspace_bytes(arr, 5)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        assert lib.isr_wgrad3x3_group(arr, 5, ws.data_ptr(), ws.numel(), st) == 0
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.reps)]
    for i in range(a.reps):
        ev[2 * i].record()
        lib.isr_wgrad3x3_group(arr, 5, ws.data_ptr(), ws.numel(), st)
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    ms = sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(a.reps))
    macs = a.n * a.hw * a.hw * 9 * sum(ci * co for ci, co, _, _ in shapes)
    med = ms[len(ms) // 2]
    print(json.dumps({"cfg": os.environ.get("ISR_WGRAD_GROUP_CFG", "0"), "median_ms": round(med, 4),
                      "min_ms": round(ms[0], 4), "tflop_s": round(2 * macs / med / 1e9, 1),
                      "note": "wgrad + group reduce launches, N=%d %d^2" % (a.n, a.hw)}))
    if a.dump:
        torch.save({f"w{i}": dw.cpu() for i, (dw, _) in enumerate(outs)} |
                   {f"b{i}": db.cpu() for i, (_, db) in enumerate(outs)}, a.dump)


if __name__ == "__main__":
    main()
