#!/usr/bin/env python3
"""Persistent-trunk probes (tuning build: ISR_LIB=.../libisr_tuning.so).

1. Placement: which chain workgroups share a CU (HW_ID / XCC_ID recorded at entry) —
   block-index deltas of co-resident pairs, and whether a pair's tiles are in
   independent images.
2. Phase offset: workgroups with bit `shift` of blockIdx set start `delay` µs late; with
   co-resident pairs split across independent image groups, one group's epilogue /
   prologue can then run beside the other's main loop.  Whole-forward time per delay,
   HIP-graph replays, interleaved rounds, outputs must stay bit-identical.
usage: ISR_LIB=image_super_resolution_amd/lib/libisr_tuning.so python tools/chain_probe.py
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402

BASE = 65536  # CHAIN_STAMP_BASE in conv3x3.hip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--delays-us", default="0,4,8,12,16")
    ap.add_argument("--shift", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--variants", default="", help="chain kernel variants to A/B (isr_tuning_chain_knobs k2)")
    args = ap.parse_args()
    lib = _lib.load()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    lr, _ = synth_lr_batch(16, 128, 128, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, (0.485, 0.456, 0.406),
                                (0.229, 0.224, 0.225), chain=True)
    out = torch.empty(plan.out_shape, device=dev)
    _lib.check(lib.isr_tuning_chain_knobs(0, 0, 0, 0), "knobs")
    plan.run(x, out)
    torch.cuda.synchronize()
    ntiles = 512
    st = torch.zeros((BASE + 16 * ntiles) * 8, dtype=torch.int64, device=dev)
    _lib.check(lib.isr_tuning_conv_stamps(ctypes.c_void_p(st.data_ptr())), "stamps")
    plan.run(x, out)
    torch.cuda.synchronize()
    _lib.check(lib.isr_tuning_conv_stamps(None), "stamps off")
    a = st.view(-1, 8)[BASE:].view(16, ntiles, 8)[15].cpu()
    grid = int((a[:, 7] != 0).sum().item()) or ntiles
    cus = collections.defaultdict(list)
    for b in range(ntiles):
        hw, xcc = int(a[b, 6]), int(a[b, 7])
        cus[(xcc, (hw >> 8) & 0xFF)].append(b)  # HW_ID [15:8] = se, sh, cu
    sizes = collections.Counter(len(v) for v in cus.values())
    deltas = collections.Counter(v[1] - v[0] for v in cus.values() if len(v) == 2)
    same_img = sum(1 for v in cus.values() if len(v) == 2 and v[0] // 32 == v[1] // 32)
    print(json.dumps({"cus": len(cus), "blocks_per_cu": dict(sizes), "pair_delta_top": deltas.most_common(6),
                      "pairs_same_image": same_img, "grid_seen": grid}), flush=True)

    ref = out.clone()
    g = engine.GraphedPlan(plan, x, out)
    if args.variants:
        graphs = {}
        for v in (int(q) for q in args.variants.split(",")):
            _lib.check(lib.isr_tuning_chain_knobs(0, 0, v, 0), "knobs")
            p = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, (0.485, 0.456, 0.406),
                                     (0.229, 0.224, 0.225), chain=True)
            o = torch.empty(p.out_shape, device=dev)
            graphs[v] = (engine.GraphedPlan(p, x, o), p, o)  # captured with variant v's kernel
        _lib.check(lib.isr_tuning_chain_knobs(0, 0, 0, 0), "knobs")
        t = {v: [] for v in graphs}
        for _ in range(args.rounds):
            for v, (gv, p, o) in graphs.items():
                gv.run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.steps):
                    gv.run()
                e1.record()
                torch.cuda.synchronize()
                assert not p.chain.failed(), v
                t[v].append(e0.elapsed_time(e1) / args.steps)
        for v, (gv, p, o) in graphs.items():
            print(json.dumps({"variant": v, "ms_median": round(statistics.median(t[v]), 4), "ms_min": round(min(t[v]), 4),
                              "identical": bool(torch.equal(o, ref)),
                              "max_abs_diff": float((o - ref).abs().max())}), flush=True)
        return
    delays = [float(v) for v in args.delays_us.split(",")]
    t = {d: [] for d in delays}
    for _ in range(args.rounds):
        for d in delays:
            _lib.check(lib.isr_tuning_chain_knobs(int(d * 100), args.shift, 0, 0), "knobs")
            g.run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.steps):
                g.run()
            e1.record()
            torch.cuda.synchronize()
            assert not plan.chain.failed(), d
            assert torch.equal(out, ref), f"delay {d}: output differs"
            t[d].append(e0.elapsed_time(e1) / args.steps)
    _lib.check(lib.isr_tuning_chain_knobs(0, 0, 0, 0), "knobs")
    for d in delays:
        print(json.dumps({"delay_us": d, "shift": args.shift, "ms_median": round(statistics.median(t[d]), 4),
                          "ms_min": round(min(t[d]), 4)}), flush=True)

if __name__ == "__main__":
    main()
