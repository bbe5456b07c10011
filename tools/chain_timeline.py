#!/usr/bin/env python3
"""Per-tile timeline inside the persistent trunk kernel (tuning build:
ISR_LIB=.../libisr_tuning.so): stamps for the 15 layers of RRDB 5 — wait for the 3x3
neighbourhood, prologue (chunk 0 landed), main loop, epilogue + store drain — as
percentile rows in microseconds.  usage: python tools/chain_timeline.py"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402

L0 = 75
BASE = 65536  # CHAIN_STAMP_BASE in conv3x3.hip


def pct(v, qs=(0.1, 0.5, 0.9, 1.0)):
    v = sorted(v)
    return [round(v[min(len(v) - 1, int(q * len(v)))], 2) for q in qs]


def main():
    lib = _lib.load()
    variant = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    _lib.check(lib.isr_tuning_chain_knobs(0, 0, variant, 0), "knobs")
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
    lr, _ = synth_lr_batch(16, 128, 128, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, (0.485, 0.456, 0.406),
                                (0.229, 0.224, 0.225), chain=True)
    out = torch.empty(plan.out_shape, device=dev)
    for _ in range(3):
        plan.run(x, out)
    torch.cuda.synchronize()
    ntiles = plan.chain.ntiles if hasattr(plan.chain, 'ntiles') else (256 if variant in (2, 3, 4) else 512)
    st = torch.zeros((BASE + 15 * ntiles) * 8, dtype=torch.int64, device=dev)
    _lib.check(lib.isr_tuning_conv_stamps(ctypes.c_void_p(st.data_ptr())), "stamps")
    plan.run(x, out)
    torch.cuda.synchronize()
    _lib.check(lib.isr_tuning_conv_stamps(None), "stamps off")
    a = st.view(-1, 8)[BASE:].view(15, ntiles, 8).cpu().double() / 100.0  # 100 MHz ticks -> us
    t0 = a[0, :, 4].min().item()
    for L in range(15):
        w0, e, c0, m, dn = a[L, :, 4], a[L, :, 0], a[L, :, 1], a[L, :, 2], a[L, :, 3]
        row = {"layer": L0 + L, "kind": "final" if L % 5 == 4 else f"growth{L % 5}",
               "start_p10..max": pct((w0 - t0).tolist()), "end_p10..max": pct((dn - t0).tolist()),
               "wait": pct((e - w0).tolist()), "setup": pct((a[L, :, 5] - e).tolist()),
               "dma0": pct((c0 - a[L, :, 5]).tolist()), "prologue": pct((c0 - e).tolist()),
               "main": pct((m - c0).tolist()), "epi+drain": pct((dn - m).tolist()),
               "tile_total": pct((dn - w0).tolist())}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
