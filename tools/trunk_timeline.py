#!/usr/bin/env python3
"""Per-tile timeline inside the production trunk kernel (trunk.hip; tuning build:
ISR_LIB=.../libisr_tuning.so): stamps for the 15 layers of RRDB 5 (layers 75..89) —
tile entry, chunk 0 landed, main loop done, stores issued, and (deferred refills only) the
blocking dependency wait — as percentile rows in microseconds, plus the spacing of layer
starts.  usage: python tools/trunk_timeline.py [acquire 0/1] [batch] [lr] [variant 0/2]"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402


def pct(v, qs=(0.1, 0.5, 0.9, 1.0)):
    v = sorted(v)
    return [round(v[min(len(v) - 1, int(q * len(v)))], 2) for q in qs] if v else []


def main():
    lib = _lib.load()
    acquire = bool(int(sys.argv[1])) if len(sys.argv) > 1 else False
    engine.CHAIN_VARIANT = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    lrs = int(sys.argv[3]) if len(sys.argv) > 3 else 128
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    lr, _ = synth_lr_batch(n, lrs, lrs, seed=1234)
    x = normalize(lr).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, n, lrs, lrs, dev, False, False, (0.485, 0.456, 0.406),
                                (0.229, 0.224, 0.225), chain=True, chain_acquire=acquire)
    out = torch.empty(plan.out_shape, device=dev)
    for _ in range(3):
        plan.run(x, out)
    torch.cuda.synchronize()
    ntiles = n * (plan.bufs.feat.ha // 16) * (plan.bufs.feat.wa // 32)
    st = torch.zeros(15 * ntiles * 8, dtype=torch.int64, device=dev)
    _lib.check(lib.isr_tuning_trunk_stamps(ctypes.c_void_p(st.data_ptr())), "stamps")
    plan.run(x, out)
    torch.cuda.synchronize()
    _lib.check(lib.isr_tuning_trunk_stamps(None), "stamps off")
    assert not plan.chain.failed()
    a = st.view(15, ntiles, 8).cpu().double() / 100.0  # 100 MHz ticks -> us
    t0 = a[0, :, 0].min().item()
    for L in range(15):
        e, c0, m, dn, w0, w1 = (a[L, :, k] for k in range(6))
        deferred = (w0 > 0).nonzero().flatten().tolist()
        row = {"layer": 75 + L, "kind": "final" if L % 5 == 4 else f"growth{L % 5}",
               "start_p10..max": pct((e - t0).tolist()),
               "chunk0": pct((c0 - e).tolist()), "main": pct((m - c0).tolist()),
               "epi": pct((dn - m).tolist()), "tile": pct((dn - e).tolist()),
               "deferred_tiles": len(deferred),
               "deferred_wait": pct([(w1[i] - w0[i]).item() for i in deferred])}
        if L + 1 < 15:
            row["to_next_start"] = pct((a[L + 1, :, 0] - e).tolist())
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
