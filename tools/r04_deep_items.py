#!/usr/bin/env python3
"""Inside one K-chunk of the deep-ring trunk kernel (variant 4; tuning build, ISR_LIB=.../
libisr_tuning.so): s_memtime stamps per phase for layers 77 (growth2) and 79 (final) of each
workgroup's first tile, waves 0 and 4; prints the median cycles of each phase per chunk.
Phases: top (slow path + step-0 reads of a tile's first chunk), steps01 (steps 0-1 issued),
dma_wait (own DMA of the next chunk), barrier, decide (publish, poll, staging decisions,
mid-chunk slow path), step2 (step 2 issued), chunk (top to next top)."""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import _lib, engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402


def main():
    lib = _lib.load()
    engine.CHAIN_VARIANT = 4
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    x = normalize(synth_lr_batch(16, 128, 128, seed=1234)[0]).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, (0.485, 0.456, 0.406),
                                (0.229, 0.224, 0.225), chain=True)
    assert plan.chain is not None and plan.chain.variant == 4
    out = torch.empty(plan.out_shape, device=dev)
    for _ in range(3):
        plan.run(x, out)
    torch.cuda.synchronize()
    grid = 1024
    st = torch.zeros(grid * 2 * 16 * 2 * 8, dtype=torch.int64, device=dev)
    _lib.check(lib.isr_tuning_trunk_item_stamps(ctypes.c_void_p(st.data_ptr())), "stamps")
    plan.run(x, out)
    torch.cuda.synchronize()
    _lib.check(lib.isr_tuning_trunk_item_stamps(None), "off")
    a = st.view(grid, 2, 16, 2, 8).cpu()
    used = (a[:, 0, 0, 0, 0] != 0).nonzero().flatten()
    a = a[used].double()
    names = ["top", "steps01", "dma_wait", "barrier", "decide", "step2"]
    for li, (name, nch) in enumerate((("growth2", 8), ("final", 12))):
        for w in range(2):
            rows = []
            for ch in range(nch):
                s = a[:, li, ch, w]
                ph = {n: (s[:, j + 1] - s[:, j]).median().item() for j, n in enumerate(names)}
                if ch + 1 < nch:
                    ph["chunk"] = (a[:, li, ch + 1, w, 0] - s[:, 0]).median().item()
                rows.append({k: round(v) for k, v in ph.items()})
            print(json.dumps({"layer": name, "wave": 4 * w, "chunks": rows}), flush=True)


if __name__ == "__main__":
    main()
