#!/usr/bin/env python3
"""First GPU contact of the deep-ring trunk kernel (isr_conv_chain variant 4, trunk_deep.hip):
one geometry per call, chain vs per-conv launches bitwise, with give-up detection.
usage: python tools/r04_deep_first.py N H W BLOCKS [VARIANT]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402


def main():
    n, h, w, blocks = (int(v) for v in sys.argv[1:5])
    variant = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(blocks, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
    xs = [normalize(synth_lr_batch(n, h, w, seed=3 + i, scale=4)[0]).to(dev).contiguous() for i in range(2)]
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    ref_plan = engine.GeneratorPlan(gw, n, h, w, dev, False, False, mean, std, chain=False)
    old = engine.CHAIN_VARIANT
    engine.CHAIN_VARIANT = variant
    plan = engine.GeneratorPlan(gw, n, h, w, dev, False, False, mean, std, chain=True)
    engine.CHAIN_VARIANT = old
    assert plan.chain is not None and plan.chain.variant == variant, "no chain"
    ok = True
    for x in xs:
        ref = torch.empty(ref_plan.out_shape, device=dev)
        out = torch.empty(plan.out_shape, device=dev)
        ref_plan.run(x, ref)
        plan.run(x, out)
        torch.cuda.synchronize()
        gen, fail, cnt = plan.chain.state[:3].tolist()
        same = torch.equal(out, ref)
        d = (out - ref).abs().max().item()
        print(f"n={n} h={h} w={w} blocks={blocks} v={variant}: gen={gen} fail={fail} gaveup_count={cnt} "
              f"bitwise={same} maxdiff={d:.3e}", flush=True)
        ok = ok and same and fail != gen
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
