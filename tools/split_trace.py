#!/usr/bin/env python3
"""Run one SplitGeneratorPlan config a few times (for rocprofv3 --kernel-trace):
shows whether the sub-batch streams' kernels overlap in time."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import engine, models  # noqa: E402
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict  # noqa: E402

splits, stagger = int(sys.argv[1]), float(sys.argv[2])
dev = torch.device("cuda")
sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
lr, _ = synth_lr_batch(16, 128, 128, seed=1234)
x = normalize(lr).to(dev).contiguous()
mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
p = engine.SplitGeneratorPlan(gw, 16, 128, 128, dev, False, False, mean, std, splits=splits, stagger_us=stagger)
out = torch.empty(p.out_shape, device=dev)
for _ in range(4):
    p.run(x, out)
torch.cuda.synchronize()
print("sleep cycles/us", engine._SLEEP_CAL)
