"""Diagnostic: HIP TruncatedVGG19 input gradient vs fp32 autograd, per truncation depth."""
import sys
import warnings
from pathlib import Path

import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import vgg  # noqa: E402

warnings.simplefilter("ignore")
torch.manual_seed(0)
for (i, j, ba) in [(1, 1, True), (1, 2, True), (1, 2, False), (2, 1, True), (2, 1, False), (3, 1, False), (5, 4, False)]:
    for hw in (32, 64):
        m = vgg.TruncatedVGG19(i, j, ba).cuda()
        x = torch.randn(2, 3, hw, hw, device="cuda")
        with torch.no_grad():
            for p in m.parameters():
                p.copy_(p.to(torch.bfloat16).float())
        xb = x.to(torch.bfloat16).float().requires_grad_(True)
        ref = m.truncated_vgg19(xb)
        g = torch.randn_like(ref)
        ref.backward(g)
        xx = xb.detach().clone().requires_grad_(True)
        out = m(xx)
        out.backward(g)
        rel_f = ((out - ref).norm() / ref.norm()).item()
        rel_g = ((xx.grad - xb.grad).norm() / xb.grad.norm()).item()
        cos = F.cosine_similarity(xx.grad.flatten(), xb.grad.flatten(), dim=0).item()
        print(f"i={i} j={j} before_act={ba} hw={hw}: feat rel {rel_f:.3e}  grad rel {rel_g:.3e} cos {cos:.5f}", flush=True)
