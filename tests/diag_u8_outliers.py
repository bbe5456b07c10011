"""Where the > 1 LSB pixels of test_gpu_trained.py::test_trained_u8_model lie.

GPU diagnostic, not collected by pytest (test infrastructure: it imports the oracle).  Same case as
the test: the committed trained ResNet(16, 0.2, x4), 2 held-out dead-leaves tiles downscaled to
128² uint8, the uint8 `Model` wrapper (fused BN, Normalize in the head, TanhToArrayImage in the
tail) against the oracle's model_u8 (utils/models.py:723-751).  For every pixel off by 2 or more
it reports the position (image border distance, trunk-tile / output-tile phase), both float
values before rounding and the float HIP path's value, so a systematic site (border rows, tile
edges, one channel, the quantiser) separates from the error tail of the bf16 network.

    python tests/diag_u8_outliers.py [--tiles 4] [--out gpurun_out/u8_outliers.json]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from image_super_resolution_amd import checkpoint, models  # noqa: E402
from image_super_resolution_amd.weights import heldout_tiles  # noqa: E402
from oracle import ref_cpu as R  # noqa: E402

WEIGHTS = ROOT / "tests" / "golden" / "trained_resnet_x4.safetensors"


@torch.no_grad()
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=4)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "u8_outliers.json"))
    a = ap.parse_args()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    sd = checkpoint.load_module_state(WEIGHTS)
    _, hr = heldout_tiles(a.tiles, 128, 4, device="cuda")
    img = (hr * 255).round().to(torch.uint8)
    img = F.interpolate(img.float(), size=(128, 128), mode="bilinear", align_corners=False)
    img = (img + 0.5).floor().clamp(0, 255).to(torch.uint8)

    net = models.ResNet(16, 0.2, scaleRate=4)
    net.load_state_dict(sd)
    wrapped = models.Model(net)
    wrapped.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    wrapped = wrapped.eval().fuse().to("cuda")
    hip_u8 = wrapped(img.to("cuda")).cpu()
    # the float HIP path on the same normalised input (unfused module: BN folded at pack time)
    net2 = models.ResNet(16, 0.2, scaleRate=4)
    net2.load_state_dict(sd)
    net2 = net2.eval().to("cuda")
    x = R.normalize_u8(img)
    hip_f = net2(x.to("cuda")).float().cpu()

    fsd = R.fuse_state_dict(sd)
    ref_f = R.generator(fsd, x, num_blocks=16, scale=4)
    ref_u8 = R.tanh_to_u8(ref_f)
    pre = lambda t: (t + 1.0) / 2.0 * 255.0  # noqa: E731  the value TanhToArrayImage rounds

    d = (hip_u8.int() - ref_u8.int()).abs()
    dfl = (pre(hip_f) - pre(ref_f)).abs()  # float-path disagreement in LSB
    q = torch.tensor([0.5, 0.99, 0.999, 0.9999, 1.0], dtype=torch.float64)
    res = {"pixels": d.numel(), "n_diff_ge1": int((d >= 1).sum()), "n_diff_ge2": int((d >= 2).sum()),
           "float_path_disagreement_lsb_quantiles": dict(zip(["p50", "p99", "p999", "p9999", "max"],
                                                             [round(v, 4) for v in
                                                              torch.quantile(dfl.flatten().double()[::7], q).tolist()])),
           "u8_vs_float_hip_rounding_mismatch": int((hip_u8.int() != pre(hip_f).round().clamp(0, 255).int()).sum()),
           "outliers": []}
    H, W = ref_u8.shape[-2:]
    # HR gradient magnitude (edge strength) to see whether outliers sit on edges
    g = hr.mean(1, keepdim=True)
    gx = F.pad(g[..., :, 1:] - g[..., :, :-1], (0, 1)).abs()
    gy = F.pad(g[..., 1:, :] - g[..., :-1, :], (0, 0, 0, 1)).abs()
    edge = (gx + gy)[:, 0]
    for n, c, y, xx in (d >= 2).nonzero().tolist():
        res["outliers"].append({
            "tile": n, "ch": c, "y": y, "x": xx, "border_dist": min(y, xx, H - 1 - y, W - 1 - xx),
            "lr_phase_y": (y // 4) % 32, "lr_phase_x": (xx // 4) % 32,
            "hip_u8": int(hip_u8[n, c, y, xx]), "ref_u8": int(ref_u8[n, c, y, xx]),
            "ref_pre": round(float(pre(ref_f)[n, c, y, xx]), 4), "hip_float_pre": round(float(pre(hip_f)[n, c, y, xx]), 4),
            "hr_edge": round(float(edge[n, y, xx]), 4), "edge_p99": round(float(torch.quantile(edge.flatten()[::13], 0.99)), 4)})
    # where do 1-LSB differences concentrate? channel shares and border rows
    res["ge1_by_channel"] = [int((d[:, c] >= 1).sum()) for c in range(3)]
    res["ge1_within_8px_of_border"] = int((d[..., :8, :] >= 1).sum() + (d[..., -8:, :] >= 1).sum()
                                          + (d[..., 8:-8, :8] >= 1).sum() + (d[..., 8:-8, -8:] >= 1).sum())
    res["border_8px_share_of_pixels"] = round(1 - (H - 16) * (W - 16) / (H * W), 4)
    txt = json.dumps(res, indent=1)
    print(txt)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(txt + "\n")


if __name__ == "__main__":
    main()
