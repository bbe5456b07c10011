"""cfg5 at its own size (BASELINE.json configs[4]: 1080p → 4K, the rs.py video branch
rs.py:54-76 on the RRDB generator): ResNet(16, 0.2) x2, batch 1, uint8 in / out through
video.FrameUpscaler.  At 1080x1920 the trunk kernel deals 4,080 tiles over its resident
workgroups (8 per workgroup per layer), the HIP graph captures the whole forward and the
activation planes are ~67 MB each — the geometry the small video tests never reach.

Weights and frame (parity that bites): the committed TRAINED ResNet(16, 0.2, x2)
(tests/golden/trained_resnet_x2.safetensors: tools/train_weights.py --scale 2, 6,000 steps of
train.py --resnet on 256² dead-leaves crops; 35.6 dB vs HR on held-out tiles against 28.4 dB for
bicubic, profiles/r06_train_weights_x2.json) on a 1080p frame of its data distribution
(weights.heldout_still: a dead-leaves mosaic at 3840x2160, downscaled as train.py does).

(i)  graph replay == eager chained plan == per-conv plan (chain=False), bit for bit;
(ii) a 256x384 crop of the same frame through the HIP path vs the fp32 oracle
     (oracle.ref_cpu, Model(net).init_normalize + fuse, utils/models.py:723-751) against the HR
     crop: |dPSNR| <= 0.01 dB (and on luma) on the generator's float output, the uint8 frame within
     the rounding allowance and LSB distribution of tests/parity_bars.py, the model beats bicubic;
     < 1 % of the output pixels at 0 / 255."""
import pytest
import torch
import torch.nn.functional as F

from image_super_resolution_amd import checkpoint, engine, models, tiler, video
from image_super_resolution_amd.weights import heldout_still
from oracle import ref_cpu as R
from parity_bars import float_dpsnr, u8_bars

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, W = 1080, 1920
MEAN, STD = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
WEIGHTS = __import__("pathlib").Path(__file__).parent / "golden" / "trained_resnet_x2.safetensors"


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


@torch.no_grad()
def test_1080p_graph_eager_perconv_bitwise_and_crop_vs_oracle():
    net = models.ResNet(16, 0.2, scaleRate=2)
    sd = {k: v.float() for k, v in checkpoint.load_module_state(WEIGHTS).items()}
    net.load_state_dict(sd)
    m = models.Model(net.eval())
    m.init_normalize(MEAN, STD)
    runner = tiler.runner_for(m.fuse().eval().to(DEV), DEV)
    gw = runner.gw

    up = video.FrameUpscaler(gw, H, W, 1, runner.mean, runner.std, DEV)
    assert up.plan.chains, "the 1080p video plan must run the trunk on the persistent chain"
    lr, hr = heldout_still(H, W, 2, device=DEV)
    x_hwc = lr.permute(1, 2, 0).contiguous()[None]
    got = up(x_hwc).cpu()[0]                             # graph replay, BGR HWC
    assert tuple(got.shape) == (2 * H, 2 * W, 3)

    x = x_hwc.permute(0, 3, 1, 2).contiguous().to(DEV)
    outs = {}
    for chain in (True, False):
        plan = engine.GeneratorPlan(gw, 1, H, W, torch.device(DEV), True, True, runner.mean, runner.std, chain=chain)
        assert (plan.chain is not None) == chain
        y = torch.empty(plan.out_shape, dtype=torch.uint8, device=DEV)
        plan.run(x, y)
        plan.verify()
        outs[chain] = y[0].cpu()
        del plan
    torch.cuda.empty_cache()
    graph_rgb = got.flip(-1).permute(2, 0, 1)
    assert torch.equal(graph_rgb, outs[True]), "graph replay differs from the eager chained forward"
    assert torch.equal(outs[True], outs[False]), "chained trunk differs from the per-conv launches"

    sat = ((graph_rgb == 0) | (graph_rgb == 255)).float().mean().item()
    print(f"1080p frame: {sat * 100:.3f} % of output pixels at 0 / 255")
    assert sat < 0.01, sat

    # a crop of the same frame vs the fp32 oracle (the full frame would take the CPU minutes)
    y0, x0, ch, cw = 400, 800, 256, 384
    crop = x[:, :, y0:y0 + ch, x0:x0 + cw].contiguous()
    hip = runner(crop).cpu()[0]
    xin = R.normalize_u8(crop.cpu())
    ref_f = R.generator(R.fuse_state_dict(sd), xin, num_blocks=16, scale=2)
    ref = R.tanh_to_u8(ref_f)[0]
    hr_c = hr[:, 2 * y0:2 * (y0 + ch), 2 * x0:2 * (x0 + cw)]
    yf = net.to(DEV).eval()(xin.to(DEV)).float().cpu()  # the float output the uint8 path rounds
    p_ref, _, _ = float_dpsnr(yf[0], ref_f[0], hr_c.float() / 255.0, "1080p crop 256x384")
    u8_bars(hip, ref, hr_c, "1080p crop 256x384")
    bic = F.interpolate(crop.cpu().float() / 255.0, scale_factor=2, mode="bicubic", align_corners=False).clamp(0, 1)[0]
    p_bic = R.psnr(bic * 2 - 1, hr_c.float() / 127.5 - 1)
    print(f"1080p crop: oracle {p_ref:.3f} dB vs bicubic {p_bic:.3f} dB")
    assert p_ref > p_bic + 0.3, (p_ref, p_bic)
