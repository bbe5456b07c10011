"""End-to-end drop-in entry points on the GPU, in-process: train.py (pixel-loss
pre-training, then SRGAN mode resuming from its checkpoint, as the reference's
two-stage recipe train.py:141-163), then rs.py still-image tiling and the raw
video branch on the trained checkpoint."""
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def test_train_then_upscale(tmp_path):
    import rs
    import train
    from image_super_resolution_amd import checkpoint

    common = ["--synthetic", "--steps", "2", "--epochs", "1", "--batch_size", "2", "--shape", "64", "--rs_deep",
              "1", "--scale", "2", "--work_dir", str(tmp_path), "--save_name", "t"]
    train.main(train.parse(["--resnet"] + common))
    res_ck = tmp_path / "res_t_1_0.2.pt"
    assert res_ck.is_file()
    ck = checkpoint.load_checkpoint(res_ck)
    assert ck["epoch"] == 0 and len(ck["loss"]) == 2 and all(np.isfinite(ck["loss"]))
    train.main(train.parse(common))  # SRGAN mode, generator initialised from res_ck
    gen_ck = tmp_path / "gen_t_1_0.2.pt"
    assert gen_ck.is_file()

    # still image: 2x through 32-px windows (ragged edges), reference stitching
    from PIL import Image
    img = (np.random.default_rng(0).random((40, 56, 3)) * 255).astype(np.uint8)
    Image.fromarray(img).save(tmp_path / "in.png")
    kw = dict(model=str(gen_ck), src=str(tmp_path / "in.png"), save_dir=str(tmp_path / "out.png"), window_size=32,
              batch_size=2, worker=0, halo=0, add_rate=0.2, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225))
    rs.runer(**kw)
    out = np.asarray(Image.open(tmp_path / "out.png"))
    assert out.shape == (80, 112, 3) and out.dtype == np.uint8 and out.std() > 0
    # --shard bands on one GPU: with a halo covering the whole 40-row image the single band is the
    # whole-image forward, which the 64-px window run below also is
    rs.runer(**dict(kw, save_dir=str(tmp_path / "out_bands.png"), halo=40, shard="bands"))
    rs.runer(**dict(kw, save_dir=str(tmp_path / "out_whole.png"), window_size=64))
    assert np.array_equal(np.asarray(Image.open(tmp_path / "out_bands.png")),
                          np.asarray(Image.open(tmp_path / "out_whole.png")))

    # video: headerless rgb24 in → bgr24 out (no ffmpeg needed)
    frames = (np.random.default_rng(1).random((3, 24, 40, 3)) * 255).astype(np.uint8)
    (tmp_path / "clip.rgb").write_bytes(frames.tobytes())
    rs.runer(**dict(kw, src=str(tmp_path / "clip.rgb"), save_dir=str(tmp_path / "clip.bgr"), video_size="40x24",
                    fps=25.0, batch_size=2))
    vid = np.frombuffer((tmp_path / "clip.bgr").read_bytes(), np.uint8).reshape(3, 48, 80, 3)
    # frame 0 of the video equals the still-image path on that frame (same model, one window)
    Image.fromarray(frames[0]).save(tmp_path / "f0.png")
    rs.runer(**dict(kw, src=str(tmp_path / "f0.png"), save_dir=str(tmp_path / "f0_out.png"), window_size=64))
    still = np.asarray(Image.open(tmp_path / "f0_out.png"))
    assert np.array_equal(vid[0][..., ::-1], still)
    torch.cuda.synchronize()


def test_train_denoise_cli(tmp_path):
    """`train.py --train_denoise` (train.py:204-243): Denoise on libisr, MSE on
    synthetic noisy/clean pairs, checkpoint denoise_{save_name}_{rs_deep}_{add_rate}.pt,
    and a second run picks it up (the reference restarts at epoch 0 when the
    checkpoint holds no optimiser state, train.py:214-219)."""
    import train
    from image_super_resolution_amd import checkpoint, models

    common = ["--train_denoise", "--synthetic", "--steps", "6", "--batch_size", "2", "--shape", "48", "--rs_deep",
              "2", "--lr", "1e-3", "--work_dir", str(tmp_path), "--save_name", "d"]
    train.main(train.parse(common + ["--epochs", "1"]))
    ck_path = tmp_path / "denoise_d_2_0.2.pt"
    ck = checkpoint.load_checkpoint(ck_path)
    assert ck["epoch"] == 0 and ck["optimizer"] is None  # last epoch of the run: no optimiser state (reference)
    m = models.Denoise(2)
    m.load_state_dict({k: v.float() if v.is_floating_point() else v for k, v in ck["gen_net"].items()})
    assert int(m.conv1.bn.num_batches_tracked) == 6
    train.main(train.parse(common + ["--epochs", "2"]))
    ck2 = checkpoint.load_checkpoint(ck_path)
    assert ck2["epoch"] == 1
    # the trained denoiser runs through the inference plan
    y = m.eval().cuda()(torch.rand(1, 3, 32, 32, device="cuda") * 2 - 1)
    assert y.shape == (1, 3, 32, 32) and torch.isfinite(y).all()
