"""Video path on the GPU (video.py): the HIP-graph-captured per-batch forward equals
the eager plan bit for bit and the uint8 oracle (utils/models.py Model) within
1 LSB; the streaming pipeline writes every frame, in order, incl. a ragged last batch."""
import numpy as np
import pytest
import torch

from image_super_resolution_amd import models, tiler, video
from image_super_resolution_amd.weights import synth_state_dict
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _setup(h=24, w=40, batch=2):
    net = models.ResNet(2, 0.2, scaleRate=2)
    sd = synth_state_dict(net.state_dict(), 11)
    net.load_state_dict(sd)
    m = models.Model(net.eval())
    m.init_normalize((0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
    runner = tiler.runner_for(m.fuse().eval().to(DEV), DEV)
    up = video.FrameUpscaler(runner.gw, h, w, batch, runner.mean, runner.std, DEV)
    return sd, runner, up


@torch.no_grad()
def test_graph_forward_matches_eager_and_oracle():
    sd, runner, up = _setup()
    frames = list(video.SyntheticVideo(40, 24, 2, seed=3))
    x = torch.from_numpy(np.stack(frames))
    got = up(x).cpu()                                    # BGR HWC
    eager = runner(x.permute(0, 3, 1, 2).contiguous().to(DEV)).cpu()   # RGB CHW
    assert torch.equal(got, eager.flip(1).permute(0, 2, 3, 1))
    ref = R.model_u8(sd, x.permute(0, 3, 1, 2).contiguous(), num_blocks=2, scale=2)
    d = (eager.int() - ref.int()).abs()
    psnr_u8 = 10 * np.log10(255.0 ** 2 / (d.float() ** 2).mean().item())
    # bf16 path vs fp32 oracle on noisy frames: >= 99 % of pixels within 1 LSB, >= 45 dB
    assert (d <= 1).float().mean() >= 0.99 and d.max() <= 4 and psnr_u8 >= 45.0, (d.max(), psnr_u8)
    # replaying again with other frames gives their result (static buffers re-read)
    x2 = torch.from_numpy(np.stack(list(video.SyntheticVideo(40, 24, 2, seed=9))))
    assert torch.equal(up(x2).cpu(), runner(x2.permute(0, 3, 1, 2).contiguous().to(DEV)).cpu().flip(1).permute(0, 2, 3, 1))


@torch.no_grad()
def test_pipeline_writes_all_frames_in_order(tmp_path):
    _, runner, up = _setup(batch=2)
    frames = list(video.SyntheticVideo(40, 24, 5, seed=4))
    rec = video.RawRecorder(tmp_path / "o.bgr", (80, 48), 30)
    n = video.VideoUpscaler(up).run(frames, rec)
    rec.stopRecorder()
    assert n == 5
    out = np.frombuffer((tmp_path / "o.bgr").read_bytes(), np.uint8).reshape(5, 48, 80, 3)
    for i, f in enumerate(frames):
        ref = runner(torch.from_numpy(f).permute(2, 0, 1)[None].contiguous().to(DEV)).cpu()[0]
        assert np.array_equal(out[i], ref.flip(0).permute(1, 2, 0).numpy()), f"frame {i}"
