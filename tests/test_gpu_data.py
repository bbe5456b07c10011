"""SR_dataset's transform on the GPU (utils/datasets.py:344-355):
data.GPUTransform on a CUDA device runs ONE HIP launch (isr_sr_transform) — the crop's
scale x scale blocks read once, cv2's uint8 INTER_LINEAR resize, both Normalizes.

Checked against oracle.ref_cpu.cv2_resize_linear_u8 (the restatement of OpenCV's
fixed-point uint8 resize; cv2 is absent here, so this parity is unpinned)
followed by albumentations' Normalize, and the HR tensor against the same formulas as
torch ops on the CPU device."""
import numpy as np
import pytest
import torch

from image_super_resolution_amd import data
from oracle import ref_cpu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


@pytest.mark.parametrize("scale", [2, 3, 4])
@pytest.mark.parametrize("hr_norm", [False, True])
def test_sr_transform_vs_cv2_oracle(scale, hr_norm):
    g = torch.Generator().manual_seed(11 + scale)
    t = 12 * scale * 4  # 96 / 144 / 192: ragged against the 256-thread blocks
    crops = torch.randint(0, 256, (5, 3, t, t), generator=g, dtype=torch.uint8)
    crops[0, :, :4, :4] = 255  # saturated corner and a flat zero one
    crops[1, :, -4:, -4:] = 0
    hr, lr = data.GPUTransform(scale, hr_norm=hr_norm, device="cuda")(crops.cuda())
    assert hr.is_cuda and hr.shape == (5, 3, t, t) and lr.shape == (5, 3, t // scale, t // scale)
    mean = np.array(data.IMAGENET_MEAN, dtype=np.float32).reshape(1, 3, 1, 1)
    std = np.array(data.IMAGENET_STD, dtype=np.float32).reshape(1, 3, 1, 1)
    lr_u8 = ref_cpu.cv2_resize_linear_u8(crops.numpy(), scale)
    ref_lr = (lr_u8.astype(np.float32) - mean * 255.0) * (1.0 / (std * 255.0))  # albumentations Normalize
    np.testing.assert_allclose(lr.cpu().numpy(), ref_lr, rtol=0, atol=2e-6)
    hr_cpu, lr_cpu = data.GPUTransform(scale, hr_norm=hr_norm, device="cpu")(crops)
    torch.testing.assert_close(hr.cpu(), hr_cpu, rtol=0, atol=1e-6)
    torch.testing.assert_close(lr.cpu(), lr_cpu, rtol=0, atol=1e-6)


def test_sr_transform_rejects_bad_batches():
    tf = data.GPUTransform(4, device="cuda")
    with pytest.raises(ValueError):
        tf(torch.zeros(2, 3, 30, 30, dtype=torch.uint8, device="cuda"))  # 30 % 4 != 0
    with pytest.raises(ValueError):
        tf(torch.zeros(2, 3, 32, 32, dtype=torch.float32, device="cuda"))


def test_sr_transform_cfg3_batch_rate():
    """cfg3's per-GPU batch (16 x 512^2 HR): the transform is a few tens of microseconds,
    negligible against the ~50 ms training step it feeds."""
    crops = torch.randint(0, 256, (16, 3, 512, 512), dtype=torch.uint8, device="cuda")
    tf = data.GPUTransform(4, hr_norm=True, device="cuda")
    for _ in range(3):
        tf(crops)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        tf(crops)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    moved = crops.numel() * (1 + 4) + crops.numel() // 16 * 4
    print(f"sr_transform 16x512^2: {ms * 1e3:.1f} us/batch = {moved / ms / 1e6:.0f} GB/s")
    assert ms < 2.0
