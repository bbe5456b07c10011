"""Host-side checks of the training data transforms (no GPU: torch ops on the CPU
device).  GPUTransform mirrors SR_dataset (utils/datasets.py:344-355);
NoisyTransform mirrors Noisy_dataset's GaussNoise (utils/datasets.py:361-389)."""
import torch

from image_super_resolution_amd import data


def test_noisy_transform_statistics():
    t = data.NoisyTransform(device="cpu", seed=3)
    crops = torch.full((64, 3, 16, 16), 128, dtype=torch.uint8)
    hr, lr = t(crops)
    assert hr.shape == lr.shape == (64, 3, 16, 16)
    torch.testing.assert_close(hr, torch.full_like(hr, 128 / 255 * 2 - 1))
    mean = torch.tensor(data.IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(data.IMAGENET_STD).view(1, 3, 1, 1)
    noisy255 = (lr * std + mean) * 255
    dev = (noisy255 - 128).flatten(1)
    clean = dev.abs().amax(1) < 1e-3
    # p = 0.5 per sample: some samples untouched, the rest with sigma in [sqrt(10), sqrt(50)]
    assert 10 <= int(clean.sum()) <= 54
    sig = dev[~clean].std(1)
    assert bool((sig > 10 ** 0.5 * 0.8).all()) and bool((sig < 50 ** 0.5 * 1.2).all())


def test_noisy_transform_clips_to_pixel_range():
    t = data.NoisyTransform(device="cpu", seed=4, p=1.0)
    crops = torch.cat([torch.zeros(4, 3, 8, 8), torch.full((4, 3, 8, 8), 255.0)]).to(torch.uint8)
    _, lr = t(crops)
    mean = torch.tensor(data.IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(data.IMAGENET_STD).view(1, 3, 1, 1)
    px = (lr * std + mean) * 255
    assert float(px.min()) >= -1e-3 and float(px.max()) <= 255 + 1e-3


def test_gpu_transform_shapes_cpu():
    t = data.GPUTransform(2, device="cpu")
    hr, lr = t(torch.randint(0, 256, (2, 3, 32, 32), dtype=torch.uint8))
    assert hr.shape == (2, 3, 32, 32) and lr.shape == (2, 3, 16, 16)
    assert float(hr.min()) >= -1 and float(hr.max()) <= 1
