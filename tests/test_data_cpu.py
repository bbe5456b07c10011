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


def test_gpu_transform_lr_matches_cv2_linear_u8():
    """LR = Normalize(uint8 cv2 INTER_LINEAR resize) of SR_dataset (utils/datasets.py:302-304):
    GPUTransform (run on the CPU device) vs the oracle's restatement of OpenCV's fixed-point
    uint8 resize at the integer factors train.py uses; HR = PIL_to_tanh (:96-106) or
    Normalize (set_transform_hr, :336-339).  cv2 itself is absent: parity unpinned."""
    import numpy as np
    from oracle import ref_cpu
    g = torch.Generator().manual_seed(7)
    crops = torch.randint(0, 256, (3, 3, 48, 48), generator=g, dtype=torch.uint8)
    mean = np.array(data.IMAGENET_MEAN, dtype=np.float32).reshape(1, 3, 1, 1)
    std = np.array(data.IMAGENET_STD, dtype=np.float32).reshape(1, 3, 1, 1)
    for scale in (2, 3, 4):
        for hr_norm in (False, True):
            hr, lr = data.GPUTransform(scale, hr_norm=hr_norm, device="cpu")(crops)
            lr_u8 = ref_cpu.cv2_resize_linear_u8(crops.numpy(), scale)
            ref_lr = (lr_u8.astype(np.float32) - mean * 255.0) * (1.0 / (std * 255.0))  # albumentations Normalize
            assert lr.shape == (3, 3, 48 // scale, 48 // scale)
            np.testing.assert_allclose(lr.numpy(), ref_lr, rtol=0, atol=2e-6)
            x = crops.numpy().astype(np.float32)
            ref_hr = (x / 255.0 - mean) / std if hr_norm else 2.0 * (x / 255.0) - 1.0
            np.testing.assert_allclose(hr.numpy(), ref_hr, rtol=0, atol=2e-6)


def test_heldout_tiles_do_not_depend_on_n():
    """The trained-weight parity bar (tests/test_gpu_trained.py, bench.py parity) draws tile i from
    its own generator, so the first tiles of a longer draw are the same tiles bit for bit."""
    from image_super_resolution_amd.weights import heldout_tiles
    lr2, hr2 = heldout_tiles(2, lr_size=32, scale=4)
    lr3, hr3 = heldout_tiles(3, lr_size=32, scale=4)
    assert lr2.shape == (2, 3, 32, 32) and hr2.shape == (2, 3, 128, 128)
    assert torch.equal(lr2, lr3[:2]) and torch.equal(hr2, hr3[:2])
    assert not torch.equal(hr3[1], hr3[2])  # distinct tiles
    # HR is uint8-exact in [0, 1]; LR is the rounded bilinear resize of it, normalised
    assert torch.equal((hr3 * 255).round() / 255, hr3)


def test_leaves_images_have_edges_and_full_range():
    """Dead-leaves crops (the trained weights' distribution): opaque discs give sharp edges (large
    neighbour differences on a few pixels) over a wide intensity range."""
    from image_super_resolution_amd.data import leaves_hr_u8
    x = leaves_hr_u8(2, 96, torch.Generator().manual_seed(5), device="cpu").float()
    assert x.dtype == torch.float32 and x.shape == (2, 3, 96, 96)
    assert x.min() < 40 and x.max() > 215
    d = (x[..., 1:] - x[..., :-1]).abs()
    assert (d > 60).float().mean() > 0.002  # edges
    assert (d < 8).float().mean() > 0.5     # mostly flat or smooth inside the discs
