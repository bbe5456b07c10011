"""Host side of the fp16 inference storage (round 6), CPU only: the activation buffer's storage
type, the descriptors' f16 flag and the one-storage-type-per-launch rule (ops._same_storage), and
the chain's exactness test of the residual-fold scale in the storage type (engine._storage_exact).
The kernels themselves are tested on the GPU (tests/test_gpu_fp16.py)."""
import pytest
import torch

from image_super_resolution_amd import engine, ops

F16, BF16 = torch.float16, torch.bfloat16


def test_act_buffer_storage_type():
    a = ops.ActBuffer.alloc(1, 5, 7, 32, 1, "cpu", dtype=F16)
    assert a.t.dtype == F16 and a.f16 == 1 and (a.ha, a.wa) == (ops.round_up(5, ops.TILE_H), 32)
    assert ops.ActBuffer.alloc(1, 5, 7, 32, 1, "cpu").f16 == 0  # bf16 stays the default
    x = torch.randn(1, 32, 5, 7)
    a.set_nchw(x)
    assert a.t.dtype == F16 and torch.equal(a.to_nchw(), x.to(F16).float())
    assert a.outside_valid().abs().max().item() == 0.0
    with pytest.raises(TypeError):
        ops.ActBuffer.alloc(1, 5, 7, 32, 1, "cpu", dtype=torch.float32)


def test_conv_desc_takes_its_storage_from_the_launch():
    xh = ops.ActBuffer.alloc(1, 16, 32, 64, 1, "cpu", dtype=F16)
    yh = ops.ActBuffer.alloc(1, 16, 32, 64, 1, "cpu", dtype=F16)
    wh = torch.zeros(64 * 64 * 9, dtype=F16)
    assert ops.conv3x3_desc(xh, 64, wh, None, 64, yh).f16 == 1
    xb = ops.ActBuffer.alloc(1, 16, 32, 64, 1, "cpu")
    yb = ops.ActBuffer.alloc(1, 16, 32, 64, 1, "cpu")
    assert ops.conv3x3_desc(xb, 64, wh.to(BF16), None, 64, yb).f16 == 0
    for args in ((xb, wh, yb), (xh, wh.to(BF16), yh), (xh, wh, yb)):
        with pytest.raises(TypeError):
            ops.conv3x3_desc(args[0], 64, args[1], None, 64, args[2])
    with pytest.raises(TypeError):  # a residual of the other storage type
        ops.conv3x3_desc(xh, 64, wh, None, 64, yh, r1=xb, s1=0.2)


def test_fold_scale_exactness_per_storage_type():
    # add_rate 0.2 -> 1/s1 = 5: exact in both; 1/0.3 is in neither; 1/0.15 = 6.666.. likewise
    for f16 in (0, 1):
        assert engine._storage_exact(1 / 0.2, f16)
        assert not engine._storage_exact(1 / 0.3, f16)
    # 1 + 2^-9 has 9 mantissa bits: exact in fp16 (10), not in bf16 (7)
    v = 1 + 2 ** -9
    assert engine._storage_exact(v, 1) and not engine._storage_exact(v, 0)
