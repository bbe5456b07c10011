"""Host logic of the rs.py tiler (image_super_resolution_amd/tiler.py) on CPU:
window planning, stitching, halo semantics and the multi-rank tile deal.

The batch runner is injected (a deterministic uint8 operator), so these tests
pin the tiler against the oracle's restatement of the reference stitch
(oracle/ref_cpu.py:tiled_u8, rs.py:78-111) without needing a GPU; the HIP
generator runner is covered in test_gpu_parity.py."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from image_super_resolution_amd import tiler
from oracle import ref_cpu

S = 4


def box_up(x: torch.Tensor) -> torch.Tensor:
    """uint8 [b,3,h,w] → uint8 [b,3,4h,4w]: 3x3 zero-padded box sum (radius 1,
    so image-border semantics matter) then nearest x4 upsample."""
    xf = x.float()
    k = torch.ones(3, 1, 3, 3)
    y = torch.nn.functional.conv2d(xf, k, padding=1, groups=3) / 9.0
    y = y.round().clamp(0, 255).to(torch.uint8)
    return y.repeat_interleave(S, -2).repeat_interleave(S, -1)


def image(h, w, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (3, h, w), generator=g, dtype=torch.uint8)


@pytest.mark.parametrize("h,w,window", [(37, 53, 16), (16, 16, 16), (10, 70, 32), (64, 40, 96), (1, 1, 4)])
def test_plan_matches_sliding_window(h, w, window):
    img = image(h, w)
    ref = [(x, y, tuple(win.shape[-2:])) for _, x, y, win in ref_cpu.sliding_window(img, window)]
    got = [(t.x, t.y, (t.h, t.w)) for t in tiler.plan_tiles(h, w, window)]
    assert got == ref


@pytest.mark.parametrize("h,w,window,batch", [(37, 53, 16, 1), (37, 53, 16, 5), (64, 40, 96, 8), (33, 33, 8, 3)])
def test_halo0_matches_reference_stitch(h, w, window, batch):
    img = image(h, w, seed=h * w)
    ref = ref_cpu.tiled_u8(box_up, img, window)
    up = tiler.TileUpscaler(box_up, S, window=window, halo=0, batch=batch, device="cpu")
    assert torch.equal(up(img), ref)


@pytest.mark.parametrize("halo", [1, 3])
def test_halo_removes_seams(halo):
    """With halo >= the operator's receptive radius, tiled == whole-image run."""
    img = image(45, 61, seed=7)
    full = box_up(img[None])[0]
    up = tiler.TileUpscaler(box_up, S, window=16, halo=halo, batch=4, device="cpu")
    assert torch.equal(up(img), full)
    seams = tiler.TileUpscaler(box_up, S, window=16, halo=0, batch=4, device="cpu")(img)
    assert not torch.equal(seams, full)


def test_shard_lpt_balanced_and_complete():
    tiles = tiler.plan_tiles(2160, 3840, 512, 32)  # cfg4: 40 tiles
    assert len(tiles) == 40
    for world in (1, 2, 3, 8):
        shards = tiler.shard_tiles(tiles, world)
        assert sorted(t.index for s in shards for t in s) == list(range(40))
        loads = [sum(t.cost for t in s) for s in shards]
        assert max(loads) - min(loads) <= max(t.cost for t in tiles)


@pytest.mark.parametrize("h,w,world,halo,max_rows", [(2160, 3840, 8, 32, None), (45, 61, 2, 2, None),
                                                      (45, 61, 3, 1, 8), (5, 9, 8, 1, None), (100, 7, 4, 0, 12)])
def test_plan_bands_cover_and_shapes(h, w, world, halo, max_rows):
    """Bands cover every image row once, in order; every band has ONE input height (at least
    the halo of context on each side, clipped to the image), every band fits max_rows."""
    shards = tiler.plan_bands(h, w, world, halo, max_rows)
    assert len(shards) == world
    bands = [b for s in shards for b in s]
    assert [b.index for b in bands] == list(range(len(bands)))
    rows = [r for b in bands for r in range(b.y, b.y + b.h)]
    assert rows == list(range(h))
    for b in bands:
        assert (b.x, b.w, b.x0, b.x1) == (0, w, 0, w)
        assert b.y0 <= max(0, b.y - halo) and b.y1 >= min(h, b.y + b.h + halo)
        assert 0 <= b.y0 and b.y1 <= h
        if max_rows is not None and b.h > 1:
            assert b.y1 - b.y0 <= max_rows
    assert len({b.in_shape for b in bands}) == 1


def test_plan_bands_cfg4_one_plan_per_rank():
    """cfg4 (3840x2160, halo 32) over 8 ranks: one band per rank (270 core rows), ONE input
    shape in all (334 rows: the edge bands take 32 more rows of context from the interior side),
    below the trunk kernel's 2 GiB window."""
    shards = tiler.plan_bands(2160, 3840, 8, 32)
    assert [len(s) for s in shards] == [1] * 8
    assert {s[0].in_shape for s in shards} == {(334, 3840)}
    assert tiler.band_max_rows(3840) >= 334
    assert 192 * 2 * (336 + 2) * (3840 + 2) < 2 ** 31


def test_bands_single_rank_equals_whole_image():
    """shard="bands" on one rank (as few full-width bands as the 2 GiB window allows; forced to
    several here by a small max_rows through plan_bands' default being large): with a halo of at
    least the operator's radius the canvas equals the whole-image run."""
    img = image(45, 61, seed=5)
    full = box_up(img[None])[0]
    up = tiler.TileUpscaler(box_up, S, window=16, halo=1, batch=1, device="cpu", shard="bands")
    assert len(up.shards(45, 61, 1)) == 1
    assert torch.equal(up(img), full)


@pytest.mark.parametrize("h,w,world,halo", [(2160, 3840, 8, 32), (2160, 3840, 1, 32), (45, 61, 2, 2),
                                             (45, 61, 3, 1), (5, 9, 8, 1), (100, 7, 4, 0)])
def test_plan_blocks_cover_and_halo(h, w, world, halo):
    """Blocks cover every LR pixel exactly once; each block's input is its core plus the halo on
    every side, clipped to the image; every block's 16-channel activation plane fits the trunk
    kernel's 2 GiB buffer-resource window."""
    shards = tiler.plan_blocks(h, w, world, halo)
    assert len(shards) == world and all(len(s) == len(shards[0]) for s in shards)
    cover = torch.zeros(h, w, dtype=torch.int32)
    for b in (b for s in shards for b in s):
        cover[b.y:b.y + b.h, b.x:b.x + b.w] += 1
        assert (b.y0, b.x0) == (max(0, b.y - halo), max(0, b.x - halo))
        assert (b.y1, b.x1) == (min(h, b.y + b.h + halo), min(w, b.x + b.w + halo))
        bh, bw = b.in_shape
        assert 16 * 2 * (-(-bh // 16) * 16 + 2) * (-(-bw // 32) * 32 + 2) < 2 ** 31  # one 16-channel plane
    assert bool((cover == 1).all())


def test_plan_blocks_cfg4_beats_bands():
    """cfg4 over 8 ranks: a 2 x 4 grid, one block per rank, at most 1112 x 1024 LR input — the
    busiest rank runs 1.11x its ideal share against 1.24x for the 334-row bands."""
    shards = tiler.plan_blocks(2160, 3840, 8, 32)
    assert [len(s) for s in shards] == [1] * 8
    shapes = {s[0].in_shape for s in shards}
    assert shapes == {(1112, 992), (1112, 1024)}
    band = tiler.plan_bands(2160, 3840, 8, 32)[0][0].in_shape
    assert max(a * b for a, b in shapes) < 0.9 * band[0] * band[1]


def test_blocks_single_rank_equals_whole_image_host_gather():
    img = image(45, 61, seed=5)
    full = box_up(img[None])[0]
    up = tiler.TileUpscaler(box_up, S, window=16, halo=1, batch=1, device="cpu", shard="blocks", gather="host")
    assert torch.equal(up(img), full)


def test_plan_memory_bound_cfg4():
    """blocks / bands are sized by the device memory one forward needs, not only by the
    trunk kernel's 2 GiB plane window (which lets the whole 4K still through as one ~31 GiB forward)."""
    whole = tiler.forward_bytes(1, 2160, 3840, 2)
    assert 30 << 30 < whole < 34 << 30  # the measured cfg4 peak is 31.5 GiB
    assert len(tiler.plan_blocks(2160, 3840, 1, 32)[0]) == 1
    limit = 12 << 30
    blocks = tiler.plan_blocks(2160, 3840, 1, 32, mem_limit=limit, n_scalers=2)[0]
    assert len(blocks) > 1 and all(tiler.forward_bytes(1, *t.in_shape, 2) <= limit for t in blocks)
    bands = tiler.plan_bands(2160, 3840, 1, 32, mem_limit=limit, n_scalers=2)[0]
    assert len(bands) > 1 and all(tiler.forward_bytes(1, *t.in_shape, 2) <= limit for t in bands)
    covered = sorted((t.y, t.h) for t in bands)
    assert covered[0][0] == 0 and sum(h for _, h in covered) == 2160


def test_batch_capped_by_memory_budget():
    """run_tiles puts no more tiles of one shape into a forward than fit the budget."""
    seen = []

    def rec(x):
        seen.append(x.shape[0])
        return box_up(x)

    budget = 2 * tiler.forward_bytes(1, 16, 16, 2) + 1
    up = tiler.TileUpscaler(rec, S, window=16, halo=0, batch=8, device="cpu", mem_budget=budget)
    img = image(64, 64, seed=5)
    assert torch.equal(up(img), tiler.TileUpscaler(box_up, S, window=16, halo=0, batch=1, device="cpu")(img))
    assert max(seen) == 2 and sum(seen) == 16


def test_runner_shape_check():
    up = tiler.TileUpscaler(lambda x: x, S, window=8, device="cpu")
    with pytest.raises(RuntimeError, match="runner returned"):
        up(image(8, 8))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, shard="windows", gather="device"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        img = image(45, 61, seed=11)
        batch = 2 if shard == "windows" else 1
        up = tiler.TileUpscaler(box_up, S, window=16, halo=2, batch=batch, device="cpu", shard=shard,
                                gather=gather)
        out = up(img, rank=rank, world=world)
        if rank == 0:
            q.put(out.numpy())  # by value: a shared-memory tensor handle can vanish when this rank exits
        else:
            q.put(out is None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shard,gather", [("windows", "device"), ("bands", "device"), ("blocks", "device"),
                                          ("blocks", "host")])
def test_sharded_gloo_world2_matches_single(shard, gather):
    """2 ranks over gloo: the canvas rank 0 stitches equals the single-rank one (halo 2 >= the
    operator's radius, so the bands / blocks deals give the same whole-image result as windows),
    gathered point to point or through the shared host canvas."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, shard, gather)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    canvas = torch.from_numpy(next(r for r in res if not isinstance(r, bool)))
    assert any(r is True for r in res)
    img = image(45, 61, seed=11)
    single = tiler.TileUpscaler(box_up, S, window=16, halo=2, batch=2, device="cpu")(img)
    assert torch.equal(canvas, single)
