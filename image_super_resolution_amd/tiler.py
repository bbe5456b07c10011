"""Tiled uint8 super-resolution of large stills — the rs.py image branch
(rs.py:16-27 `sliding_window`, rs.py:78-114 `runer` stitch), MI355X-first.

Differences from the reference loop, none of which change its output in the
halo=0 mode:

* tiles of the same shape are batched (the reference runs batch 1), each shape
  group through one pre-built `engine.GeneratorPlan` (uint8 in → uint8 out,
  Normalize and TanhToArrayImage fused into the 9x9 head / tail kernels);
* the image is uploaded once and tiles are cut on the GPU; the output canvas
  lives in HBM and is copied to the host once;
* tiles are pasted at (y·s, x·s).  For every image the reference's cursor
  (rs.py:105-111: `width += w`, wrap at `image_width`) lands on exactly those
  coordinates, because the windows of one row sum to the image width;
* optional `halo` (cfg4: 32 px): each window is extended by `halo` LR pixels on
  every side (clipped to the image, so the network still sees its own zero
  padding at the true image border), run, and the core is cropped back out.
  This removes the seams of the reference's halo-less stitching;
* multi-GPU: tiles are dealt longest-processing-time-first
  across ranks, no collective on the data path; rank 0 receives the finished
  output tiles point-to-point.
"""
from __future__ import annotations

import heapq
import os
import warnings
from collections import defaultdict
from dataclasses import dataclass
from typing import Callable, Sequence

import torch

from . import engine


@dataclass(frozen=True)
class Tile:
    """One rs.py window.  (y, x, h, w): the core window in LR pixels, as
    `sliding_window` yields it; (y0, x0, y1, x1): the input region actually run
    (core + halo, clipped to the image)."""
    index: int
    y: int
    x: int
    h: int
    w: int
    y0: int
    x0: int
    y1: int
    x1: int

    @property
    def in_shape(self) -> tuple[int, int]:
        return self.y1 - self.y0, self.x1 - self.x0

    @property
    def cost(self) -> int:
        return (self.y1 - self.y0) * (self.x1 - self.x0)


def plan_tiles(height: int, width: int, window: int, halo: int = 0) -> list[Tile]:
    """Windows in the reference's raster order (rs.py:16-27): step = window
    clamped to the image, the last row/column ragged."""
    if window <= 0 or halo < 0:
        raise ValueError("window must be > 0 and halo >= 0")
    sy, sx = min(height, window), min(width, window)
    tiles = []
    for y in range(0, height, sy):
        for x in range(0, width, sx):
            h, w = min(window, height - y), min(window, width - x)
            tiles.append(Tile(len(tiles), y, x, h, w, max(0, y - halo), max(0, x - halo),
                              min(height, y + h + halo), min(width, x + w + halo)))
    return tiles


def shard_tiles(tiles: Sequence[Tile], world: int) -> list[list[Tile]]:
    """Longest-processing-time-first deal of tiles over `world` ranks
    (SURVEY.md §8e): biggest tile to the least-loaded rank.  Deterministic, so
    every rank computes the same assignment without communicating."""
    heap = [(0, r) for r in range(world)]
    out: list[list[Tile]] = [[] for _ in range(world)]
    for t in sorted(tiles, key=lambda t: (-t.cost, t.index)):
        load, r = heapq.heappop(heap)
        out[r].append(t)
        heapq.heappush(heap, (load + t.cost, r))
    for lst in out:
        lst.sort(key=lambda t: t.index)
    return out


def plan_bands(height: int, width: int, world: int, halo: int, max_rows: int | None = None,
               mem_limit: int | None = None, n_scalers: int = 2) -> list[list[Tile]]:
    """Multi-GPU deal of a still as horizontal bands: the image
    splits into `world` x k full-width bands of equal core height (the last one ragged), each
    extended by `halo` LR rows above and below (clipped to the image, like a window's halo);
    rank r takes the k contiguous bands [r k, (r + 1) k).  k is the smallest count that keeps a
    band's input within `max_rows` (the persistent trunk kernel's 2 GiB window per 16-channel
    plane by default, see band_max_rows).  EVERY band has the same input height, min(height, core +
    2 halo): an image-edge band (halo clipped at the edge) or the ragged last band extends its
    input further into the image instead (more context than the halo asks, never less), so a
    rank builds ONE plan for all its bands and runs each as one batch-1 forward over the full
    width — instead of the 3-4 window shapes at batch 1-2 an LPT deal of rs.py windows gives
    it, and with no vertical seams.  `mem_limit` (bytes) also bounds a band so that one batch-1
    forward over it (forward_bytes) fits the device memory the caller has.  Returns per-rank Tile
    lists (Tile.x = 0, Tile.w = width)."""
    if world < 1 or halo < 0 or height < 1 or width < 1:
        raise ValueError("plan_bands: world >= 1, halo >= 0 and a non-empty image required")
    if max_rows is None:
        max_rows = band_max_rows(width)
    if mem_limit is not None:
        from .ops import TILE_H
        while max_rows > TILE_H and forward_bytes(1, max_rows, width, n_scalers) > mem_limit:
            max_rows -= TILE_H
    k = 1
    while True:
        core = -(-height // (world * k))
        if core + 2 * halo <= max_rows or core == 1:
            break
        k += 1
    rows = min(height, core + 2 * halo)  # the one input height of every band
    bands: list[Tile] = []
    for y in range(0, height, core):
        h = min(core, height - y)
        y0 = min(max(0, y - halo), height - rows)
        bands.append(Tile(len(bands), y, 0, h, width, y0, 0, y0 + rows, width))
    out: list[list[Tile]] = [[] for _ in range(world)]
    per = -(-len(bands) // world)
    for b in bands:
        out[min(world - 1, b.index // per)].append(b)
    return out


def plan_blocks(height: int, width: int, world: int, halo: int, limit: int = 2 ** 31,
                mem_limit: int | None = None, n_scalers: int = 2) -> list[list[Tile]]:
    """Multi-GPU deal of a still as a 2-D grid of blocks: gr x gc = world x k
    blocks of equal core (split evenly: cores differ by at most one pixel), each extended by `halo` LR pixels on every
    side and clipped at the image edge (a true image edge is the network's own zero padding, so
    clipping loses no context the whole-image forward has); rank r takes blocks [r k, (r + 1) k)
    in raster order.  k is the smallest count whose blocks fit the trunk kernel's 2 GiB window per
    16-channel plane (any still up to ~8K x 8K LR fits whole: k = 1); among the grids of that count the one with the least work on the busiest rank wins
    (work = the blocks' tile-aligned LR area, what the trunk kernel computes); with `mem_limit`
    (bytes) a block must also fit one batch-1 forward in that much device memory (forward_bytes:
    ~4 KB per LR pixel at x4), so a still larger than the GPU's free memory splits into more blocks
    instead of failing to allocate.  Full-width bands
    are the gc = 1 member of this family; at cfg4 over 8 ranks the 2 x 4 grid puts 1.14 M LR px
    on the busiest rank against 1.29 M for the 334-row bands (halo 32: 8 % vs 24 % overhead).
    Returns per-rank Tile lists (raster order inside a rank)."""
    from .ops import TILE_H, TILE_W, round_up
    if world < 1 or halo < 0 or height < 1 or width < 1:
        raise ValueError("plan_blocks: world >= 1, halo >= 0 and a non-empty image required")

    def grid(gr: int, gc: int) -> list[Tile]:
        ys = [i * height // gr for i in range(gr + 1)]  # even split: cores differ by <= 1 pixel
        xs = [j * width // gc for j in range(gc + 1)]
        out = []
        for i in range(gr):
            for j in range(gc):
                y, x, h, w = ys[i], xs[j], ys[i + 1] - ys[i], xs[j + 1] - xs[j]
                out.append(Tile(len(out), y, x, h, w, max(0, y - halo), max(0, x - halo),
                                min(height, y + h + halo), min(width, x + w + halo)))
        return out

    def fits(t: Tile) -> bool:
        h, w = t.in_shape
        if mem_limit is not None and forward_bytes(1, h, w, n_scalers) > mem_limit:
            return False
        return 16 * 2 * (round_up(h, TILE_H) + 2) * (round_up(w, TILE_W) + 2) < limit

    k = 1
    while True:
        n = world * k
        best = None
        for gr in range(1, n + 1):
            if n % gr:
                continue
            gc = n // gr
            if gr > height or gc > width:
                continue
            blocks = grid(gr, gc)
            if not all(fits(t) for t in blocks):
                continue  # too big for the window
            work = max(sum(round_up(t.in_shape[0], TILE_H) * round_up(t.in_shape[1], TILE_W)
                           for t in blocks[r * k:(r + 1) * k]) for r in range(world))
            if best is None or work < best[0]:
                best = (work, blocks)
        if best is not None:
            blocks = best[1]
            return [blocks[r * k:(r + 1) * k] for r in range(world)]
        if n > height * width:
            raise ValueError("plan_blocks: no grid fits the buffer window")
        k += 1


def band_max_rows(width: int, limit: int = 2 ** 31) -> int:
    """Largest band input height whose 16-channel activation plane (engine.GeneratorBuffers:
    bf16, 16x32-rounded, 1-px border) stays below the trunk kernel's 2 GiB window (its buffer
    resources span one plane each)."""
    from .ops import TILE_H, TILE_W, round_up
    wa = round_up(width, TILE_W) + 2
    rows = limit // (16 * 2 * wa) - 2
    return max(TILE_H, rows // TILE_H * TILE_H - TILE_H)


BatchRunner = Callable[[torch.Tensor], torch.Tensor]  # uint8 [b,3,h,w] → uint8 [b,3,s·h,s·w]


def plan_bytes(n: int, h: int, w: int, n_scalers: int) -> int:
    """Device bytes of one generator plan's activation buffers (engine.GeneratorBuffers):
    feat + 3 dense 192-ch buffers at LR, one 64-ch buffer per PixelShuffle stage."""
    from .ops import TILE_H, TILE_W, round_up
    ha, wa = round_up(h, TILE_H), round_up(w, TILE_W)
    b = (64 + 3 * 192) * (ha + 2) * (wa + 2) * 2
    for s in range(n_scalers):
        ha, wa = 2 * ha, 2 * wa
        p = 4 if s == n_scalers - 1 else 1
        b += 64 * (ha + 2 * p) * (wa + 2 * p) * 2
    return n * b


def forward_bytes(n: int, h: int, w: int, n_scalers: int) -> int:
    """Device bytes one forward of an n x h x w uint8 batch needs: the plan's activation buffers
    (plan_bytes), the uint8 input and output, and the 8 MB-aligned slack of torch's allocator
    per buffer (about 4 KB per LR pixel at x4: cfg4's whole 2160 x 3840 still ~31 GiB)."""
    s2 = 4 ** n_scalers
    return plan_bytes(n, h, w, n_scalers) + n * 3 * h * w * (1 + s2) + 16 * (8 << 20)


def device_budget(device, reserve: float = 0.1) -> int | None:
    """Bytes a new forward may allocate on `device`: the device's free memory plus what torch's
    caching allocator holds unused, less `reserve` of the total (None off the GPU)."""
    device = torch.device(device)
    if device.type != "cuda":
        return None
    free, total = torch.cuda.mem_get_info(device)
    cached = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    return max(0, int(free + cached - reserve * total))


class GeneratorRunner:
    """uint8 batch runner on the HIP generator: one plan (engine.make_plan) per (b, h, w),
    kept in a least-recently-used cache bounded by `max_plans` and `max_bytes` (plan
    activation buffers; a 4 x 576² cfg4 plan is ~5 GB), so a still with many ragged
    tile shapes does not hold one full set of buffers per shape."""

    def __init__(self, gw: engine.GeneratorWeights, mean, std, device, max_plans: int = 16,
                 max_bytes: int = 32 << 30):
        from collections import OrderedDict
        self.gw, self.mean, self.std, self.device = gw, tuple(mean), tuple(std), torch.device(device)
        self.scale = 2 ** len(gw.scalers)
        self.max_plans, self.max_bytes = max(1, max_plans), max_bytes
        self.plans: "OrderedDict[tuple[int, int, int], object]" = OrderedDict()

    def cached_bytes(self) -> int:
        return sum(plan_bytes(n, h, w, len(self.gw.scalers)) for n, h, w in self.plans)

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if x.dtype != torch.uint8 or not x.is_cuda:
            raise ValueError("GeneratorRunner expects a uint8 CUDA batch")
        n, _, h, w = x.shape
        key = (n, h, w)
        plan = self.plans.get(key)
        if plan is None:
            need = plan_bytes(n, h, w, len(self.gw.scalers))
            while self.plans and (len(self.plans) >= self.max_plans or self.cached_bytes() + need > self.max_bytes):
                self.plans.popitem(last=False)  # evict least recently used (its buffers return to torch's pool)
            plan = engine.make_plan(self.gw, n, h, w, self.device, True, True, self.mean, self.std)
            self.plans[key] = plan
        else:
            self.plans.move_to_end(key)
        out = torch.empty(plan.out_shape, dtype=torch.uint8, device=self.device)
        return plan.run(x.contiguous(), out)

    def verify(self) -> None:
        """Blocking persistent-chain give-up check of every forward issued so far (engine.ChainFailed)."""
        for plan in self.plans.values():
            plan.verify()

    def free(self):
        self.plans.clear()


def runner_for(model, device) -> GeneratorRunner:
    """Build the HIP runner from the drop-in modules: a `Model` wrapper with
    `init_normalize` (uint8 I/O), or a bare ResNet/EResNet/SRGAN generator with
    ImageNet normalisation (utils/datasets.py:53 defaults)."""
    from . import models
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    net = model
    if isinstance(model, models.Model):
        net = model.net
        if isinstance(net, torch.nn.Sequential) and len(net) == 3 and isinstance(net[0], models.Normalize):
            mean = tuple(net[0].mean.flatten().tolist())
            std = tuple(net[0].std.flatten().tolist())
            net = net[1]
    if isinstance(net, models.SRGAN):
        net = net.res_net
    if not isinstance(net, models._Generator):
        raise TypeError(f"tiled inference needs a ResNet/EResNet/SRGAN generator, got {type(net).__name__}")
    return GeneratorRunner(net._packed(torch.device(device)), mean, std, device)


class TileUpscaler:
    """rs.py image branch as a reusable object.

    `runner` maps uint8 [b,3,h,w] → uint8 [b,3,s·h,s·w] on `device` (the HIP
    GeneratorRunner in production).  `batch` tiles of one shape run together.
    """

    def __init__(self, runner: BatchRunner, scale: int, window: int = 96, halo: int = 0, batch: int = 8,
                 device="cuda", shard: str = "windows", gather: str = "device", mem_budget: int | None = None):
        """`shard`: "windows" runs rs.py's windows (dealt longest-processing-time-first over
        ranks, shard_tiles; the canvas equals the single-rank one bit for bit); "bands" runs
        full-width horizontal bands with the same halo (plan_bands: one rank's share is one or a
        few bands of one input shape, `batch` bands per forward; on one GPU the image splits into
        as few bands as the trunk kernel's 2 GiB window per activation plane allows (one, up to
        ~8K x 8K LR); needs halo > 0 to hide its seams, and differs from the windowed canvas by the
        seams each form leaves); "blocks" runs a 2-D grid of blocks with the same halo (plan_blocks:
        at cfg4 over 8 ranks 2 x 4 blocks, 8 % halo work instead of the bands' 24 %).
        `gather` (world > 1): "device" sends every finished tile to rank 0's device canvas point to
        point; "host" has every rank copy its tiles (device → pinned host) into one shared host canvas
        (a file in /dev/shm, all ranks on one node) that rank 0 returns as a CPU tensor — the
        still's output is written from host memory anyway (rs.py: cv2.imwrite), and the ranks' D2H
        copies run in parallel over their own links instead of one after another into rank 0.
        `mem_budget` (bytes; default: the device's free memory when the image arrives, device_budget)
        bounds every forward: bands / blocks are sized so that one fits, and a shape's `batch` is cut
        to as many tiles as fit together (forward_bytes) — ADVICE r5: the 2 GiB plane window alone
        would allow a ~250 GiB forward."""
        if batch < 1:
            raise ValueError("batch must be >= 1")
        if shard not in ("windows", "bands", "blocks"):
            raise ValueError(f"shard must be 'windows', 'bands' or 'blocks', got {shard!r}")
        if gather not in ("device", "host"):
            raise ValueError(f"gather must be 'device' or 'host', got {gather!r}")
        if shard != "windows" and halo == 0:
            warnings.warn(f"shard={shard!r} with halo=0: the seams are not hidden (pass halo > 0)", stacklevel=2)
        self.runner, self.scale, self.window, self.halo, self.batch = runner, scale, window, halo, batch
        self.device = torch.device(device)
        self.shard = shard
        self.gather = gather
        self.mem_budget = mem_budget
        self.n_scalers = max(0, int(scale).bit_length() - 1)

    def _budget(self) -> int | None:
        return self.mem_budget if self.mem_budget is not None else device_budget(self.device)

    def shards(self, height: int, width: int, world: int) -> list[list[Tile]]:
        """The per-rank tile lists of an image (deterministic: every rank computes the same)."""
        if self.shard == "bands":
            return plan_bands(height, width, world, self.halo, mem_limit=self._budget(), n_scalers=self.n_scalers)
        if self.shard == "blocks":
            return plan_blocks(height, width, world, self.halo, mem_limit=self._budget(), n_scalers=self.n_scalers)
        tiles = plan_tiles(height, width, self.window, self.halo)
        return shard_tiles(tiles, world) if world > 1 else [tiles]

    def run_tiles(self, image: torch.Tensor, tiles: Sequence[Tile]) -> dict[int, torch.Tensor]:
        """Upscale `tiles` of `image` (uint8 [3,H,W] on self.device); returns
        {tile.index: uint8 [3, s·h, s·w] core output} (views into batch outputs)."""
        s = self.scale
        groups: dict[tuple[int, int], list[Tile]] = defaultdict(list)
        for t in tiles:
            groups[t.in_shape].append(t)
        out: dict[int, torch.Tensor] = {}
        budget = self._budget()
        for (h, w), lst in groups.items():
            # windows, bands and blocks of one input shape share a batched forward, as many as fit
            step = self.batch
            if budget is not None:
                step = max(1, min(step, budget // max(1, forward_bytes(1, h, w, self.n_scalers))))
            for i in range(0, len(lst), step):
                chunk = lst[i:i + step]
                x = torch.stack([image[:, t.y0:t.y1, t.x0:t.x1] for t in chunk])
                y = self.runner(x)
                if tuple(y.shape) != (len(chunk), 3, h * s, w * s):
                    raise RuntimeError(f"runner returned {tuple(y.shape)} for a {len(chunk)}x3x{h}x{w} batch "
                                       f"at scale {s}")
                for j, t in enumerate(chunk):
                    oy, ox = (t.y - t.y0) * s, (t.x - t.x0) * s
                    out[t.index] = y[j, :, oy:oy + t.h * s, ox:ox + t.w * s]
        return out

    def __call__(self, image: torch.Tensor, rank: int = 0, world: int = 1, group=None) -> torch.Tensor | None:
        """Upscale a uint8 [3,H,W] image.  With world > 1 (torch.distributed
        initialised, every rank passing the same image), each rank runs its
        share of the tiles and rank 0 returns the stitched [3,s·H,s·W] uint8
        canvas (on self.device); other ranks return None."""
        if image.dim() != 3 or image.dtype != torch.uint8:
            raise ValueError("expected a uint8 CHW image")
        c, H, W = image.shape
        s = self.scale
        image = image.to(self.device, non_blocking=True)
        shards = self.shards(H, W, world)
        tiles = [t for lst in shards for t in lst]
        mine = shards[rank]
        done = self.run_tiles(image, mine)
        verify = getattr(self.runner, "verify", None)
        if verify is not None:
            verify()  # every forward of this image, the last included, before anything is stitched
        if self.gather == "host":
            return _gather_host(mine, done, s, (c, H * s, W * s), rank, world, group)
        if world == 1:
            canvas = torch.zeros((c, H * s, W * s), dtype=torch.uint8, device=self.device)
            for t in tiles:
                canvas[:, t.y * s:(t.y + t.h) * s, t.x * s:(t.x + t.w) * s] = done[t.index]
            return canvas
        return _gather_to_rank0(tiles, shards, done, s, (c, H * s, W * s), rank, group, self.device)


def copy_tiles_to_host(mine, done, s, canvas: torch.Tensor) -> None:
    """Device → host copy of a rank's finished tiles into the CPU `canvas` (through one pinned
    staging buffer per tile when the tiles live on a GPU; one synchronisation at the end)."""
    staged = []
    for t in mine:
        part = done[t.index]
        if part.is_cuda:
            pin = torch.empty(part.shape, dtype=part.dtype, pin_memory=True)
            pin.copy_(part, non_blocking=True)
            staged.append((t, pin))
        else:
            canvas[:, t.y * s:(t.y + t.h) * s, t.x * s:(t.x + t.w) * s] = part
    if staged:
        torch.cuda.synchronize(done[mine[0].index].device)
    for t, pin in staged:
        canvas[:, t.y * s:(t.y + t.h) * s, t.x * s:(t.x + t.w) * s] = pin


def _gather_host(mine, done, s, canvas_shape, rank, world, group):
    """gather="host": every rank writes its tiles into one shared host canvas (module doc of
    TileUpscaler.__init__); rank 0 returns it, the others None."""
    import numpy as np
    if world == 1:
        canvas = torch.zeros(canvas_shape, dtype=torch.uint8)
        copy_tiles_to_host(mine, done, s, canvas)
        return canvas
    import socket
    import tempfile
    import torch.distributed as dist
    # one shared /dev/shm canvas needs every rank on rank 0's node: refuse otherwise (every
    # rank gets the same verdict, so none is left waiting in a collective)
    hosts = [None] * world
    dist.all_gather_object(hosts, socket.gethostname(), group=group)
    if len(set(hosts)) != 1:
        raise RuntimeError(f"gather='host' needs every rank on one node (ranks on {sorted(set(hosts))}); "
                           "use gather='device'")
    name = [None]
    if rank == 0:
        fd, name[0] = tempfile.mkstemp(prefix="isr_canvas_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
        os.close(fd)
        np.memmap(name[0], dtype=np.uint8, mode="w+", shape=canvas_shape).flush()  # sized, zero-filled
    dist.broadcast_object_list(name, src=0, group=group)
    try:
        err = None
        try:
            mm = np.memmap(name[0], dtype=np.uint8, mode="r+", shape=canvas_shape)
            copy_tiles_to_host(mine, done, s, torch.from_numpy(mm))
        except Exception as e:  # reported to every rank below instead of leaving rank 0 waiting
            err = f"rank {rank}: {type(e).__name__}: {e}"
        errs = [None] * world
        dist.all_gather_object(errs, err, group=group)  # also the "every rank's tiles are in" barrier
        bad = [e for e in errs if e is not None]
        if bad:
            raise RuntimeError("gather='host' failed: " + "; ".join(bad))
        out = torch.from_numpy(mm) if rank == 0 else None  # rank 0 keeps the mapping (no copy)
    finally:
        if rank == 0:
            os.unlink(name[0])  # the name only: the mapping lives as long as the returned tensor
    return out


def _gather_to_rank0(tiles, shards, done, s, canvas_shape, rank, group, device):
    """Point-to-point collection of finished tiles on rank 0 (no data-path
    collective).  gloo needs host tensors, RCCL device ones."""
    import torch.distributed as dist
    comm_dev = torch.device("cpu") if dist.get_backend(group) == "gloo" else device
    if rank != 0:
        for t in shards[rank]:
            dist.send(done[t.index].contiguous().to(comm_dev), dst=0, group=group)
        return None
    canvas = torch.zeros(canvas_shape, dtype=torch.uint8, device=device)
    owner = {t.index: r for r, lst in enumerate(shards) for t in lst}
    for r, lst in enumerate(shards):
        for t in lst:
            if r == 0:
                part = done[t.index]
            else:
                part = torch.empty((canvas_shape[0], t.h * s, t.w * s), dtype=torch.uint8, device=comm_dev)
                dist.recv(part, src=owner[t.index], group=group)
            canvas[:, t.y * s:(t.y + t.h) * s, t.x * s:(t.x + t.w) * s] = part.to(device)
    return canvas
