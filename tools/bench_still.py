#!/usr/bin/env python3
"""cfg4 benchmark (BASELINE.json configs[3]): a 3840x2160 uint8 still → 15360x8640
through the HIP tiler (rs.py image branch: 512-px windows, here with a 32-px halo),
ResNet(16, 0.2, x4) with synthetic weights, tiles batched per shape.

One process per GPU (torch.distributed.run for N > 1): tiles are dealt
longest-processing-time-first over the ranks (tiler.shard_tiles, no data-path
collective), rank 0 receives finished tiles point-to-point and owns the canvas.
Reports HR megapixels/s of the whole image (after one warm-up call that builds
the plans), seconds per image, and peak device memory.

--shard bands runs full-width bands (tiler.plan_bands) instead of rs.py's windows, on one GPU
too (as few bands as the 2 GiB trunk-buffer window allows); --shard blocks a 2-D grid of blocks
(tiler.plan_blocks: 2 x 4 at 8 ranks).
--sim-world N (one GPU, no torch.distributed): predicts the N-GPU wall time.  After the
1-GPU run (t1, with the same --shard), every rank's share of an N-rank deal runs alone on this
GPU, timed like the real run (same plans, median of --reps); the predicted N-GPU time is the
slowest rank's, reported against t1 / N.  Each rank's time includes the hand-off of its finished
tiles to the host: a device → pinned-host copy of its share of the canvas (1/N of it), as
tiler's gather="host" does before the host assembly (reported apart, "assemble_s").
usage: python tools/bench_still.py [--reps 3] [--batch 4] [--halo 32] [--shard bands] [--sim-world 8]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import models, tiler  # noqa: E402
from image_super_resolution_amd.weights import synth_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--window", type=int, default=512)
    ap.add_argument("--halo", type=int, default=32)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--shard", default="windows", choices=("windows", "bands", "blocks"))
    ap.add_argument("--sim-world", type=int, default=0)
    args = ap.parse_args()
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    net = models.ResNet(args.blocks, 0.2, scaleRate=4)
    net.load_state_dict(synth_state_dict(net.state_dict(), seed=4))
    model = models.Model(net)
    model.init_normalize([0.485, 0.456, 0.406], [0.229, 0.224, 0.225])
    model = model.eval().fuse().to(dev)
    g = torch.Generator().manual_seed(21)
    lo = torch.rand(1, 3, args.height // 32, args.width // 32, generator=g)
    img = torch.nn.functional.interpolate(lo, size=(args.height, args.width), mode="bicubic")
    img = (img.clamp(0, 1)[0] * 255).round().to(torch.uint8)
    runner = tiler.runner_for(model, dev)
    up = tiler.TileUpscaler(runner, 4, window=args.window, halo=args.halo, batch=args.batch, device=dev,
                            shard=args.shard)
    torch.cuda.reset_peak_memory_stats(dev)
    with torch.no_grad():
        t0 = time.perf_counter()
        up(img, rank=rank, world=world)  # warm-up: builds the plans
        torch.cuda.synchronize()
        warm = time.perf_counter() - t0
        ts = []
        for _ in range(args.reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            canvas = up(img, rank=rank, world=world)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            el = time.perf_counter() - t0
            if world > 1:
                tt = torch.tensor([el], device=dev, dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                el = tt.item()
            ts.append(el)
    t = statistics.median(ts)
    tiles = [tt for lst in up.shards(args.height, args.width, 1) for tt in lst]
    run_px = sum(tt.cost for tt in tiles) * 16
    res = {"metric": "cfg4 4K->16K still, HR MPix/s", "value": round(args.height * args.width * 16 / t / 1e6, 2),
           "unit": "MPix/s", "n_gpus": world, "s_per_image": round(t, 4), "s_first_call": round(warm, 3),
           "shard_1gpu": args.shard, "tiles": len(tiles), "window": args.window, "halo": args.halo,
           "batch": args.batch,
           "shapes": sorted({tt.in_shape for tt in tiles}),
           "halo_overhead": round(run_px / (args.height * args.width * 16), 4),
           "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 2),
           "plans_cached": len(runner.plans), "plan_cache_gib": round(runner.cached_bytes() / 2**30, 2),
           "canvas": list(canvas.shape) if canvas is not None else None}
    if args.sim_world > 1 and world == 1:
        res.update(simulate(args, up, runner, img.to(dev), t, dev))
    if rank == 0:
        print(json.dumps(res), flush=True)
        if args.out:
            Path(args.out).write_text(json.dumps(res, indent=1))
    if world > 1:
        dist.destroy_process_group()


def simulate(args, up, runner, img, t1, dev):
    """Each rank's share of an args.sim_world deal run alone on this GPU (see module doc)."""
    N = args.sim_world
    shards = up.shards(img.shape[1], img.shape[2], N)
    ranks = []
    s = up.scale
    canvas = torch.zeros((3, img.shape[1] * s, img.shape[2] * s), dtype=torch.uint8)
    with torch.no_grad():
        for r in range(N):
            done = up.run_tiles(img, shards[r])  # warm: builds this rank's plans
            runner.verify()
            pins = {tt.index: torch.empty(done[tt.index].shape, dtype=torch.uint8, pin_memory=True)
                    for tt in shards[r]}
            ts, td, ta = [], [], []
            for _ in range(args.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                done = up.run_tiles(img, shards[r])
                runner.verify()
                torch.cuda.synchronize()
                t1r = time.perf_counter()
                for tt in shards[r]:  # the hand-off: device → pinned host, 1/N of the canvas
                    pins[tt.index].copy_(done[tt.index], non_blocking=True)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                for tt in shards[r]:  # host assembly into the canvas (reported apart)
                    canvas[:, tt.y * s:(tt.y + tt.h) * s, tt.x * s:(tt.x + tt.w) * s] = pins[tt.index]
                t3 = time.perf_counter()
                ts.append(t2 - t0)
                td.append(t2 - t1r)
                ta.append(t3 - t2)
            shapes = sorted({tt.in_shape for tt in shards[r]})
            out_bytes = sum(pins[tt.index].numel() for tt in shards[r])
            ranks.append({"rank": r, "s": round(statistics.median(ts), 4), "d2h_s": round(statistics.median(td), 5),
                          "assemble_s": round(statistics.median(ta), 5), "out_mb": round(out_bytes / 1e6, 1),
                          "tiles": len(shards[r]), "shapes": shapes, "run_px": sum(tt.cost for tt in shards[r])})
            print(json.dumps({"sim_rank": ranks[-1]}), flush=True)
    mx = max(x["s"] for x in ranks)
    return {"sim_world": N, "shard": args.shard, "sim_ranks": ranks, "sim_max_rank_s": mx,
            "sim_t1_over_n_s": round(t1 / N, 4), "sim_ratio": round(mx / (t1 / N), 3),
            "sim_value_mpix_s": round(args.height * args.width * 16 / mx / 1e6, 1),
            "sim_note": "per-rank shares run alone on one GPU; each rank's time includes the device -> "
                        "pinned-host copy of its share of the canvas (d2h_s); host assembly (assemble_s) apart"}


if __name__ == "__main__":
    main()
