#!/usr/bin/env python3
"""Video super-resolution throughput (BASELINE configs[4]): 1080p → 4K with the
x2 RRDB generator (ResNet(16, 0.2, scaleRate=2), synthetic weights), uint8 frames
through video.VideoUpscaler (pinned staging, HIP-graph forward, writer thread)
into a NullRecorder.  Prints one JSON line: end-to-end fps and the graph-only
per-batch GPU time.

python tools/bench_video.py [--frames 24] [--batch 1] [--height 1080 --width 1920]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from image_super_resolution_amd import engine, models, video  # noqa: E402
from image_super_resolution_amd.weights import synth_state_dict  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=24)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--no-graph", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(args.blocks, 0.2, scaleRate=2).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
    up = video.FrameUpscaler(gw, args.height, args.width, args.batch, device=dev, graph=not args.no_graph)
    src = list(video.SyntheticVideo(args.width, args.height, min(args.frames, 8)))
    frames = [src[i % len(src)] for i in range(args.frames)]
    # graph-only GPU time per batch
    up(torch.from_numpy(np.stack(frames[:args.batch])))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record(up.stream)
    for _ in range(reps):
        up.run_async()
    e1.record(up.stream)
    torch.cuda.synchronize()
    gpu_ms = e0.elapsed_time(e1) / reps
    # the persistent trunk kernel alone (its launch replayed on the plan's stream): its share of
    # the per-batch GPU time, and the batch's trunk FLOPs per second
    import ctypes

    from image_super_resolution_amd import ops
    plan = up.plan.subs[0] if hasattr(up.plan, "subs") else up.plan
    chain = getattr(plan, "chain", None)
    trunk_ms = None
    if chain is not None:
        with torch.cuda.stream(up.stream):
            sp = ops._stream()
            t0e, t1e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0e.record(up.stream)
            for _ in range(reps):
                chain.fn(ctypes.byref(chain.desc), sp)
            t1e.record(up.stream)
        torch.cuda.synchronize()
        trunk_ms = t0e.elapsed_time(t1e) / reps
        assert not chain.failed()
    frame_flops = engine.generator_flops(args.height, args.width, args.blocks, 1)
    # end to end
    pipe = video.VideoUpscaler(up)
    rec = video.NullRecorder()
    pipe.run(frames[:2 * args.batch], rec)  # warm the pinned path
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = pipe.run(frames, rec)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    H, W = up.out_hw
    print(json.dumps({"metric": "video SR frames/s (1080p -> 4K, x2 RRDB)", "value": round(n / dt, 3),
                      "unit": "frames/s", "frames": n, "batch": args.batch, "in": f"{args.width}x{args.height}",
                      "out": f"{W}x{H}", "graph": not args.no_graph,
                      "gpu_ms_per_batch": round(gpu_ms, 3), "gpu_fps": round(args.batch * 1e3 / gpu_ms, 3),
                      "trunk": "persistent trunk kernel" if chain is not None else "per-conv launches",
                      "trunk_ms_per_batch": None if trunk_ms is None else round(trunk_ms, 3),
                      "trunk_share": None if trunk_ms is None else round(trunk_ms / gpu_ms, 4),
                      "model_tflops_per_s": round(frame_flops * args.batch / gpu_ms / 1e9, 1),
                      "tflop_per_frame": round(frame_flops / 1e12, 2),
                      "out_mpix_s": round(n * H * W / dt / 1e6, 1),
                      "data": "synthetic frames, synthetic weights, NullRecorder (no encoder)"}))


if __name__ == "__main__":
    main()
