#!/usr/bin/env python3
"""4x RRDB super-resolution inference benchmark on MI355X (BASELINE.json configs[1]).

Workload: ResNet(num_block_resnet=16, add_rate=0.2, scaleRate=4) — the reference's
RRDB generator (utils/models.py:592-618) — bf16 on the HIP kernels, 16 synthetic
128x128 LR tiles per GPU → 16 x 512x512 HR, inputs resident in HBM.  One step =
one generator forward over the batch, split over 2 HIP streams (8 tiles each,
engine.SplitGeneratorPlan; --streams 1 for the single-stream plan).  Multi-GPU: one process per GPU, each
rank runs its own 16 tiles (tiles are independent: weak scaling, no
collective on the data path; only the timing uses a MAX all-reduce).

Prints one JSON line (rank 0).  Extra fields:
  roofline      — dominant kernel (conv3x3 192→64, 48 launches per forward):
                  timed in isolation on a single-stream full-batch plan (same
                  kernel, full-batch grid; under the split plan two half-batch
                  launches share the CUs, so their durations are not their own):
                  its 48 launches of one forward replayed back to back on the
                  launch stream between one pair of HIP events (5 rounds, after
                  the timed region), so the per-launch average matches the
                  rocprofv3 kernel-trace average of the same command; the
                  in-network bracketed average (events around each launch of 3
                  untimed forwards after the timed region: event records inside
                  the timed loop would cost ~4 % of a step) is reported beside it.  achieved =
                  algorithmic FLOPs per launch / avg launch time, against the
                  2.5 PFLOP/s dense bf16 MFMA peak.
                  traffic = PMC HBM bytes per launch from
                  profiles/<round>_pmc_traffic.json (rocprofv3 --pmc pass of this
                  command, corrected per MI355X_MICROARCH.md), or null.
  cpu_baseline  — the parity-verified CPU restatement (oracle/ref_cpu.py, torch
                  fp32) timed on this host on a bounded sample (batch-1 tiles).
  parity        — PSNR of the GPU output vs that CPU reference on the same
                  tile, and the |ΔPSNR| against the synthetic HR target.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense, MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0
DOMINANT = ("conv3x3", 192, 64)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="LR tiles per GPU")
    ap.add_argument("--lr-size", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--scale", type=int, default=4)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--round", default="r01")
    ap.add_argument("--backend", default="nccl", help="process-group backend for N>1 (nccl = RCCL)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the batch is split over (default engine.DEFAULT_STREAMS)")
    return ap.parse_args()


def load_traffic(round_tag: str):
    p = ROOT / "profiles" / f"{round_tag}_pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run (one process per GPU)")
    # one process per GPU; local % device_count only matters for a rehearsal with more
    # ranks than GPUs (tools/rehearse_multi.sh on a 1-GPU box, --backend gloo)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL
        else:
            dist.init_process_group(args.backend)

    from image_super_resolution_amd import engine, models, ops
    from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict

    n, hw, S = args.batch, args.lr_size, args.scale
    tmpl = models.ResNet(args.blocks, 0.2, scaleRate=S)
    sd_cpu = synth_state_dict(tmpl.state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd_cpu.items()}, enchant=False, add_rate=0.2, device=dev)
    lr, hr = synth_lr_batch(n, hw, hw, seed=1234 + rank * n, scale=S)
    x_cpu = normalize(lr)
    x = x_cpu.to(dev).contiguous()
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    plan = engine.get_plan(gw, x, False, mean, std, streams=args.streams)
    n_streams = len(plan.streams) if isinstance(plan, engine.SplitGeneratorPlan) else 1
    out = torch.empty(plan.out_shape, dtype=plan.out_dtype, device=dev)

    for _ in range(args.warmup):
        plan.run(x, out)
    torch.cuda.synchronize()

    pairs = []

    def around(tag):
        if tag == DOMINANT:
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            pairs.append(e)
            return e
        return None

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.run(x, out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()

    ms = elapsed / args.steps * 1e3
    hr_px = n * (hw * S) * (hw * S)
    mpix_s = world * hr_px * args.steps / elapsed / 1e6
    # The dominant kernel is timed in isolation: the full batch on ONE stream (with the
    # split plan two half-batch launches share the CUs, so a launch's duration is not
    # its own).  First its launches inside the network, event-bracketed, in untimed
    # forwards of their own (96 event records cost ~4 % of a step, so they stay out of
    # the timed loop) ...
    iso = plan if n_streams == 1 else engine.GeneratorPlan(gw, n, hw, hw, dev, False, False, mean, std)
    for _ in range(3):
        iso.run(x, out, around=around)
    torch.cuda.synchronize()
    in_net_ms = statistics.mean(a.elapsed_time(b) for a, b in pairs)
    # ... then back to back (per-launch time without the event packets interleaved
    # between every launch)
    dom = [(fn, d) for fn, d, tag, var in iso.launches if tag == DOMINANT and var is None]
    stream = torch.cuda.current_stream()
    sp = ops._stream()
    rounds = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for fn, d in dom:
            fn(ctypes.byref(d), sp)
        e1.record(stream)
        torch.cuda.synchronize()
        rounds.append(e0.elapsed_time(e1) / len(dom))
    kernel_ms = statistics.median(rounds)
    flops_launch = 2.0 * n * hw * hw * 9 * DOMINANT[1] * DOMINANT[2]
    achieved = flops_launch / (kernel_ms * 1e-3) / 1e12
    model_flops = engine.generator_flops(hw, hw, args.blocks, S // 2) * n
    traffic = load_traffic(args.round)

    result = None
    if rank == 0:
        cpu = None
        parity = None
        if not args.no_cpu_baseline:
            from oracle import ref_cpu
            torch.set_grad_enabled(False)
            x1 = x_cpu[:1]
            ts = []
            ref = None
            t_start = time.perf_counter()
            while True:
                t1 = time.perf_counter()
                ref = ref_cpu.generator(sd_cpu, x1, num_blocks=args.blocks, scale=S)
                ts.append(time.perf_counter() - t1)
                if len(ts) >= 8 or time.perf_counter() - t_start > args.cpu_seconds:
                    break
            tcpu = statistics.median(ts[1:]) if len(ts) > 1 else ts[0]
            cpu = {"value": round((hw * S) ** 2 / tcpu / 1e6, 4), "unit": "MPix/s",
                   "cores": torch.get_num_threads(), "kind": "port",
                   "sample": f"oracle/ref_cpu.generator fp32, 1 tile {hw}x{hw}->{hw * S}x{hw * S}, "
                             f"{len(ts)} runs (first = warm-up), median {tcpu:.3f} s/tile"}
            g = out[:1].float().cpu()
            hr1 = hr[:1] * 2 - 1
            parity = {"psnr_gpu_vs_cpu_ref_db": round(ref_cpu.psnr(g, ref), 3),
                      "dpsnr_vs_hr_db": round(abs(ref_cpu.psnr(g, hr1) - ref_cpu.psnr(ref, hr1)), 5),
                      "tolerance_db": 0.01}
        result = {
            "metric": "4x SR megapixels/sec (HR output) + PSNR vs reference CPU path",
            "value": round(mpix_s, 3),
            "unit": "MPix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (seeded smooth HR/LR tiles, synth weights: no COCO / no trained weights offline)",
            "config": {"workload": f"ResNet({args.blocks}, 0.2, scaleRate={S}) RRDB inference, "
                                   f"{hw}x{hw}->{hw * S}x{hw * S}",
                       "global_batch": n * world, "per_gpu_batch": n, "lr_size": hw, "scale": S,
                       "parallelism": f"dp{world} (independent tile shards)",
                       "streams_per_gpu": n_streams},
            "roofline": {"bound": "mfma", "kernel": "conv3x3_fwd 192->64 (RDB final conv)",
                         "achieved": round(achieved, 2), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic,
                         "avg_launch_ms": round(kernel_ms, 5), "in_network_avg_launch_ms": round(in_net_ms, 5),
                         "launches_per_step": len(dom), "flops_per_launch": flops_launch},
            "model_tflops_per_s": round(model_flops * world / (ms * 1e-3) / 1e12 / world, 2),
            "model_mfma_frac": round(model_flops / (ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
