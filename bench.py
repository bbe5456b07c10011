#!/usr/bin/env python3
"""4x RRDB super-resolution inference benchmark on MI355X (BASELINE.json configs[1]).

Workload: ResNet(num_block_resnet=16, add_rate=0.2, scaleRate=4) — the reference's
RRDB generator (utils/models.py:592-618) — bf16 on the HIP kernels, 16 synthetic
128x128 LR tiles per GPU → 16 x 512x512 HR, inputs resident in HBM.  One step =
one generator forward over the batch on one HIP stream: head9x9, the whole RRDB trunk as
ONE persistent launch (isr_conv_chain → trunk.hip), conv1, two Scalers, tail9x9
(--streams k > 1 selects the per-conv split plan, engine.SplitGeneratorPlan, for A/B
only).  Multi-GPU: one process per GPU, each
rank runs its own 16 tiles (tiles are independent: weak scaling, no
collective on the data path; only the timing uses a MAX all-reduce).

Prints one JSON line (rank 0).  The timed steps replay the forward as one HIP
graph (engine.GraphedPlan; --no-graph for the eager ctypes launch loop, whose
~15 us of host time per launch would otherwise bound the step).  Extra fields:
  roofline      — the dominant kernel: the persistent RRDB-trunk kernel
                  (isr_conv_chain: all 240 RDB convs in one launch, ~85 % of the
                  step), against the HBM bound (the trunk's layer-
                  granularity bytes bind, B/BW > F/P).  Algorithmic bytes per launch
                  = 48 RDBs x (each conv's input read once + output written once:
                  832 channels) x 2 B x N*H*W = 20.9 GB at N=16, 128²; its launch is
                  replayed back to back on the launch stream between one pair of HIP
                  events (5 rounds, median), so the per-launch time matches
                  rocprofv3's kernel trace of the same command.  traffic = PMC HBM
                  bytes per launch from profiles/<round>_pmc_traffic.json
                  (rocprofv3 --pmc, corrected per MI355X_MICROARCH.md), or null.
  roofline_kernels — the chain kernel, the per-conv kernels it is built from, and the 9x9 tail
                  (used by the training path and the non-chained plan), each against
                  its own bound: growth convs (32-cout tile, HBM: (cin + 32) channels x
                  2 B x N*H*W per launch) and the RDB final conv 192->64 (MFMA,
                  2*9*192*64 FLOP per output pixel), timed on a per-conv plan.
  model_roofline — SURVEY.md §8d: max(F / P_mfma, B / BW_hbm) / t_step for the
                  whole forward (F = 410.9 GFLOP and B = 1.403 GB bf16 per 128²
                  tile at layer granularity).
  cpu_baseline  — the parity-verified CPU restatement (oracle/ref_cpu.py, torch
                  fp32) on this host's CPUs available to the process (affinity,
                  capped by the cgroup CPU quota; the count is stated), batch 1
                  and batch 16 (`value` = batch 16, the GPU workload's shape).
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
GROWTH = tuple(("conv3x3", 64 + 32 * k, 32) for k in range(4))  # RDB growth convs (32-cout tile)
FINAL = (("conv3x3", 192, 64),)                                  # RDB final conv
# SURVEY.md §8d, per 128x128 LR tile of ResNet(16, x4): FLOPs and layer-granularity bf16 bytes
TILE_FLOP = 410.9e9
TILE_BYTES = 1.403e9


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
    ap.add_argument("--round", default="r04")
    ap.add_argument("--no-graph", action="store_true", help="eager launch loop instead of the HIP graph")
    ap.add_argument("--backend", default="nccl", help="process-group backend for N>1 (nccl = RCCL)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the batch is split over (default engine.DEFAULT_STREAMS)")
    return ap.parse_args()


def load_traffic(round_tag: str) -> dict:
    """{family: PMC HBM bytes per launch} from profiles/<round>_pmc_traffic.json."""
    p = ROOT / "profiles" / f"{round_tag}_pmc_traffic.json"
    if not p.exists():
        return {}
    try:
        d = json.loads(p.read_text())
        return {k: v.get("hbm_bytes_per_launch") for k, v in d.get("families", {}).items()}
    except Exception:
        return {}


def cpu_cores() -> dict:
    """CPUs this process may actually use: affinity, capped by the cgroup v2 quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    return {"use": min(aff, quota) if quota else aff, "os_cpu_count": os.cpu_count(), "affinity": aff,
            "cgroup_quota": quota}


def time_family(plan, tags, stream, sp, rounds=5):
    """Median per-launch ms of `plan`'s launches tagged in `tags`, replayed back to
    back in forward order between one pair of HIP events on the launch stream."""
    launches = [(fn, d, tag) for fn, d, tag, var in plan.launches if tag in tags and var is None]
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for fn, d, _ in launches:
            fn(ctypes.byref(d), sp)
        e1.record(stream)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / len(launches))
    return statistics.median(res), [t for _, _, t in launches]


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
    if args.no_graph:
        step = lambda: plan.run(x, out)  # noqa: E731
    else:
        step = engine.GraphedPlan(plan, x, out).run

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = tt.item()

    ms = elapsed / args.steps * 1e3
    plan.verify()  # a persistent-chain give-up in any timed step (sticky count) voids the run: raises
    hr_px = n * (hw * S) * (hw * S)
    mpix_s = world * hr_px * args.steps / elapsed / 1e6
    # Per-kernel roofline, after the timed region.  The production forward's dominant kernel
    # is the persistent trunk kernel (isr_conv_chain, all 240 RDB convs): its launch replayed
    # back to back on the launch stream between HIP events.  The per-conv kernels (used by the
    # training path and the non-chained plan) are timed the same way on a single-stream,
    # full-batch, per-conv plan (under a split plan two half-batch launches share the CUs, so
    # a launch's duration is not its own).
    stream, sp = torch.cuda.current_stream(), ops._stream()
    npx = n * hw * hw
    traffic = load_traffic(args.round)
    kernels = {}
    chained = (plan.subs[0] if n_streams > 1 else plan).chain is not None
    if chained and n_streams == 1:
        c_ms, c_tags = time_family(plan, {("chain", 15 * args.blocks)}, stream, sp)
        trunk_bytes = args.blocks * 3 * (sum(64 + 32 * k + 32 for k in range(4)) + 192 + 64) * 2 * npx
        trunk_flops = args.blocks * 3 * (sum(2.0 * 9 * (64 + 32 * k) * 32 for k in range(4))
                                         + 2.0 * 9 * 192 * 64) * npx
        c_gbs = trunk_bytes / (c_ms * 1e-3) / 1e9
        kernels["chain"] = {"bound": "hbm", "kernel": "trunk_kernel (trunk.hip: the RRDB trunk, 240 convs, one persistent launch)",
                            "achieved": round(c_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(c_gbs / HBM_PEAK_GBS, 4), "traffic": traffic.get("chain"),
                            "bytes_per_launch": trunk_bytes, "flops_per_launch": trunk_flops,
                            "avg_launch_ms": round(c_ms, 5), "launches_per_step": len(c_tags),
                            "mfma_frac": round(trunk_flops / (c_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4),
                            "share_of_step": round(c_ms / ms, 4)}
    iso = engine.GeneratorPlan(gw, n, hw, hw, dev, False, False, mean, std, chain=False)
    iso.run(x, out)
    torch.cuda.synchronize()
    g_ms, g_tags = time_family(iso, GROWTH, stream, sp)
    g_bytes = statistics.mean((t[1] + t[2]) * 2 * npx for t in g_tags)
    g_flops = statistics.mean(2.0 * 9 * t[1] * t[2] * npx for t in g_tags)
    g_gbs = g_bytes / (g_ms * 1e-3) / 1e9
    kernels["growth"] = {"bound": "hbm", "kernel": "conv3x3_fwd 32-cout tile (RDB growth convs, cin 64/96/128/160)",
                         "achieved": round(g_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(g_gbs / HBM_PEAK_GBS, 4), "traffic": traffic.get("growth"),
                         "bytes_per_launch": g_bytes, "avg_launch_ms": round(g_ms, 5),
                         "launches_per_step": len(g_tags),
                         "mfma_frac": round(g_flops / (g_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4)}
    f_ms, f_tags = time_family(iso, FINAL, stream, sp)
    f_flops = 2.0 * npx * 9 * 192 * 64
    f_tf = f_flops / (f_ms * 1e-3) / 1e12
    kernels["final"] = {"bound": "mfma", "kernel": "conv3x3_fwd 192->64 (RDB final conv)",
                        "achieved": round(f_tf, 1), "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(f_tf / MFMA_BF16_PEAK_TFLOPS, 4), "traffic": traffic.get("final"),
                        "flops_per_launch": f_flops, "avg_launch_ms": round(f_ms, 5),
                        "launches_per_step": len(f_tags)}
    # the 9x9 tail (conv2 64->3 + tanh, row-streaming kernel) on the production plan: HBM-bound,
    # algorithmic bytes = its bf16 input once + the output once
    p0 = plan.subs[0] if n_streams > 1 else plan
    t_ms, t_tags = time_family(p0, {("tail9x9", 64, 3)}, stream, sp)
    hr_side = hw * S
    t_bytes = (n // max(1, n_streams)) * hr_side * hr_side * (64 * 2 + 3 * out.element_size())
    t_gbs = t_bytes / (t_ms * 1e-3) / 1e9
    t_flops = 2.0 * 81 * 64 * 3 * (n // max(1, n_streams)) * hr_side * hr_side
    kernels["tail"] = {"bound": "hbm", "kernel": "tail9x9 (conv2 9x9 64->3 + tanh, row-streaming, 8 waves)",
                       "achieved": round(t_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(t_gbs / HBM_PEAK_GBS, 4), "traffic": traffic.get("tail"),
                       "bytes_per_launch": t_bytes, "avg_launch_ms": round(t_ms, 5),
                       "launches_per_step": len(t_tags) * max(1, n_streams),
                       "flops_per_launch": t_flops,
                       "mfma_frac": round(t_flops / (t_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4)}
    model_flops = engine.generator_flops(hw, hw, args.blocks, S // 2) * n
    f_over_p = model_flops / (MFMA_BF16_PEAK_TFLOPS * 1e12) * 1e3
    b_over_bw = TILE_BYTES * n * (hw * hw) / (128 * 128) / (HBM_PEAK_GBS * 1e9) * 1e3
    model_roofline = {"F_over_P_ms": round(f_over_p, 4), "B_over_BW_ms": round(b_over_bw, 4),
                      "frac": round(max(f_over_p, b_over_bw) / ms, 4),
                      "mfma_frac": round(f_over_p / ms, 4), "hbm_frac": round(b_over_bw / ms, 4)}

    result = None
    if rank == 0:
        cpu = None
        parity = None
        if not args.no_cpu_baseline:
            from oracle import ref_cpu
            torch.set_grad_enabled(False)
            cores = cpu_cores()
            torch.set_num_threads(cores["use"])
            x1 = x_cpu[:1]
            ts = []
            ref = None
            t_start = time.perf_counter()
            while True:  # batch 1: one warm-up + up to 3 timed
                t1 = time.perf_counter()
                ref = ref_cpu.generator(sd_cpu, x1, num_blocks=args.blocks, scale=S)
                ts.append(time.perf_counter() - t1)
                if len(ts) >= 4 or time.perf_counter() - t_start > args.cpu_seconds / 2:
                    break
            t_b1 = statistics.median(ts[1:]) if len(ts) > 1 else ts[0]
            nb = min(n, 16)
            t1 = time.perf_counter()
            ref_cpu.generator(sd_cpu, x_cpu[:nb], num_blocks=args.blocks, scale=S)
            t_b16 = time.perf_counter() - t1
            cpu = {"value": round(nb * (hw * S) ** 2 / t_b16 / 1e6, 4), "unit": "MPix/s",
                   "cores": cores["use"], "kind": "port",
                   "batch1_mpix_s": round((hw * S) ** 2 / t_b1 / 1e6, 4),
                   "os_cpu_count": cores["os_cpu_count"], "cgroup_quota_cpus": cores["cgroup_quota"],
                   "sample": f"oracle/ref_cpu.generator fp32 (torch CPU, {cores['use']} threads), "
                             f"batch {nb} of {hw}x{hw}->{hw * S}x{hw * S}: one run {t_b16:.2f} s; batch 1: "
                             f"{len(ts)} runs (first = warm-up), median {t_b1:.3f} s/tile"}
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
                       "streams_per_gpu": n_streams, "hip_graph": not args.no_graph,
                       "trunk": "persistent chain kernel" if chained else "one launch per conv"},
            "roofline": kernels.get("chain", kernels["growth"]),
            "roofline_kernels": kernels,
            "model_roofline": model_roofline,
            "model_tflops_per_s": round(model_flops / (ms * 1e-3) / 1e12, 2),
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
