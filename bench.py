#!/usr/bin/env python3
"""4x RRDB super-resolution inference benchmark on MI355X (BASELINE.json configs[1]).

Workload: ResNet(num_block_resnet=16, add_rate=0.2, scaleRate=4) — the reference's
RRDB generator (utils/models.py:592-618) — fp16 storage, fp32 accumulation on the HIP kernels, 16 synthetic
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
                  timed INSIDE whole forwards run back to back (HIP events around the
                  chain launch on its stream, time_in_forward), so the per-launch time
                  matches rocprofv3's kernel trace of the same command (isolated
                  launches after an idle gap run at a boosted clock: reported as
                  avg_launch_ms_isolated, not used).  traffic = PMC HBM
                  bytes per launch from profiles/<round>_pmc_traffic.json
                  (rocprofv3 --pmc, corrected per MI355X_MICROARCH.md), or null.
  roofline_kernels — the chain kernel, the per-conv kernels it is built from, and the 9x9 tail
                  (used by the training path and the non-chained plan), each against
                  its own bound: growth convs (32-cout tile, HBM: (cin + 32) channels x
                  2 B x N*H*W per launch) and the RDB final conv 192->64 (MFMA,
                  2*9*192*64 FLOP per output pixel), timed on a per-conv plan.
  model_roofline — SURVEY.md §8d: max(F / P_mfma, B / BW_hbm) / t_step for the
                  whole forward (F = 410.9 GFLOP and B = 1.403 GB of 2-byte storage per 128²
                  tile at layer granularity).
  storage_ab    — N=1 only: ms per step of the same forward with bf16 storage beside the fp16
                  default, interleaved in this process (the ~4 % clock price of fp16, DESIGN.md
                  round 6); informational, value is the fp16 default.
  cpu_baseline  — the parity-verified CPU restatement (oracle/ref_cpu.py, torch
                  fp32) on this host's CPUs available to the process (affinity,
                  capped by the cgroup CPU quota; the count is stated): the bench's
                  first 16 tiles one per call (batch 1, as rs.py runs its windows);
                  the first call is the warm-up, `value` = the median of the other 15
                  (warm-up + median).
  parity        — north star: |PSNR(GPU, HR) - PSNR(CPU reference, HR)| <= 0.01 dB over
                  those 16 tiles (and per tile, and on luma with the 4-px crop), with
                  the committed TRAINED weights (tests/golden/trained_resnet_x4.safetensors,
                  tools/train_weights.py) on held-out tiles of their data distribution —
                  weights that actually super-resolve, so the bar can fail.
  train         — BASELINE.json configs[2] per GPU: the SRGAN-mode train.py step
                  (EResNet(16) x4, VGG19 5_4 L1 + adversarial, D step, Adam/clip/EMA),
                  16 x 512² per GPU; at N > 1 with the bucketed RCCL gradient
                  all-reduce, plus the same step without it in the same job, once on
                  every rank at once (scaling_eff = its time / the data-parallel time)
                  and once on rank 0 with the other ranks idle (ms_per_step_1gpu_alone,
                  scaling_x_vs_alone: the north star's "x at 8 GPUs vs one GPU").
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
    ap.add_argument("--cpu-tiles", type=int, default=16,
                    help="tiles the CPU baseline runs one by one (the first is the warm-up; all of them are the "
                         "parity reference)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-storage-ab", dest="storage_ab", action="store_false",
                    help="skip the informational bf16-vs-fp16 storage timing")
    ap.add_argument("--round", default="r06")  # PMC traffic file (profiles/<round>_pmc_traffic.json)
    ap.add_argument("--weights", default=str(ROOT / "tests" / "golden" / "trained_resnet_x4.safetensors"),
                    help="generator state_dict (default: the committed trained ResNet(16, 0.2, x4)); "
                         "'synth' = the seeded synthetic weights of earlier rounds")
    ap.add_argument("--train-steps", type=int, default=10, help="timed steps of the cfg3 training leg (0 = skip)")
    ap.add_argument("--train-warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true", help="eager launch loop instead of the HIP graph")
    ap.add_argument("--backend", default="nccl", help="process-group backend for N>1 (nccl = RCCL)")
    ap.add_argument("--streams", type=int, default=None,
                    help="HIP streams the batch is split over (default engine.DEFAULT_STREAMS)")
    return ap.parse_args()


def log(msg: str) -> None:
    """Progress on stderr (the JSON line stays the only stdout line)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


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


def time_in_forward(plan, x, out, tags, steps):
    """Mean per-launch ms of the launches tagged in `tags` INSIDE whole forwards: `steps` eager
    forwards of the production plan back to back (no synchronisation between them, so the chip
    stays in the sustained state of the timed region), each tagged launch bracketed by HIP events
    on its launch stream (GeneratorPlan.run's `around` hook).  Isolated launches with an idle gap
    before each run at a boosted clock (round 6: 5.0-5.3 ms for the fp16 trunk against ~6.0 ms
    sustained, profiles/r06_trunk_dispatches.json), so they overstate a kernel's rate."""
    evs = []

    def around(tag):
        if tag not in tags:
            return None
        e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        evs.append(e)
        return e

    for _ in range(steps):
        plan.run(x, out, around=around)
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) for a, b in evs]
    return statistics.mean(ts), ts


def parity_report(ref_cpu, gpu: torch.Tensor, ref: torch.Tensor, hr01: torch.Tensor, weights_desc: str) -> dict:
    """North-star parity over every tile the CPU reference ran: |PSNR(GPU, HR) - PSNR(ref, HR)| on
    the [-1, 1] output (peak 2) and on BT.601 luma with the 4-px border crop (utils/datasets.py:
    159-166), aggregate over the tiles and the worst tile, plus PSNR(GPU vs CPU reference)."""
    hr1 = hr01 * 2 - 1
    p_ref, p_gpu = ref_cpu.psnr(ref, hr1), ref_cpu.psnr(gpu, hr1)
    per_tile = [abs(ref_cpu.psnr(gpu[i:i + 1], hr1[i:i + 1]) - ref_cpu.psnr(ref[i:i + 1], hr1[i:i + 1]))
                for i in range(len(gpu))]
    to01 = lambda t: (t.clamp(-1, 1) + 1) / 2  # noqa: E731
    py_ref, py_gpu = ref_cpu.psnr_y(to01(ref), hr01), ref_cpu.psnr_y(to01(gpu), hr01)
    d = abs(p_gpu - p_ref)
    return {"weights": weights_desc, "tiles": len(gpu),
            "psnr_ref_vs_hr_db": round(p_ref, 4), "psnr_gpu_vs_hr_db": round(p_gpu, 4),
            "psnr_gpu_vs_cpu_ref_db": round(ref_cpu.psnr(gpu, ref), 3),
            "dpsnr_vs_hr_db": round(d, 5), "dpsnr_worst_tile_db": round(max(per_tile), 5),
            "y_psnr_ref_vs_hr_db": round(py_ref, 4), "y_dpsnr_vs_hr_db": round(abs(py_gpu - py_ref), 5),
            "tolerance_db": 0.01, "pass": bool(d <= 0.01 and abs(py_gpu - py_ref) <= 0.01)}


def train_step_flops(batch: int, hr: int, blocks: int) -> float:
    """Algorithmic FLOPs of one SRGAN-mode step per GPU (2*MAC of every conv): G fwd
    (engine.generator_flops) + G bwd (dgrad + wgrad = 2x fwd); VGG19 to conv5_4 on SR and HR
    (203.8 GFLOP per 512² image) + its input gradient on SR; the discriminator (49.26 GFLOP per
    512² image): D(sr) fwd + dgrad for the G loss, D(sr), D(hr) fwd + dgrad + wgrad for the D loss."""
    from image_super_resolution_amd import engine
    g_fwd = engine.generator_flops(hr // 4, hr // 4, blocks, 2) * batch
    scale = (hr / 512) ** 2 * batch
    vgg_fwd, d_fwd = 203.8e9 * scale, 49.26e9 * scale
    return 3 * g_fwd + 3 * vgg_fwd + 2 * d_fwd + 2 * d_fwd + 2 * 2 * d_fwd


def train_leg(args, dev, world: int, rank: int) -> dict:
    """BASELINE.json configs[2] per GPU: one SRGAN-mode train.py step (train.py:70-129 of the
    reference) of EResNet(16, 0.2) x4 with the VGG19 conv5_4 L1 perceptual loss + adversarial
    term, discriminator step, Adam + clip + EMA, on 16 synthetic 512² HR crops per GPU.  At N > 1
    the generator's gradients go through the bucketed RCCL all-reduce overlapped with the HIP
    backward and the discriminator's through one flat all-reduce (DDP's math); the same step is
    also timed with both all-reduces off (each rank alone = the 1-GPU step, in the same job), and
    scaling_eff = that time / the data-parallel time (weak scaling: 16 samples per GPU)."""
    import warnings

    from image_super_resolution_amd import data, loss as L, models, optim, trainer
    from image_super_resolution_amd.train_engine import broadcast_params, enable_grad_allreduce
    batch, hr, blocks = 16, 512, 16
    torch.manual_seed(0)
    mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
    batches = data.SyntheticSR(batch, hr, seed=rank, device=dev)
    total = args.train_warmup + 2 * args.train_steps
    gen = models.SRGAN(blocks, 0.2, True, 4).to(dev)
    dis = models.Discriminator(3, 64, 8, 1024).to(dev).use_libisr(True)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gl = L.gen_loss(device=dev, beforeAct=True)
    og = optim.FusedAdam(gen.parameters(), lr=1e-4, betas=(0.9, 0.999))
    od = optim.FusedAdam(dis.parameters(), lr=1e-4, betas=(0.9, 0.999))
    sg = torch.optim.lr_scheduler.LinearLR(og, 1, 0.01, total_iters=total)
    sdl = torch.optim.lr_scheduler.LinearLR(od, 1, 0.01, total_iters=total)
    ema = models.ModelEMA(gen, tau=total)
    ema.ema.to(dev)
    sc = (torch.amp.GradScaler("cuda", enabled=False), torch.amp.GradScaler("cuda", enabled=False))
    tf = data.GPUTransform(4, hr_norm=True, mean=mean, std=std, device=dev)
    if world > 1:
        broadcast_params(list(gen.parameters()) + list(dis.parameters()))

    def run(steps: int, ddp: bool) -> float:
        enable_grad_allreduce(gen, True if ddp else None)
        if ddp:  # identical replicas again after an all-reduce-free run
            broadcast_params(list(gen.parameters()) + list(dis.parameters()))
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        trainer.train_srgan(gen, ema, dis, batches, tf, gl, og, od, sc, (sg, sdl), 0, None, mean=mean, std=std,
                            steps=steps, log_every=10 ** 9, dist_group=True if ddp else None)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([dt], device=dev if args.backend == "nccl" else "cpu", dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            dt = tt.item()
        return dt * 1e3 / steps

    def run_alone(steps: int) -> float:
        """The 1-GPU step with no peer running: rank 0 times the all-reduce-free
        step while every other rank waits idle on the rendezvous store (a blocking socket read, no
        spinning host thread), so the host CPUs the job shares are rank 0's alone."""
        enable_grad_allreduce(gen, None)
        store = dist.distributed_c10d._get_default_store()
        key = f"isr_bench_alone_{steps}"
        dist.barrier()
        dt = 0.0
        if rank == 0:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            trainer.train_srgan(gen, ema, dis, batches, tf, gl, og, od, sc, (sg, sdl), 0, None, mean=mean, std=std,
                                steps=steps, log_every=10 ** 9, dist_group=None)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            store.set(key, "1")
        else:
            store.wait([key])
        dist.barrier()
        return dt * 1e3 / steps

    run(args.train_warmup, world > 1)
    ms_local = run(args.train_steps, False) if world > 1 else None
    ms_alone = run_alone(args.train_steps) if world > 1 else None
    ms = run(args.train_steps, world > 1)
    flops = train_step_flops(batch, hr, blocks)
    res = {"workload": f"SRGAN(EResNet({blocks}, 0.2), x4) train step: VGG19 conv5_4 L1 + 1e-3 adversarial, "
                       f"discriminator step, Adam + clip + EMA, {batch} x {hr}² HR per GPU (BASELINE.json configs[2])",
           "data": "synthetic smooth crops (data.SyntheticSR)",
           "n_gpus": world, "global_batch": batch * world, "steps": args.train_steps, "warmup": args.train_warmup,
           "ms_per_step": round(ms, 3), "samples_per_s": round(batch * world / ms * 1e3, 2),
           "hr_mpix_s": round(batch * world * hr * hr / ms / 1e3, 2),
           "tflop_per_step_per_gpu": round(flops / 1e12, 3),
           "tflops_per_s_per_gpu": round(flops / ms / 1e9, 1),
           "mfma_frac": round(flops / ms / 1e9 / MFMA_BF16_PEAK_TFLOPS, 4),
           "parallelism": f"dp{world}" + (f" (bucketed {'RCCL' if args.backend == 'nccl' else args.backend} "
                                           "all-reduce overlapped with the HIP backward)" if world > 1 else ""),
           "dtype": "bf16 storage, fp32 accumulation and master weights"}
    if world > 1:
        # two 1-GPU denominators: every rank running the all-reduce-free step at once (host CPUs
        # shared by all N processes) and rank 0 running it with the other ranks idle
        res["ms_per_step_no_allreduce"] = round(ms_local, 3)
        res["ms_per_step_1gpu_alone"] = round(ms_alone, 3)
        res["scaling_eff"] = round(ms_local / ms, 4)
        res["scaling_x"] = round(world * ms_local / ms, 3)
        res["scaling_eff_vs_alone"] = round(ms_alone / ms, 4)
        res["scaling_x_vs_alone"] = round(world * ms_alone / ms, 3)
        cores = cpu_cores()
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        res["host_cpus"] = cores["use"]
        res["host_cpus_per_rank"] = round(cores["use"] / max(1, local_world), 2)
    del gen, dis, gl, og, od, ema
    torch.cuda.empty_cache()
    return res


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

    from image_super_resolution_amd import checkpoint, engine, models, ops
    from image_super_resolution_amd.weights import (HELDOUT_SEED, heldout_tiles, normalize, synth_lr_batch,
                                                    synth_state_dict)

    n, hw, S = args.batch, args.lr_size, args.scale
    tmpl = models.ResNet(args.blocks, 0.2, scaleRate=S)
    if args.weights == "synth":
        sd_cpu = synth_state_dict(tmpl.state_dict(), seed=0)
        lr, hr = synth_lr_batch(n, hw, hw, seed=1234 + rank * n, scale=S)
        x_cpu = normalize(lr)
        weights_desc = "seeded synthetic weights (weights.synth_state_dict), smooth synthetic tiles"
    else:  # the committed trained weights (tools/train_weights.py) on held-out tiles of their distribution
        sd_cpu = checkpoint.load_module_state(args.weights)
        tmpl.load_state_dict(sd_cpu)  # raises unless the file is a ResNet(blocks, 0.2, xS) state_dict
        x_cpu, hr = heldout_tiles(n, hw, S, seed=HELDOUT_SEED + 7919 * rank)
        weights_desc = (f"trained ResNet({args.blocks}, 0.2, x{S}) ({Path(args.weights).name}: train.py --resnet on "
                        "synthetic dead-leaves crops), held-out tiles of that distribution")
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd_cpu.items()}, enchant=False, add_rate=0.2, device=dev)
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
    log(f"inference: {ms:.3f} ms per step")
    out_timed = out.float().cpu()  # the last timed step's output (the parity leg compares it)
    plan.verify()  # a persistent-chain give-up in any timed step (sticky count) voids the run: raises
    hr_px = n * (hw * S) * (hw * S)
    mpix_s = world * hr_px * args.steps / elapsed / 1e6
    # Per-kernel roofline, after the timed region.  The production forward's dominant kernel
    # is the persistent trunk kernel (isr_conv_chain, all 240 RDB convs): timed inside whole
    # forwards run back to back (time_in_forward; its isolated replay is reported beside it).  The per-conv kernels (used by the
    # training path and the non-chained plan) are timed the same way on a single-stream,
    # full-batch, per-conv plan (under a split plan two half-batch launches share the CUs, so
    # a launch's duration is not its own).
    stream, sp = torch.cuda.current_stream(), ops._stream()
    npx = n * hw * hw
    traffic = load_traffic(args.round)
    kernels = {}
    chained = (plan.subs[0] if n_streams > 1 else plan).chain is not None
    if chained and n_streams == 1:
        chain_tag = ("chain", 15 * args.blocks)
        c_iso_ms, c_tags = time_family(plan, {chain_tag}, stream, sp)
        c_ms, c_all = time_in_forward(plan, x, out, {chain_tag}, max(args.steps, 10))
        trunk_bytes = args.blocks * 3 * (sum(64 + 32 * k + 32 for k in range(4)) + 192 + 64) * 2 * npx
        trunk_flops = args.blocks * 3 * (sum(2.0 * 9 * (64 + 32 * k) * 32 for k in range(4))
                                         + 2.0 * 9 * 192 * 64) * npx
        c_gbs = trunk_bytes / (c_ms * 1e-3) / 1e9
        # what the kernel stages into LDS per launch: per (tile, 16-channel
        # chunk) its 18 x 34 halo plane and the chunk's 32- / 64-cout weights, for every tile of every layer
        tiles = n * (-(-hw // 16)) * (-(-hw // 32))
        halo_b, wg_b, wf_b = 18 * 34 * 32, 9 * 32 * 16 * 2, 9 * 64 * 16 * 2
        staged_halo = args.blocks * 3 * tiles * (sum(4 + 2 * k for k in range(4)) + 12) * halo_b
        staged_w = args.blocks * 3 * tiles * (sum(4 + 2 * k for k in range(4)) * wg_b + 12 * wf_b)
        kernels["chain"] = {"bound": "hbm", "kernel": "trunk_kernel (trunk.hip: the RRDB trunk, 240 convs, one persistent launch)",
                            "achieved": round(c_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(c_gbs / HBM_PEAK_GBS, 4), "traffic": traffic.get("chain"),
                            "bytes_per_launch": trunk_bytes, "flops_per_launch": trunk_flops,
                            "avg_launch_ms": round(c_ms, 5), "launches_per_step": len(c_tags),
                            "timing": f"mean over {len(c_all)} launches inside back-to-back eager forwards "
                                      "(bench.time_in_forward)",
                            "avg_launch_ms_isolated": round(c_iso_ms, 5),
                            "lds_staged_bytes_per_launch": {"halo": staged_halo, "weights": staged_w,
                                                            "gb_s": round((staged_halo + staged_w) / (c_ms * 1e-3) / 1e9, 1)},
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
    if n_streams == 1:  # in situ, as the trunk (the isolated replay stays beside it)
        t_iso_ms = t_ms
        t_ms, _ = time_in_forward(p0, x, out, {("tail9x9", 64, 3)}, max(args.steps, 10))
    hr_side = hw * S
    t_bytes = (n // max(1, n_streams)) * hr_side * hr_side * (64 * 2 + 3 * out.element_size())
    t_gbs = t_bytes / (t_ms * 1e-3) / 1e9
    t_flops = 2.0 * 81 * 64 * 3 * (n // max(1, n_streams)) * hr_side * hr_side
    kernels["tail"] = {"bound": "hbm", "kernel": "tail9x9 (conv2 9x9 64->3 + tanh, row-streaming, 8 waves)",
                       "achieved": round(t_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(t_gbs / HBM_PEAK_GBS, 4), "traffic": traffic.get("tail"),
                       "bytes_per_launch": t_bytes, "avg_launch_ms": round(t_ms, 5),
                       **({"avg_launch_ms_isolated": round(t_iso_ms, 5)} if n_streams == 1 else {}),
                       "launches_per_step": len(t_tags) * max(1, n_streams),
                       "flops_per_launch": t_flops,
                       "mfma_frac": round(t_flops / (t_ms * 1e-3) / 1e12 / MFMA_BF16_PEAK_TFLOPS, 4)}
    model_flops = engine.generator_flops(hw, hw, args.blocks, S // 2) * n
    f_over_p = model_flops / (MFMA_BF16_PEAK_TFLOPS * 1e12) * 1e3
    b_over_bw = TILE_BYTES * n * (hw * hw) / (128 * 128) / (HBM_PEAK_GBS * 1e9) * 1e3
    model_roofline = {"F_over_P_ms": round(f_over_p, 4), "B_over_BW_ms": round(b_over_bw, 4),
                      "frac": round(max(f_over_p, b_over_bw) / ms, 4),
                      "mfma_frac": round(f_over_p / ms, 4), "hbm_frac": round(b_over_bw / ms, 4)}

    log("per-kernel roofline timings done")
    # The storage trade of round 6 on this box: the same forward with bf16 storage
    # (pack_generator(f16=False)), interleaved with the fp16 default in one process.  Informational:
    # value / ms_per_step above are the fp16 default; bf16 misses the north-star bar at x2.
    storage_ab = None
    if world == 1 and n_streams == 1 and not args.no_graph and gw.dtype == torch.float16 and args.storage_ab:
        gw_b = engine.pack_generator({k: v.to(dev) for k, v in sd_cpu.items()}, enchant=False, add_rate=0.2,
                                     device=dev, f16=False)
        plan_b = engine.GeneratorPlan(gw_b, n, hw, hw, dev, False, False, mean, std)
        out_b = torch.empty_like(out)
        run_b = engine.GraphedPlan(plan_b, x, out_b).run
        reps, ts = max(5, args.steps // 2), {"fp16": [], "bf16": []}
        for _ in range(3):
            for name, fn in (("fp16", step), ("bf16", run_b)):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(reps):
                    fn()
                torch.cuda.synchronize()
                ts[name].append((time.perf_counter() - t1) / reps * 1e3)
        plan_b.verify()
        storage_ab = {k: round(statistics.median(v), 4) for k, v in ts.items()}
        storage_ab.update({"unit": "ms_per_step", "rounds": 3, "steps_per_round": reps,
                           "fp16_over_bf16": round(storage_ab["fp16"] / storage_ab["bf16"], 4)})
        del plan_b, run_b, gw_b, out_b
        torch.cuda.empty_cache()
        log(f"storage A/B: fp16 {storage_ab['fp16']} ms, bf16 {storage_ab['bf16']} ms per step")
    train = train_leg(args, dev, world, rank) if args.train_steps > 0 else None
    if train is not None:
        log(f"train leg: {train['ms_per_step']} ms per step")

    result = None
    if rank == 0:
        cpu = None
        parity = None
        if not args.no_cpu_baseline:
            from oracle import ref_cpu
            torch.set_grad_enabled(False)
            cores = cpu_cores()
            torch.set_num_threads(cores["use"])
            nt = min(n, max(2, args.cpu_tiles))
            refs, ts = [], []
            for i in range(nt):  # one tile at a time (batch 1, as rs.py runs its windows)
                t1 = time.perf_counter()
                refs.append(ref_cpu.generator(sd_cpu, x_cpu[i:i + 1], num_blocks=args.blocks, scale=S))
                ts.append(time.perf_counter() - t1)
                if i % 4 == 3:
                    log(f"cpu baseline: {i + 1}/{nt} tiles")
            t_tile = statistics.median(ts[1:])
            cpu = {"value": round((hw * S) ** 2 / t_tile / 1e6, 4), "unit": "MPix/s",
                   "cores": cores["use"], "kind": "port",
                   "os_cpu_count": cores["os_cpu_count"], "cgroup_quota_cpus": cores["cgroup_quota"],
                   "tiles": nt, "warmup_tile_s": round(ts[0], 3), "median_tile_s": round(t_tile, 3),
                   "sample": f"oracle/ref_cpu.generator fp32 (torch CPU, {cores['use']} threads) on the bench's "
                             f"first {nt} {hw}x{hw}->{hw * S}x{hw * S} tiles, one tile per call: the first call "
                             f"is the warm-up, value = median of the other {nt - 1} ({sum(ts):.1f} s in all)"}
            parity = parity_report(ref_cpu, out_timed[:nt], torch.cat(refs), hr[:nt], weights_desc)
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
            "dtype": "fp16" if gw.dtype == torch.float16 else "bf16",
            "data": f"synthetic: {weights_desc} (no COCO offline)",
            "config": {"workload": f"ResNet({args.blocks}, 0.2, scaleRate={S}) RRDB inference, "
                                   f"{hw}x{hw}->{hw * S}x{hw * S}",
                       "global_batch": n * world, "per_gpu_batch": n, "lr_size": hw, "scale": S,
                       "parallelism": f"dp{world} (independent tile shards)",
                       "streams_per_gpu": n_streams, "hip_graph": not args.no_graph,
                       "trunk": "persistent chain kernel" if chained else "one launch per conv",
                       "storage": ("fp16" if gw.dtype == torch.float16 else "bf16")
                                  + " activations and packed weights, fp32 accumulation"},
            "roofline": kernels.get("chain", kernels["growth"]),
            "roofline_kernels": kernels,
            "model_roofline": model_roofline,
            "model_tflops_per_s": round(model_flops / (ms * 1e-3) / 1e12, 2),
            "cpu_baseline": cpu,
            "storage_ab": storage_ab,
            "parity": parity,
            "train": train,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
