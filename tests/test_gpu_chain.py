"""The persistent RRDB-trunk kernel (isr_conv_chain: trunk.hip, conv3x3.hip): the whole trunk of
RDB convs in one launch with tile-level dependencies must reproduce the per-conv
launches BIT FOR BIT (same tile arithmetic; only the hand-off differs: sc1 loads /
write-through stores, progress words).  Repeated launches stress the hand-off for
races or stale reads; several geometries cover ragged tiles and more tiles than
resident workgroups (a workgroup walking several tiles per layer)."""
import os

import pytest
import torch

from image_super_resolution_amd import engine, models
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict

pytestmark = pytest.mark.gpu
DEV = "cuda"
# The production libisr.so carries the production trunk form (variant 0) only; the A/B forms are
# built into lib/libisr_tuning.so (ISR_LIB=.../libisr_tuning.so runs this file on all of them).
TUNING_LIB = "tuning" in os.environ.get("ISR_LIB", "")


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _gw(blocks, scale=4, enchant=False, seed=0, f16=True):
    m = (models.EResNet if enchant else models.ResNet)(blocks, 0.2, scaleRate=scale)
    sd = synth_state_dict(m.state_dict(), seed)
    return engine.pack_generator({k: v.to(DEV) for k, v in sd.items()}, enchant=enchant, device=DEV, f16=f16)


def _run(gw, xs, chain, acquire=False, variant=0):
    """One plan, one forward per input in `xs` (different inputs back to back: a stale
    hand-off read would return the previous input's activations and show up)."""
    x0 = xs[0]
    old = engine.CHAIN_VARIANT
    engine.CHAIN_VARIANT = variant
    try:
        plan = engine.GeneratorPlan(gw, x0.shape[0], x0.shape[2], x0.shape[3], x0.device, False, False,
                                    (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), chain=chain,
                                    chain_acquire=acquire)
    finally:
        engine.CHAIN_VARIANT = old
    if chain:
        assert plan.chain is not None and plan.chain.variant == variant
    outs = []
    for x in xs:
        out = torch.empty(plan.out_shape, device=DEV)
        plan.run(x, out)
        outs.append(out)
    torch.cuda.synchronize()
    if chain:
        assert plan.chain is not None and not plan.chain.failed(), "a chain dependency wait gave up"
    return outs


def _inputs(n, h, w, k, seed):
    return [normalize(synth_lr_batch(n, h, w, seed=seed + i, scale=4)[0]).to(DEV).contiguous() for i in range(k)]


# (4, 512, 512) = 2,048 tiles and (1, 540, 960) = 1,020 ragged tiles: more tiles than the 512
# resident workgroups of a 256-CU chip, so every workgroup walks several tiles per layer (the
# video and 4K-still geometry)
# (10, 768, 768): every dense buffer is 2.28 GB, past the 2 GiB a single buffer resource can span —
# the trunk kernel addresses each 16-channel plane through its own resource (round 5)
@pytest.mark.parametrize("n,h,w,blocks", [(2, 36, 52, 2), (1, 128, 128, 1), (16, 128, 128, 16), (4, 256, 256, 2),
                                          (4, 512, 512, 1), (1, 540, 960, 1), (10, 768, 768, 1)])
@pytest.mark.parametrize("f16", [True, False], ids=["fp16", "bf16"])
def test_chain_bitwise_equals_per_conv_launches(n, h, w, blocks, f16):
    """fp16 storage (the inference default) runs the production trunk form only; the bf16 forms
    (the training forward's storage) also sweep the tuning library's A/B forms."""
    gw = _gw(blocks, f16=f16)
    xs = _inputs(n, h, w, 3, seed=3)
    refs = _run(gw, xs, chain=False)
    # variants 3 and 4 (32x32 tiles) need the 16-row-rounded height to be a multiple of 32
    variants = ((0, 7, 8, 6, 5, 2, 1) + ((3,) if -(-h // 16) % 2 == 0 else ())) if TUNING_LIB else (0,)
    if os.environ.get("ISR_TEST_CHAIN_VARIANTS"):
        variants = tuple(int(v) for v in os.environ["ISR_TEST_CHAIN_VARIANTS"].split(","))
    if f16:
        variants = (0,)
    if n * 12 * (h + 2) * (w + 2) * 32 >= 2 ** 31:  # the round-2 kernel (1) addresses a buffer with 32-bit offsets
        variants = tuple(v for v in variants if v != 1)
    for variant in variants:
        for acquire in (False, True):
            for out, ref in zip(_run(gw, xs, chain=True, acquire=acquire, variant=variant), refs):
                assert torch.equal(out, ref), \
                    f"chain variant {variant} (acquire={acquire}) differs: max {(out - ref).abs().max().item()}"


def test_chain_repeated_stress_eresnet():
    """EResNet (no BN; conv weights scaled 0.2): 20 back-to-back chained forwards at the
    bench shape over 4 different inputs in turn, every output bitwise equal to the
    per-conv launches of the same input."""
    gw = _gw(4, enchant=True, seed=2)
    xs = _inputs(16, 128, 128, 4, seed=9)
    refs = _run(gw, xs, chain=False)
    for _ in range(5):
        for out, ref in zip(_run(gw, xs, chain=True), refs):
            assert torch.equal(out, ref)


def test_chain_rejects_a_bad_layer_table_loudly():
    """The trunk kernel's prep pass refuses a layer table its records cannot express (here: a
    growth layer whose kind says 'final'): the launch gives up (state[1] == state[0]) instead of
    computing garbage silently, and the product-path check raises."""
    gw = _gw(1)
    x = _inputs(2, 32, 32, 1, seed=1)[0]
    plan = engine.GeneratorPlan(gw, 2, 32, 32, x.device, False, False, (0.485, 0.456, 0.406),
                                (0.229, 0.224, 0.225), chain=True)
    assert plan.chain.variant == 0
    plan.chain._kinds[0] = 1  # growth conv (cout 32) declared as an RDB final conv
    out = torch.empty(plan.out_shape, device=DEV)
    plan.run(x, out)
    torch.cuda.synchronize()
    assert plan.chain.failed()


def test_chain_poll_reports_a_give_up():
    """The product path's lagged check (engine.ConvChain.poll, called by GeneratorPlan.run):
    a launch whose dependency wait gave up (simulated: give-up word = generation) raises on a
    later call instead of passing silently."""
    from image_super_resolution_amd import engine, models
    from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict
    dev = torch.device("cuda")
    sd = synth_state_dict(models.ResNet(1, 0.2, scaleRate=4).state_dict(), seed=0)
    gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev)
    lr, _ = synth_lr_batch(2, 32, 32, seed=1)
    x = normalize(lr).to(dev).contiguous()
    plan = engine.GeneratorPlan(gw, 2, 32, 32, dev, False, False, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225),
                                chain=True)
    out = torch.empty(plan.out_shape, device=dev)
    plan.run(x, out)
    torch.cuda.synchronize()
    plan.run(x, out)  # clean launches: no error
    torch.cuda.synchronize()
    plan.verify()
    plan.chain.state[2] += 1  # as if a dependency wait had given up (the sticky give-up count)
    torch.cuda.synchronize()
    with pytest.raises(engine.ChainFailed):
        plan.run(x, out)
        torch.cuda.synchronize()
        plan.run(x, out)  # the lagged check raises on the call after the snapshot has landed
    plan.chain.state[2] += 1
    with pytest.raises(engine.ChainFailed):
        plan.verify()  # the blocking check of one-shot consumers raises at once
    plan.verify()      # reported once


def test_give_up_raises_from_video_and_tiler_before_output():
    """A give-up (simulated through the sticky count) must surface from the shipped consumers
    BEFORE their outputs leave: the video writer (graph replays), FrameUpscaler's synchronous
    call and the tiler's canvas."""
    import numpy as np
    from image_super_resolution_amd import tiler, video
    gw = _gw(1, scale=2)
    up = video.FrameUpscaler(gw, 24, 40, batch=2)
    assert up.plan.chains, "the video plan must run the trunk on the persistent chain"
    frames = [np.full((24, 40, 3), i, np.uint8) for i in range(5)]
    rec = video.NullRecorder()
    assert video.VideoUpscaler(up).run(frames, rec) == 5
    up.plan.chain.state[2] += 1
    rec = video.NullRecorder()
    with pytest.raises(engine.ChainFailed):
        video.VideoUpscaler(up).run(frames, rec)
    assert rec.frames <= 2  # at most the batch in flight before the failing one was written
    up.plan.chain.state[2] += 1
    with pytest.raises(engine.ChainFailed):
        up(torch.from_numpy(np.stack(frames[:2])))
    runner = tiler.GeneratorRunner(gw, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), DEV)
    tu = tiler.TileUpscaler(runner, scale=2, window=32, halo=0, batch=4)
    img = torch.randint(0, 255, (3, 40, 70), dtype=torch.uint8)
    tu(img)
    for plan in runner.plans.values():
        for c in plan.chains:
            c.state[2] += 1
    with pytest.raises(engine.ChainFailed):
        tu(img)


def test_give_up_training_step_leaves_parameters_unchanged():
    """A training forward whose trunk kernel gave up (simulated through the sticky count) must
    not reach the parameters: trainer.train's Adam and EMA updates of that step are skipped on
    the device (optim.step_guard → isr_mt_adam_guarded / isr_mt_lerp_guarded), the epoch-end
    check raises ChainFailed, and once the host has reported it the next step updates again."""
    from image_super_resolution_amd import optim, trainer
    torch.manual_seed(0)
    m = models.EResNet(1, 0.2, 4)
    m.load_state_dict(synth_state_dict(m.state_dict(), 7))
    m = m.to(DEV).train()
    ema = models.ModelEMA(m, tau=100)
    opt = optim.FusedAdam(m.parameters(), lr=1e-3)
    sched = torch.optim.lr_scheduler.LinearLR(opt, 1.0, 0.5, 10)
    sc = torch.amp.GradScaler("cuda", enabled=False)
    lr, hr01 = synth_lr_batch(2, 24, 32, seed=3, scale=4)
    batch = (hr01.to(DEV) * 2 - 1, normalize(lr).to(DEV))
    ident = lambda b: b  # noqa: E731  (the batch is already (hr, lr))
    loss = torch.nn.functional.mse_loss

    def snap():
        return ([p.detach().clone() for p in m.parameters()],
                [v.detach().clone() for v in ema.ema.state_dict().values() if v.dtype.is_floating_point])

    trainer.train(m, ema, [batch], ident, loss, opt, sc, sched, 0, steps=1)
    plan = m.__dict__["_isr_train_plan"]
    assert plan.chain is not None, "the training forward must run the trunk on the persistent kernel"
    p0, e0 = snap()
    plan.chain.state[2] += 1  # a give-up of the next forward's trunk launch
    with pytest.raises(engine.ChainFailed):
        trainer.train(m, ema, [batch], ident, loss, opt, sc, sched, 1, steps=1)
    p1, e1 = snap()
    for a, b in zip(p0 + e0, p1 + e1):
        assert torch.equal(a, b), "a failed trunk forward changed a parameter or the EMA"
    trainer.train(m, ema, [batch], ident, loss, opt, sc, sched, 2, steps=1)  # reported: updates resume
    p2, _ = snap()
    assert any(not torch.equal(a, b) for a, b in zip(p1, p2))


def test_give_up_srgan_step_leaves_parameters_unchanged():
    """The same guard on trainer.train_srgan: the SRGAN wrapper's training plan lives on its
    res_net; a step whose trunk gave up changes neither G, the EMA nor D, the epoch-end check
    raises ChainFailed, and the next step updates again."""
    import warnings
    from image_super_resolution_amd import data, loss as L, optim, trainer
    torch.manual_seed(0)
    g = models.SRGAN(1, 0.2, True, 4)
    g.load_state_dict(synth_state_dict(g.state_dict(), 7))
    g = g.to(DEV).train()
    d = models.Discriminator(3, 64, 8, 1024).to(DEV)
    d.use_libisr(True)
    ema = models.ModelEMA(g, tau=100)
    og = optim.FusedAdam(g.parameters(), lr=1e-3)
    od = optim.FusedAdam(d.parameters(), lr=1e-3)
    sg = torch.optim.lr_scheduler.LinearLR(og, 1.0, 0.5, 10)
    sd = torch.optim.lr_scheduler.LinearLR(od, 1.0, 0.5, 10)
    sc = (torch.amp.GradScaler("cuda", enabled=False), torch.amp.GradScaler("cuda", enabled=False))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gl = L.gen_loss(device=DEV, beforeAct=True)
    mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
    lr, hr01 = synth_lr_batch(2, 24, 32, seed=3, scale=4)
    batch = (hr01.to(DEV), normalize(lr).to(DEV))
    ident = lambda b: b  # noqa: E731

    def step(epoch):
        trainer.train_srgan(g, ema, d, [batch], ident, gl, og, od, sc, (sg, sd), epoch, None, mean=mean, std=std,
                            steps=1)

    def snap():
        return ([p.detach().clone() for p in g.parameters()] + [p.detach().clone() for p in d.parameters()]
                + [v.detach().clone() for v in ema.ema.state_dict().values() if v.dtype.is_floating_point])

    step(0)
    plan = g.res_net.__dict__["_isr_train_plan"]
    assert plan.chain is not None and trainer.step_guard_ptr(g) is not None
    s0 = snap()
    plan.chain.state[2] += 1  # a give-up of the next forward's trunk launch
    with pytest.raises(engine.ChainFailed):
        step(1)
    s1 = snap()
    for a, b in zip(s0, s1):
        assert torch.equal(a, b), "a failed trunk forward changed G, D or the EMA"
    step(2)  # reported: updates resume
    s2 = snap()
    assert any(not torch.equal(a, b) for a, b in zip(s1, s2))
