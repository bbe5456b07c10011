"""Training at cfg3's per-GPU shape (train.py:70-129 `train_srgan`):
SRGAN(16, 0.2, enchant=True, 4) — the 16-RRDB EResNet x4 generator — on a batch of 16 crops of
512² HR / 128² LR, VGG19 conv5_4 L1 + adversarial loss, one step through trainer.train_srgan.

* The same step with the training forward's trunk on the persistent trunk kernel and on 240
  per-conv launches (ISR_TRAIN_CHAIN=0): the kernel is bit-identical to the per-conv launches
  (tests/test_gpu_chain.py), so every generator gradient must agree bit for bit (asserted after
  the test_gpu_train.py bar, rel L2 <= 5e-2 and cos >= 0.998, so a failure shows how far off).  Learning rates are 0, so the step leaves G and D unchanged and both runs see
  the same discriminator and VGG.
* A 2-sample slice of the batch (full 128² LR crops, the same 16 RRDBs) through a pixel-loss
  step vs autograd of the fp32 oracle (oracle/ref_cpu.generator) at the test_gpu_train.py bars.
* train.py's DEFAULT SRGAN mode (enchant=False, train.py:304-388): the BatchNorm ResNet generator
  inside SRGAN with the post-ReLU VGG MSE content loss (utils/loss.py:16-24), one train_srgan step
  end to end vs the fp32 oracle.
"""
import os
import warnings

import pytest
import torch
import torch.nn.functional as F

from image_super_resolution_amd import checkpoint, data, loss as L, models, optim, trainer
from image_super_resolution_amd.weights import synth_state_dict
from oracle import ref_cpu as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
BLOCKS, SCALE, BATCH, HR = 16, 4, 16, 512


@pytest.fixture(scope="module", autouse=True)
def lib(built_lib):
    return built_lib


def _gen(seed):
    g = models.SRGAN(BLOCKS, 0.2, True, SCALE)
    g.load_state_dict(synth_state_dict(g.state_dict(), seed))
    return g.to(DEV)


def _srgan_step_grads(chain: bool, dis, gl):
    """One train_srgan step (lr 0) with the trunk kernel on or off; the generator's gradients."""
    old = os.environ.get("ISR_TRAIN_CHAIN")
    os.environ["ISR_TRAIN_CHAIN"] = "1" if chain else "0"
    try:
        gen = _gen(5)
        mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
        og = optim.FusedAdam(gen.parameters(), lr=0.0)
        od = optim.FusedAdam(dis.parameters(), lr=0.0)
        sg = torch.optim.lr_scheduler.LinearLR(og, 1, 0.01, total_iters=1)
        sd = torch.optim.lr_scheduler.LinearLR(od, 1, 0.01, total_iters=1)
        ema = models.ModelEMA(gen, tau=1)
        ema.ema.to(DEV)
        sc = (torch.amp.GradScaler("cuda", enabled=False), torch.amp.GradScaler("cuda", enabled=False))
        tf = data.GPUTransform(SCALE, hr_norm=True, mean=mean, std=std, device=DEV)
        batches = data.SyntheticSR(BATCH, HR, seed=3, device=DEV)
        losses = trainer.train_srgan(gen, ema, dis, batches, tf, gl, og, od, sc, (sg, sd), 0, None, mean=mean,
                                     std=std, steps=1, log_every=1)
        torch.cuda.synchronize()
        plan = gen.res_net.__dict__["_isr_train_plan"]
        assert (plan.chain is not None) == chain, "trunk kernel on/off as requested"
        # the SRGAN wrapper's step is guarded by its res_net's trunk give-up count
        assert (trainer.step_guard_ptr(gen) is not None) == chain
        return losses[0], {n: p.grad.detach().clone() for n, p in gen.named_parameters()}
    finally:
        if old is None:
            os.environ.pop("ISR_TRAIN_CHAIN", None)
        else:
            os.environ["ISR_TRAIN_CHAIN"] = old


def test_cfg3_srgan_step_chain_vs_per_conv():
    torch.manual_seed(0)
    dis = models.Discriminator(3, 64, 8, 1024).to(DEV)
    dis.use_libisr(True)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gl = L.gen_loss(device=DEV, beforeAct=True)
    l_chain, g_chain = _srgan_step_grads(True, dis, gl)
    l_conv, g_conv = _srgan_step_grads(False, dis, gl)
    assert abs(l_chain - l_conv) <= 1e-4 * abs(l_conv) + 1e-6, (l_chain, l_conv)
    bitwise = 0
    worst = []
    for name, gc in g_conv.items():
        gk = g_chain[name]
        bitwise += int(torch.equal(gk, gc))
        rel = ((gk - gc).norm() / gc.norm().clamp_min(1e-12)).item()
        cos = F.cosine_similarity(gk.flatten().double(), gc.flatten().double(), dim=0).item()
        worst.append((rel, cos, name))
        assert rel <= 5e-2 and cos >= 0.998, f"{name}: rel {rel:.3e} cos {cos:.5f}"
    worst.sort(reverse=True)
    print(f"cfg3 SRGAN step: content loss {l_chain:.6f} vs {l_conv:.6f}; {bitwise}/{len(g_conv)} generator "
          f"gradients bitwise equal; worst {worst[:2]}")
    # measured on MI355X: 490 / 490 bitwise (the trunk kernel and the per-conv launches compute
    # every activation bit for bit alike, and the backward is the same code on both)
    assert bitwise == len(g_conv), f"{len(g_conv) - bitwise} gradients differ (within the bars above)"


def test_cfg3_two_sample_slice_vs_oracle():
    gen = _gen(5)
    batches = data.SyntheticSR(BATCH, HR, seed=3, device=DEV)
    tf = data.GPUTransform(SCALE, hr_norm=True, device=DEV)
    hr, lr = tf(next(batches))
    hr, lr = hr[:2].float(), lr[:2].float()
    sd = {k: v.detach().cpu().clone().float() for k, v in gen.res_net.state_dict().items()}
    params = {k: v.requires_grad_(True) for k, v in sd.items() if v.is_floating_point()}
    y_ref = R.generator(sd, lr.cpu(), num_blocks=BLOCKS, scale=SCALE, enchant=True)
    ref_loss = F.mse_loss(y_ref, hr.cpu())
    ref_loss.backward()

    gen.train()
    loss = F.mse_loss(gen(lr), hr)
    loss.backward()
    torch.cuda.synchronize()
    assert gen.res_net.__dict__["_isr_train_plan"].chain is not None
    assert abs(loss.item() - ref_loss.item()) <= 1e-3 * abs(ref_loss.item()) + 1e-5, (loss.item(), ref_loss.item())
    worst = []
    for name, p in gen.res_net.named_parameters():
        r = params[name].grad.to(DEV)
        rel = ((p.grad - r).norm() / r.norm().clamp_min(1e-12)).item()
        cos = F.cosine_similarity(p.grad.flatten(), r.flatten(), dim=0).item()
        worst.append((rel, cos, name))
        assert rel <= 5e-2 and cos >= 0.998, f"{name}: rel {rel:.3e} cos {cos:.5f}"
    worst.sort(reverse=True)
    print("cfg3 2-sample slice, worst grads vs oracle:", worst[:3])


def test_srgan_d_overlap_same_updates(monkeypatch):
    """train_srgan with the discriminator's forwards + backward on a second stream beside the
    generator's backward and VGG(hr) beside the D(sr) / VGG(sr) forwards (default) updates G and D
    exactly as the serial order (bit for bit)."""
    def run(overlap):
        monkeypatch.setenv("ISR_TRAIN_D_OVERLAP", "1" if overlap else "0")
        torch.manual_seed(0)
        gen = models.SRGAN(2, 0.2, True, SCALE)
        gen.load_state_dict(synth_state_dict(gen.state_dict(), 9))
        gen = gen.to(DEV)
        dis = models.Discriminator(3, 64, 8, 1024).to(DEV)
        dis.use_libisr(True)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            gl = L.gen_loss(device=DEV, beforeAct=True)
        mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
        og = optim.FusedAdam(gen.parameters(), lr=1e-4)
        od = optim.FusedAdam(dis.parameters(), lr=1e-4)
        sg = torch.optim.lr_scheduler.LinearLR(og, 1, 0.01, total_iters=2)
        sd = torch.optim.lr_scheduler.LinearLR(od, 1, 0.01, total_iters=2)
        ema = models.ModelEMA(gen, tau=2)
        ema.ema.to(DEV)
        sc = (torch.amp.GradScaler("cuda", enabled=False), torch.amp.GradScaler("cuda", enabled=False))
        tf = data.GPUTransform(SCALE, hr_norm=True, mean=mean, std=std, device=DEV)
        batches = data.SyntheticSR(4, 128, seed=5, device=DEV)
        losses = trainer.train_srgan(gen, ema, dis, batches, tf, gl, og, od, sc, (sg, sd), 0, None, mean=mean,
                                     std=std, steps=2, log_every=1)
        torch.cuda.synchronize()
        return losses, [p.detach().clone() for p in gen.parameters()], [p.detach().clone() for p in dis.parameters()]

    l0, g0, d0 = run(False)
    l1, g1, d1 = run(True)
    assert l0 == l1
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))
    assert all(torch.equal(a, b) for a, b in zip(d0, d1))


def test_srgan_default_mode_step_vs_oracle():
    """One trainer.train_srgan step of SRGAN(16, 0.2, enchant=False, x2) — train.py's default mode,
    started as train.py starts it from the pretrained --resnet generator (the committed x2 weights):
    BatchNorm ResNet generator (train-mode batch statistics), content loss = MSE of VGG19 conv5_4
    AFTER its ReLU, + 1e-3 BCE adversarial — on 2 crops of 128² HR, against the fp32 oracle:
    * the generator output (train-mode BN) vs oracle.ref_cpu.generator(train_bn=True): >= 40 dB;
    * the logged content / adversarial losses vs the oracle's content_loss (utils/loss.py:16-24) on
      the oracle's own SR image, the stock fp32 discriminator modules and the same VGG weights:
      rel <= 3 % (the VGG feature bar of test_gpu_vgg.py);
    * every generator parameter gradient of the step vs autograd of the oracle generator fed the
      step's own upstream gradient dL/dSR (the VGG + discriminator input gradients, pinned by
      test_gpu_vgg.py / test_gpu_disc.py): rel L2 <= max(5e-2, 1.3 x torch bf16 autocast's own
      rel L2 + 0.02) (test_gpu_train.py's bar, widened as test_gpu_denoise.py's for BatchNorm
      graphs), and the cosine that rel bar implies (>= min(0.998, 1 - bar^2 / 2))."""
    import copy

    torch.manual_seed(0)
    # train.py's default mode starts SRGAN from the --resnet checkpoint (SRGAN.init_weight loads its
    # EMA generator, utils/models.py:659-665): the committed trained ResNet(16, 0.2, x2)
    gen = models.SRGAN(16, 0.2, False, 2)
    gen.res_net.load_state_dict(checkpoint.load_module_state(
        __import__("pathlib").Path(__file__).parent / "golden" / "trained_resnet_x2.safetensors"))
    gen = gen.to(DEV)
    assert isinstance(gen.res_net, models.ResNet)  # the BatchNorm generator
    dis = models.Discriminator(3, 64, 8, 1024).to(DEV)
    dis.use_libisr(True)
    dis_ref = copy.deepcopy(dis).cpu().use_libisr(False).train()
    sd_g = {k: v.detach().cpu().clone().float() for k, v in gen.res_net.state_dict().items()}
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        gl = L.gen_loss(device=DEV, beforeAct=False)
    sd_vgg = {k: v.detach().cpu().float() for k, v in gl.vgg_net.state_dict().items()}
    mean, std = list(data.IMAGENET_MEAN), list(data.IMAGENET_STD)
    og = optim.FusedAdam(gen.parameters(), lr=1e-4)
    od = optim.FusedAdam(dis.parameters(), lr=1e-4)
    sg = torch.optim.lr_scheduler.LinearLR(og, 1, 0.01, total_iters=1)
    sdl = torch.optim.lr_scheduler.LinearLR(od, 1, 0.01, total_iters=1)
    ema = models.ModelEMA(gen, tau=1)
    ema.ema.to(DEV)
    sc = (torch.amp.GradScaler("cuda", enabled=False), torch.amp.GradScaler("cuda", enabled=False))
    tf = data.GPUTransform(2, hr_norm=True, mean=mean, std=std, device=DEV)
    crops = next(data.SyntheticSR(2, 128, seed=7, device=DEV, kind="leaves"))
    hr, lr = tf(crops)
    trainer.TAPS = []
    try:
        trainer.train_srgan(gen, ema, dis, iter([crops]), tf, gl, og, od, sc, (sg, sdl), 0, None, mean=mean,
                            std=std, steps=1, log_every=1)
        torch.cuda.synchronize()
        taps = {name: [t.cpu() if t is not None else None for t in ts] for name, ts in trainer.TAPS}
    finally:
        trainer.TAPS = None
    sr_hip, gy = taps["sr"][0], taps["sr_grad"][0].float()
    perceptual, adversarial, content = (t.float().item() for t in taps["g_loss"])

    # oracle: the same generator (train-mode BN), the same loss on its own SR image
    pnames = {k for k, _ in gen.res_net.named_parameters()}
    params = {k: v.requires_grad_(True) for k, v in sd_g.items() if k in pnames}
    sr_ref = R.generator(sd_g, lr.float().cpu(), num_blocks=16, scale=2, enchant=False, train_bn=True)
    agree = R.psnr(sr_hip, sr_ref.detach())
    m, s_ = torch.tensor(mean).view(1, 3, 1, 1), torch.tensor(std).view(1, 3, 1, 1)
    with torch.no_grad():
        srn = ((sr_ref.detach() + 1) / 2 - m) / s_
        for p in dis_ref.parameters():
            p.requires_grad_(False)
        p_ref, a_ref, c_ref = R.content_loss(sd_vgg, srn, hr.float().cpu(), dis_ref(srn), before_act=False)
    print(f"default SRGAN mode: SR agreement {agree:.2f} dB; content {content:.6f} vs {c_ref.item():.6f}, "
          f"adversarial {adversarial:.5f} vs {a_ref.item():.5f}")
    assert agree >= 40.0, agree
    assert abs(content - c_ref.item()) <= 3e-2 * abs(c_ref.item()), (content, c_ref.item())
    assert abs(adversarial - a_ref.item()) <= 3e-2 * abs(a_ref.item()) + 1e-3, (adversarial, a_ref.item())
    assert abs(perceptual - (content + 1e-3 * adversarial)) <= 1e-5 * abs(perceptual) + 1e-7

    # generator gradients for the step's own upstream gradient; the yardstick beside the fixed bar is
    # the error torch's own bf16 autocast makes on the same graph (the reference trains under
    # autocast, train.py:54; as tests/test_gpu_denoise.py): train-mode BatchNorm subtracts batch
    # means in its backward, so the BN generator's gradients carry more relative rounding error
    # than the BN-free EResNet's (test_gpu_train.py)
    sr_ref.backward(gy)
    sd_amp = {k: v.detach().clone().to(DEV) for k, v in sd_g.items()}
    p_amp = {k: v.requires_grad_(True) for k, v in sd_amp.items() if k in pnames}
    with torch.autocast("cuda", dtype=torch.bfloat16):
        sr_amp = R.generator(sd_amp, lr.float(), num_blocks=16, scale=2, enchant=False, train_bn=True)
    sr_amp.float().backward(gy.to(DEV))
    names = [k for k, _ in gen.named_parameters()]
    worst = []
    for name, g in zip(names, taps["g_grad"]):
        key = name[len("res_net."):]
        r = params[key].grad
        rel = ((g - r).norm() / r.norm().clamp_min(1e-12)).item()
        ga = p_amp[key].grad.cpu()
        rel_amp = ((ga - r).norm() / r.norm().clamp_min(1e-12)).item()
        cos = F.cosine_similarity(g.flatten().double(), r.flatten().double(), dim=0).item()
        cos_amp = F.cosine_similarity(ga.flatten().double(), r.flatten().double(), dim=0).item()
        worst.append((round(rel, 4), round(rel_amp, 4), round(cos, 5), name))
        bar = max(5e-2, 1.3 * rel_amp + 0.02)
        # the cosine bar implied by the rel bar (1 - cos ~ rel^2 / 2 for a small error)
        assert rel <= bar and cos >= min(0.998, 1 - bar ** 2 / 2), \
            f"{name}: rel {rel:.3e} (bf16 autocast {rel_amp:.3e}) cos {cos:.5f} (autocast {cos_amp:.5f})"
    worst.sort(reverse=True)
    print("default SRGAN mode, worst generator gradients vs oracle autograd (rel, autocast rel, cos):", worst[:4])
