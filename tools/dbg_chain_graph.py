import sys, torch
sys.path.insert(0, "/root/repo")
from image_super_resolution_amd import engine, models
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict
dev = torch.device("cuda")
sd = synth_state_dict(models.ResNet(16, 0.2, scaleRate=4).state_dict(), seed=0)
gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, device=dev, f16=False)
lr, _ = synth_lr_batch(16, 128, 128, seed=1234)
x = normalize(lr).to(dev).contiguous()
mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
plan = engine.GeneratorPlan(gw, 16, 128, 128, dev, False, False, mean, std, chain=True)
out = torch.empty(plan.out_shape, device=dev)
for i in range(3):
    plan.run(x, out); torch.cuda.synchronize()
    st = plan.chain.state.cpu()
    print("eager", i, "fail", int(st[0]), "progress min/max", int(st[4:4+512].min()), int(st[4:4+512].max()), flush=True)
g = engine.GraphedPlan(plan, x, out)
st = plan.chain.state.cpu(); print("after capture warmup fail", int(st[0]), int(st[4:516].min()), int(st[4:516].max()), flush=True)
for i in range(3):
    g.run(); torch.cuda.synchronize()
    st = plan.chain.state.cpu()
    p = st[4:4+512]
    print("graph", i, "fail", int(st[0]), "progress min/max", int(p.min()), int(p.max()), "hist", torch.bincount(p.clamp(0,240).long(), minlength=241).nonzero().flatten().tolist()[:10], flush=True)
ref = torch.empty_like(out)
plan.run(x, ref); torch.cuda.synchronize()
print("eager state[:8]", plan.chain.state[:8].tolist())
for i in range(3):
    plan.chain.state.fill_(7); torch.cuda.synchronize()
    g.run(); torch.cuda.synchronize()
    print("graph", i, "state[:8]", plan.chain.state[:8].tolist(), "state[-4:]", plan.chain.state[-4:].tolist(), "equal", torch.equal(out, ref), flush=True)
