import time, torch, statistics, sys
sys.path.insert(0, '.')
import bench
from image_super_resolution_amd import engine, models, ops
from image_super_resolution_amd.weights import normalize, synth_lr_batch, synth_state_dict
dev = torch.device('cuda')
tm = models.ResNet(16, 0.2, scaleRate=4)
sd = synth_state_dict(tm.state_dict(), seed=0)
gw = engine.pack_generator({k: v.to(dev) for k, v in sd.items()}, enchant=False, add_rate=0.2, device=dev)
lr, hr = synth_lr_batch(16, 128, 128, seed=1234, scale=4)
x = normalize(lr).to(dev).contiguous()
plan = engine.get_plan(gw, x, False, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
out = torch.empty(plan.out_shape, dtype=plan.out_dtype, device=dev)
for _ in range(5): plan.run(x, out)
def around(tag):
    if tag == bench.DOMINANT:
        return (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
res = {"plain": [], "events": []}
for r in range(6):
    for k in res:
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(20): plan.run(x, out, around=around if k == "events" else None)
        torch.cuda.synchronize(); res[k].append((time.perf_counter() - t0) / 20 * 1e3)
print({k: round(statistics.median(v), 3) for k, v in res.items()})
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    plan.run(x, out); torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        plan.run(x, out)
torch.cuda.synchronize()
ref = out.clone(); plan.run(x, out); torch.cuda.synchronize()
eager = out.clone()
out.zero_()
with torch.cuda.stream(s):
    g.replay()
torch.cuda.synchronize()
print("graph==eager", torch.equal(out, eager))
res = {"plain": [], "graph": []}
for r in range(6):
    for k in res:
        torch.cuda.synchronize(); t0 = time.perf_counter()
        if k == "graph":
            with torch.cuda.stream(s):
                for _ in range(20): g.replay()
        else:
            for _ in range(20): plan.run(x, out)
        torch.cuda.synchronize(); res[k].append((time.perf_counter() - t0) / 20 * 1e3)
print({k: round(statistics.median(v), 3) for k, v in res.items()})
