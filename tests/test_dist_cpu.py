"""Multi-process (gloo, world size 2) checks of the data-parallel gradient
averaging used by train.py (train_engine.allreduce_grads) — same math as DDP."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from image_super_resolution_amd.train_engine import allreduce_grads
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
        x = torch.randn(8, 4)[rank * 4:(rank + 1) * 4]
        with torch.enable_grad():
            m(x).pow(2).sum().backward()
        allreduce_grads(m.parameters())
        q.put((rank, [p.grad.numpy().copy() for p in m.parameters()]))
    finally:
        dist.destroy_process_group()


def test_allreduce_grads_matches_full_batch_mean():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: [torch.from_numpy(a) for a in v] for r, v in (q.get(timeout=120) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    x = torch.randn(8, 4)
    with torch.enable_grad():
        (m(x[:4]).pow(2).sum() + m(x[4:]).pow(2).sum()).div(2).backward()
    for r in (0, 1):
        for g, p in zip(res[r], m.parameters()):
            torch.testing.assert_close(g, p.grad)


def _mean_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from image_super_resolution_amd.train_engine import allreduce_mean
        ts = [torch.full((3, 2), float(rank + 1)), torch.arange(4.0) * (rank + 1), torch.tensor([float(rank)])]
        q.put((rank, [t.numpy().copy() for t in allreduce_mean(ts)]))
    finally:
        dist.destroy_process_group()


def test_allreduce_mean_flat_bucket():
    """The flat one-bucket mean used by the Denoise training plan (denoise._DenoiseFn)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_mean_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: [torch.from_numpy(a) for a in v] for r, v in (q.get(timeout=120) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        a, b, c = res[r]
        torch.testing.assert_close(a, torch.full((3, 2), 1.5))
        torch.testing.assert_close(b, torch.arange(4.0) * 1.5)
        torch.testing.assert_close(c, torch.tensor([0.5]))
