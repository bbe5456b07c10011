"""Multi-process (gloo, world size 2) checks of the data-parallel gradient
averaging used by train.py (train_engine.allreduce_grads) — same math as DDP."""
import os
import socket

import pytest
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


def _guard_worker(rank, world, port, q, variant="chain"):
    """A trunk give-up on rank 1 only: the step guard every rank's optimiser reads must say
    "skip" on both ranks, and the epoch-end check must raise on both (the gradients
    are averaged before the guard is read, so a per-rank guard lets peers apply poisoned ones)."""
    import types

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from image_super_resolution_amd.engine import ChainFailed
        from image_super_resolution_amd.train_engine import enable_grad_allreduce, step_guard_ptr, verify_chains

        state = torch.zeros(8, dtype=torch.int32)
        if rank == 1:
            state[2] = 1  # sticky give-up count 1, accepted count 0

        def verify():
            if int(state[2]) != int(state[3]):
                state[3] = state[2]
                raise ChainFailed("gave up")

        chain = types.SimpleNamespace(state=state, guard_ptr=state.data_ptr() + 8, verify=verify)
        if rank == 0 and variant == "fallback":  # rank 0's trunk ran per conv: no chain, still votes
            chain = None
        if rank == 0 and variant == "error":  # rank 0's check fails with another error: votes bad, re-raises
            def broken():
                raise RuntimeError("HIP error in the chain check")
            chain.verify = broken
        gen = torch.nn.Linear(2, 2)
        gen.__dict__["_isr_train_plan"] = types.SimpleNamespace(chain=chain, device=torch.device("cpu"))
        enable_grad_allreduce(gen, True)
        ptr = step_guard_ptr(gen)
        g = gen.__dict__["_isr_train_plan"]._global_guard
        assert ptr == g.data_ptr()
        words = g.tolist()
        raised = False
        try:
            verify_chains(gen)
        except ChainFailed:
            raised = True
        except RuntimeError as e:
            raised = "other: " + str(e)
        # after the report, the accepted count caught up: the next step's guard lets updates run
        ptr2 = step_guard_ptr(gen)
        q.put((rank, words, raised, g.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("variant", ["chain", "fallback", "error"])
def test_trunk_give_up_guard_is_global_under_data_parallel(variant):
    """variant 'fallback': rank 0 built no persistent chain (per-conv trunk) — it still joins both
    collectives; 'error': rank 0's chain check raises another error — it votes 'bad', its peer
    raises ChainFailed, rank 0 re-raises its own error, and neither blocks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_guard_worker, args=(r, 2, port, q, variant)) for r in range(2)]
    for p in ps:
        p.start()
    res = {r: (w, raised, w2) for r, w, raised, w2 in (q.get(timeout=120) for _ in range(2))}
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        words, raised, after = res[r]
        assert words[0] != words[1], f"rank {r}: the guard must skip the step (words {words})"
        if variant == "error" and r == 0:
            assert raised == "other: HIP error in the chain check", raised
        else:
            assert raised is True, f"rank {r}: the epoch-end check must raise ChainFailed on every rank ({raised})"
        assert after[0] == after[1], f"rank {r}: once reported, later steps update again ({after})"
