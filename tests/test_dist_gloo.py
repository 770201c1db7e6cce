"""Multi-process (world_size 2, gloo on CPU) tests of the trajectory-sharded DP logic.
The GPU kernels cannot run here; the collective, sharding and gradient-bucket logic can."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fet_ode_amd.dist as D
    torch.manual_seed(0)
    # reference-style linear model in plain torch (CPU): the shard/all-reduce logic is what's tested
    w = torch.nn.Parameter(torch.randn(3, 2))
    if rank == 1:
        with torch.no_grad():
            w.add_(1.0)               # diverged init -> broadcast must repair it
    m = torch.nn.Module()
    m.w = w
    D.broadcast_parameters(m)
    xg = torch.arange(10, dtype=torch.float32).reshape(5, 2)   # 5 trajectories, 2 ranks: 3 + 2
    lo, hi = D.shard_bounds(5, rank, world)
    x = D.shard(xg)
    assert x.shape[0] == hi - lo
    loss = (x @ w.T).square().mean()
    loss.backward()
    D.allreduce_gradients([w], weights=(hi - lo) / 5)
    q.put((rank, w.detach().clone(), w.grad.clone()))
    dist.destroy_process_group()


def test_sharded_gradient_equals_global_gradient():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, w0, g0), (_, w1, g1) = res
    assert torch.equal(w0, w1)
    torch.manual_seed(0)
    w = torch.randn(3, 2, requires_grad=True)
    xg = torch.arange(10, dtype=torch.float32).reshape(5, 2)
    (xg @ w.T).square().mean().backward()
    assert torch.allclose(g0, w.grad, atol=1e-5) and torch.allclose(g1, w.grad, atol=1e-5)


def test_shard_bounds_rules():
    import fet_ode_amd.dist as D
    assert [D.shard_bounds(4096, r, 8) for r in (0, 7)] == [(0, 512), (3584, 4096)]
    assert [D.shard_bounds(5, r, 2) for r in (0, 1)] == [(0, 3), (3, 5)]
    with pytest.raises(ValueError):
        D.shard_bounds(3, 2, 3)          # shard of 1 flips the ferro first-call rule
    assert D.shard_bounds(1, 0, 1) == (0, 1)
