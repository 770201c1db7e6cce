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


# ---------------------------------------------------------------------------------------------
# sharded dopri5 under autograd: the norm all-reduce and its backward (dopri5._NormAllReduce)
# ---------------------------------------------------------------------------------------------

def _field64():
    torch.manual_seed(4)
    W1 = torch.nn.Parameter(torch.randn(2, 16, dtype=torch.float64) * 0.7)
    W2 = torch.nn.Parameter(torch.randn(16, 2, dtype=torch.float64) * 0.5)
    b = torch.nn.Parameter(torch.randn(2, dtype=torch.float64) * 0.1)
    return [W1, W2, b], (lambda tt, y: torch.tanh(y @ W1) @ W2 + b - 0.3 * y)


def _y0_64():
    return torch.linspace(-1.0, 1.5, 12, dtype=torch.float64).reshape(6, 2)


def _sharded_grad(rank, world, sizes, group_opt):
    from fet_ode_amd.dopri5 import _Dopri5Grad
    ps, f = _field64()
    y0g = _y0_64()
    lo = sum(sizes[:rank])
    y0 = y0g[lo:lo + sizes[rank]]
    opts = {"norm_group": group_opt} if group_opt else {}
    s = _Dopri5Grad(f, y0, 1e-6, 1e-8, opts, False, check_device=False)
    sol = s.integrate(torch.tensor([0.0, 0.4, 1.0], dtype=torch.float64))
    # this shard's share of the global mean loss (odeint_sharded docstring)
    loss = (sol * sol.flip(-1)).sum() / (sol.shape[0] * y0g.shape[0] * sol.shape[2])
    loss.backward()
    return sol.detach(), [p.grad.clone() for p in ps], [(a[1], a[3]) for a in s.attempts]


def _dopri_worker(rank, world, port, q, sizes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sol, grads, att = _sharded_grad(rank, world, sizes, "world")
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)           # == allreduce_gradients(average=False)
        q.put((rank, sol, flat, att))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [(3, 3), (4, 2)])
def test_sharded_dopri5_gradient_through_step_control_fp64(sizes):
    """fp64 on CPU (no rounding noise): 2 ranks with the global-batch RMS norm take the single
    process's steps, and the summed gradients equal the single-process gradient — including the
    d loss / d dt terms that cross ranks (the all-reduced norm adjoint), with unequal shards too."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dopri_worker, args=(r, 2, port, q, sizes)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, s0, g0, a0), (_, s1, g1, a1) = res
    sol, grads, att = _sharded_grad(0, 1, (6,), None)
    ref = torch.cat([g.reshape(-1) for g in grads])
    assert a0 == a1 and [a[1] for a in a0] == [a[1] for a in att] and len(att) > 3
    for (d0, _), (dr, _) in zip(a0, att):
        assert abs(d0 - dr) <= 1e-12 * abs(dr)
    assert torch.allclose(torch.cat([s0, s1], dim=1), sol, rtol=1e-12, atol=1e-14)
    assert torch.equal(g0, g1)
    assert ((g0 - ref).norm() / ref.norm()).item() <= 1e-10, ((g0 - ref).norm() / ref.norm()).item()


def _views_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fet_ode_amd.dist as D
    # gradients that are views of one flat buffer (what the fused backward hands autograd):
    # reduced in place, no copies; a mixed set falls back to the flatten path
    ps = [torch.nn.Parameter(torch.zeros(3, 2)), torch.nn.Parameter(torch.zeros(4))]
    flat = torch.arange(10, dtype=torch.float32) * (rank + 1)
    # detached, as AccumulateGrad stores them (their ._base is None; the storage is still shared)
    ps[0].grad, ps[1].grad = flat[:6].view(3, 2).detach(), flat[6:].detach()
    sf = D._shared_flat([p.grad for p in ps])
    assert sf is not None and sf.data_ptr() == flat.data_ptr() and sf.numel() == 10
    # a gap or a reordering is not one run
    assert D._shared_flat([ps[1].grad, ps[0].grad]) is None
    assert D._shared_flat([flat[:4], flat[6:]]) is None
    D.allreduce_gradients(ps)
    q.put((rank, flat.clone(), ps[0].grad.data_ptr() == flat.data_ptr()))
    dist.destroy_process_group()


def test_allreduce_in_place_on_shared_gradient_buffer():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_views_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = torch.arange(10, dtype=torch.float32) * 1.5   # mean of rank 0 (x1) and rank 1 (x2)
    for _, flat, still_view in res:
        assert still_view and torch.equal(flat, exp)


def _bcast_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fet_ode_amd as F
    import fet_ode_amd.dist as D
    torch.manual_seed(rank)          # deliberately different weights per rank
    m = F.KANFET([2, 10, 2], grid_size=5)
    # per-rank hysteresis memory of unequal shards (B_local = 3 + rank): stays this rank's own
    mem = [torch.full((3 + rank, l.ferro.in_dim), float(rank + 1)) for l in m.layers]
    for l, p in zip(m.layers, mem):
        l.ferro._prev = p.clone()
    D.broadcast_parameters(m)
    kept = all(torch.equal(l.ferro._prev, p) for l, p in zip(m.layers, mem))
    q.put((rank, ({k: v.detach().clone().numpy() for k, v in m.named_parameters()}, kept)))
    dist.destroy_process_group()


def test_broadcast_parameters_gives_every_rank_rank0_weights():
    """dist.broadcast_parameters (the efficient_kan init is not bitwise reproducible across
    processes, so DP ranks take rank 0's weights and persistent buffers); each rank's hysteresis
    memory — unequal shard sizes — is left alone (no mismatched collective, no overwrite)."""
    import socket
    import numpy as np
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert res[0][1] and res[1][1]
    for k in res[0][0]:
        assert np.array_equal(res[0][0][k], res[1][0][k]), k


def test_host_dopri5_grad_matches_oracle_fp64():
    """The single-device _Dopri5Grad loop (host copies of t / dt, one read-back per attempt, dense
    output formed only where an output needs it) against the oracle's restated torchdiffeq solver
    under autograd, fp64 on the CPU: the same attempts, solution and gradients (incl. d / d dt)."""
    from fet_ode_amd.dopri5 import _Dopri5Grad
    from oracle import torch_ref as O
    t = torch.tensor([0.0, 0.05, 0.4, 0.41, 1.0], dtype=torch.float64)
    res = []
    for impl in ("host", "oracle"):
        ps, f = _field64()
        y0 = _y0_64().requires_grad_(True)
        if impl == "host":
            s = _Dopri5Grad(f, y0, 1e-6, 1e-8, {}, False, check_device=False)
            sol = s.integrate(t)
            n = s.nfev
        else:
            tr = O.Dopri5Trace()
            sol = O.odeint(f, y0, t, rtol=1e-6, atol=1e-8, trace=tr)
            n = tr.nfev
        loss = (sol * sol.flip(-1)).sum()
        loss.backward()
        res.append((sol.detach(), [p.grad.clone() for p in ps] + [y0.grad.clone()], n))
    (s0, g0, n0), (s1, g1, n1) = res
    assert n0 == n1
    assert torch.allclose(s0, s1, rtol=1e-12, atol=1e-14)
    for a, b in zip(g0, g1):
        assert torch.allclose(a, b, rtol=1e-9, atol=1e-12), (a, b)
