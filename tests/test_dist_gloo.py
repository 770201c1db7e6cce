"""Multi-process (world_size 2, gloo on CPU) tests of the trajectory-sharded DP logic.
The GPU kernels cannot run here; the collective, sharding and gradient-bucket logic can.

Harness (round 6): the ranks rendezvous through a file (``init_method="file://..."`` in pytest's
tmp_path: no port to race for) and hand their results back as numpy arrays.  Round 5's harness put
torch tensors on a torch.multiprocessing queue, which moves them through shared memory whose file
descriptors the SENDING process serves; a worker that had already exited when the parent unpickled
its result made ``q.get`` fail (one failure in 17 runs, after 8.4 s)."""
import multiprocessing
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist


def _init(rank, world, init_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)


def _spawn(target, world, tmp_path, *args):
    """Run target(rank, world, init_file, q, *args) on `world` spawned ranks; returns their queue
    items (plain Python / numpy objects) sorted by rank, after every rank exited with status 0."""
    ctx = multiprocessing.get_context("spawn")
    q = ctx.Queue()
    init_file = str(tmp_path / f"rdzv_{target.__name__}")
    procs = [ctx.Process(target=target, args=(r, world, init_file, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=120) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
    codes = [p.exitcode for p in procs]
    assert codes == [0] * world, f"rank exit codes {codes}"
    return sorted(res, key=lambda r: r[0])


def _np(t):
    return t.detach().cpu().clone().numpy()


def _worker(rank, world, init_file, q):
    _init(rank, world, init_file)
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
    q.put((rank, _np(w), _np(w.grad)))
    dist.destroy_process_group()


def test_sharded_gradient_equals_global_gradient(tmp_path):
    (_, w0, g0), (_, w1, g1) = _spawn(_worker, 2, tmp_path)
    assert np.array_equal(w0, w1), f"rank weights differ after broadcast: {w0} vs {w1}"
    torch.manual_seed(0)
    w = torch.randn(3, 2, requires_grad=True)
    xg = torch.arange(10, dtype=torch.float32).reshape(5, 2)
    (xg @ w.T).square().mean().backward()
    ref = w.grad.numpy()
    for r, g in ((0, g0), (1, g1)):
        assert np.allclose(g, ref, atol=1e-5), f"rank {r} all-reduced gradient {g} vs global {ref}"


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


def _dopri_worker(rank, world, init_file, q, sizes):
    torch.set_num_threads(1)            # one fixed reduction order per rank
    _init(rank, world, init_file)
    try:
        sol, grads, att = _sharded_grad(rank, world, sizes, "world")
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)           # == allreduce_gradients(average=False)
        q.put((rank, _np(sol), _np(flat), att))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("sizes", [(3, 3), (4, 2)])
def test_sharded_dopri5_gradient_through_step_control_fp64(sizes, tmp_path):
    """fp64 on CPU (no rounding noise): 2 ranks with the global-batch RMS norm take the single
    process's steps, and the summed gradients equal the single-process gradient — including the
    d loss / d dt terms that cross ranks (the all-reduced norm adjoint), with unequal shards too."""
    (_, s0, g0, a0), (_, s1, g1, a1) = _spawn(_dopri_worker, 2, tmp_path, sizes)
    sol, grads, att = _sharded_grad(0, 1, (6,), None)
    ref = torch.cat([g.reshape(-1) for g in grads]).numpy()
    assert a0 == a1, f"the ranks took different attempts: {a0} vs {a1}"
    assert [a[1] for a in a0] == [a[1] for a in att], \
        f"accept pattern sharded {[a[1] for a in a0]} vs single process {[a[1] for a in att]}"
    assert len(att) > 3, f"only {len(att)} attempts"
    for j, ((d0, _), (dr, _)) in enumerate(zip(a0, att)):
        assert abs(d0 - dr) <= 1e-12 * abs(dr), f"attempt {j}: dt sharded {d0!r} vs single process {dr!r}"
    sol_sh = np.concatenate([s0, s1], axis=1)
    assert np.allclose(sol_sh, sol.detach().numpy(), rtol=1e-12, atol=1e-14), \
        f"solution max abs diff {np.abs(sol_sh - sol.detach().numpy()).max()}"
    assert np.array_equal(g0, g1), f"all-reduced gradients differ between ranks: max {np.abs(g0 - g1).max()}"
    rel = np.linalg.norm(g0 - ref) / np.linalg.norm(ref)
    assert rel <= 1e-10, f"summed sharded gradient vs single process: relative {rel}"


def _views_worker(rank, world, init_file, q):
    _init(rank, world, init_file)
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
    q.put((rank, _np(flat), ps[0].grad.data_ptr() == flat.data_ptr()))
    dist.destroy_process_group()


def test_allreduce_in_place_on_shared_gradient_buffer(tmp_path):
    res = _spawn(_views_worker, 2, tmp_path)
    exp = np.arange(10, dtype=np.float32) * 1.5   # mean of rank 0 (x1) and rank 1 (x2)
    for r, flat, still_view in res:
        assert still_view, f"rank {r}: the gradient is no longer a view of the flat buffer"
        assert np.array_equal(flat, exp), f"rank {r}: {flat} vs {exp}"


def _bcast_worker(rank, world, init_file, q):
    _init(rank, world, init_file)
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


def test_broadcast_parameters_gives_every_rank_rank0_weights(tmp_path):
    """dist.broadcast_parameters (the efficient_kan init is not bitwise reproducible across
    processes, so DP ranks take rank 0's weights and persistent buffers); each rank's hysteresis
    memory — unequal shard sizes — is left alone (no mismatched collective, no overwrite)."""
    res = dict(_spawn(_bcast_worker, 2, tmp_path))
    assert res[0][1] and res[1][1], "a rank's hysteresis memory was overwritten by the broadcast"
    for k in res[0][0]:
        assert np.array_equal(res[0][0][k], res[1][0][k]), f"parameter {k} differs between ranks"


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


@pytest.mark.parametrize("nan_at", [3, 9, 15])
def test_host_dopri5_grad_dt_underflow_checked_before_evaluating(nan_at):
    """the single-device _Dopri5Grad loop reads each attempt's dt back together with its
    ratio, so its dt-underflow assert could only run after the attempt's six evaluations — six
    evaluations more than torchdiffeq makes, which on a stateful (hysteretic) field leaves a later
    prev_x.  A field that turns NaN after `nan_at` calls makes the ratio NaN, the next dt NaN, and
    the next attempt's top assert fire: the host loop must fail with the oracle's message after
    exactly the oracle's number of field evaluations."""
    from fet_ode_amd.dopri5 import _Dopri5Grad
    from oracle import torch_ref as O
    t = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
    calls = {}
    for impl in ("host", "oracle"):
        n = [0]

        def f(tt, y):
            n[0] += 1
            return -y * (float("nan") if n[0] > nan_at else 1.0)

        y0 = _y0_64()
        with pytest.raises(AssertionError, match="underflow in dt"):
            if impl == "host":
                _Dopri5Grad(f, y0, 1e-6, 1e-8, {}, False, check_device=False).integrate(t)
            else:
                O.odeint(f, y0, t, rtol=1e-6, atol=1e-8)
        calls[impl] = n[0]
    assert calls["host"] == calls["oracle"], f"field evaluations before the assert: {calls}"
