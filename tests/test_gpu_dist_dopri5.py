"""Trajectory-sharded dopri5 (dist.odeint_sharded) on the GPU: 2 ranks on cuda:0 (gloo carries
the two-word norm all-reduce) take exactly the steps a single device takes on the global batch,
and their shards concatenate to the single-device solution (SURVEY §8e caveat 2)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, golden_sd, load_golden

T_GRID = [0.0, 0.25, 0.5]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(F, sd):
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    return m.to("cuda:0")


def _worker(rank, world, port, q, resident=False, bench=None):
    import sys
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fet_ode_amd as F
    import fet_ode_amd.dist as D
    D.set_resident_sharded(resident)
    if bench is not None:
        m, y0g, t, tol = _bench_problem(F, {k: torch.from_numpy(v) for k, v in bench.items()})
    else:
        g = load_golden("traj_kanfet")
        m = _model(F, golden_sd(g))
        y0g, t, tol = torch.from_numpy(g["y0_B64"]), torch.tensor(T_GRID, dtype=torch.float64), (1e-3, 1e-4)
    y0 = D.shard(y0g).to("cuda:0")
    with torch.no_grad():
        sol = D.odeint_sharded(lambda tt, yy: m(yy), y0, t, rtol=tol[0], atol=tol[1])
    s = F.dopri5.dopri5_solve.last
    took = type(s).__name__
    q.put((rank, sol.cpu().numpy(), [(a[1], a[2], a[3]) for a in s.attempts], s.nfev, took, s.n_attempts
           if hasattr(s, "n_attempts") else len(s.attempts)))
    dist.destroy_process_group()


def _bench_problem(F, sd=None):
    """The north-star call's tolerances (torchdiffeq defaults rtol 1e-7, atol 1e-9) on the bench
    field and 35-point grid, global batch 2048 (two ranks' grids share one GPU here).  The weights
    come from the parent: the efficient_kan init (curve2coeff's lstsq) is not bitwise reproducible
    across processes, in the reference as here, so ranks never re-create them."""
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5)
    if sd is not None:
        m.load_state_dict(sd)
    m = m.to("cuda:0")
    g = torch.Generator().manual_seed(0)
    y0 = (0.5 + 2.5 * torch.rand(2048, 2, generator=g)).to(torch.float32)
    return m, y0, torch.tensor(np.linspace(0, 3.5, 35)), (1e-7, 1e-9)


def _run_ranks(resident, bench=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, resident, bench)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


@pytest.mark.gpu
def test_sharded_resident_dopri5_reproduces_single_device_exactly(dev):
    """The north-star default call (dopri5 at rtol 1e-7 / atol 1e-9, thousands of attempts) sharded
    over 2 ranks, each ONE resident launch whose exchange workgroup sums the norms across the ranks
    (fetode_integrate_dopri5_xrank; both ranks on cuda:0, the inboxes IPC-mapped between the two
    processes): the same attempts, accept pattern and nfev as one device on the global batch."""
    import fet_ode_amd as F
    m, y0, t, tol = _bench_problem(F)
    sd = {k: v.detach().cpu().numpy().copy() for k, v in m.state_dict().items()}
    with torch.no_grad():
        ref = F.odeint(F.autonomous(m), y0.to(dev), t, rtol=tol[0], atol=tol[1]).cpu()
    s = F.dopri5.dopri5_solve.last
    assert type(s).__name__ == "ResidentSolve"
    ref_att = [(a[1], a[2], a[3]) for a in s.attempts]
    (_, s0, a0, n0, k0, na0), (_, s1, a1, n1, k1, na1) = _run_ranks(True, bench=sd)
    s0, s1 = torch.from_numpy(s0), torch.from_numpy(s1)
    assert k0 == k1 == "ResidentSolve"                     # the one-launch path on both ranks
    assert na0 == na1 == s.n_attempts and n0 == n1 == s.nfev, (na0, s.n_attempts, n0, s.nfev)
    # equal even shards are whole leaves of the single-device reduction tree: bitwise the same
    # norms, so the same attempt record and the same solution bit for bit
    assert a0 == a1 == ref_att
    sol = torch.cat([s0, s1], dim=1)
    assert torch.equal(sol, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("resident", [False, True], ids=["host-loop", "resident"])
def test_sharded_dopri5_matches_single_device(dev, kernel_switch, resident):
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    m = _model(F, golden_sd(g))
    with torch.no_grad(), F.closure_fusion(False):   # the host-driven solver (its attempt record)
        ref = F.odeint(lambda tt, yy: m(yy), torch.from_numpy(g["y0_B64"]).to(dev),
                       torch.tensor(T_GRID, dtype=torch.float64), rtol=1e-3, atol=1e-4).cpu()
    s = F.dopri5.dopri5_solve.last
    ref_att = [(a[1], a[2], a[3]) for a in s.attempts]

    (_, s0, a0, n0, k0, _), (_, s1, a1, n1, k1, _) = _run_ranks(resident)
    s0, s1 = torch.from_numpy(s0), torch.from_numpy(s1)
    assert k0 == k1 == ("ResidentSolve" if resident else "_Dopri5")
    assert a0 == a1 and n0 == n1                    # both ranks took identical steps
    if resident:   # equal even shards of 64: whole leaves, so bitwise the single-device resident solve
        kernel_switch(False)   # on v4, as the sharded kernels (small single-device batches take v6)
        with torch.no_grad():
            one = F.odeint(F.autonomous(_model(F, golden_sd(g))), torch.from_numpy(g["y0_B64"]).to(dev),
                           torch.tensor(T_GRID, dtype=torch.float64), rtol=1e-3, atol=1e-4).cpu()
        so = F.dopri5.dopri5_solve.last
        assert a0 == [(a[1], a[2], a[3]) for a in so.attempts] and n0 == so.nfev
        assert torch.equal(torch.cat([s0, s1], dim=1), one)
        # (the resident and host-driven single-device solvers agree to the tolerances of
        # test_gpu_dopri5.py::test_dopri5_resident_matches_host_driven, not bitwise)
        return
    assert len(a0) == len(ref_att) and n0 == s.nfev
    assert [a[2] for a in a0] == [a[2] for a in ref_att]
    np.testing.assert_allclose([a[0] for a in a0], [a[0] for a in ref_att], rtol=1e-5)   # dt
    np.testing.assert_allclose([a[1] for a in a0], [a[1] for a in ref_att], rtol=1e-4)   # error ratio
    sol = torch.cat([s0, s1], dim=1)
    assert ((sol - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max() < 1e-5
