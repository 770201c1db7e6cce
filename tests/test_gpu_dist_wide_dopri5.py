"""Trajectory-sharded device-resident dopri5 of the wide KAN-FET field (fetode_wide_dopri5_xrank):
the ETT forecaster's solve, odeint(self.dynamics, z0, t_fut, method="dopri5") (train_kan_fet_ett.py:192)
with KANFET([64, 128, 64]), sharded over ranks (BASELINE configs[3] "sharded 8x", SURVEY §8e
caveat 2).  2 ranks on cuda:0: each rank's kernel owns its rows, the error norms are exchanged
between the two kernels through IPC-mapped inboxes (no host round trip per attempt).

* Equal shards of 64-row tiles (global B = 2048): the ranks exchange the norm's leaf sums and form
  the single device's xor tree, so attempts, solution and hysteresis memory are BITWISE the single
  device's resident solve of the global batch (whose norm order depends on the batch alone).
* Shards that split a row tile (global B = 2000): the shards' layers are input-sliced for their own
  batch (other fp32 sums than the single device's, which in an ill-conditioned KAN-FET field can
  flip an accept decision), and the ranks exchange their totals in rank order — checked against
  the host-driven sharded loop on the same shards (dist.odeint_sharded with the resident path off:
  per-layer launches, one norm all-reduce per attempt), whose per-row arithmetic is the same: the
  same attempts, step sizes to fp64 rounding, the solution and memory to 1e-6.

The persistent grids are capped (FETODE_WIDE_DOPRI_GRID) so that both ranks' grids are co-resident
on the one GPU; the result does not depend on the grid (tests/test_gpu_wide_dopri5.py)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO

pytestmark = pytest.mark.gpu

GRID_CAP = "96"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(B, sd=None):
    from fet_ode_amd import ett
    torch.manual_seed(0)
    dyn = ett.KANFETDynamics(64, hidden=128, num_fet_basis=10)
    if sd is not None:
        dyn.load_state_dict(sd)
    g = torch.Generator().manual_seed(3)
    z0 = torch.randn(B, 64, generator=g) * 0.6
    t = torch.linspace(0.0, 0.5, steps=4)
    return dyn, z0, t


KW = dict(method="dopri5", rtol=1e-3, atol=1e-4)


def _worker(rank, world, port, q, B, sd):
    import sys
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["FETODE_WIDE_DOPRI_GRID"] = GRID_CAP
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import fet_ode_amd as F
        import fet_ode_amd.dist as D
        from fet_ode_amd.autograd_ops import field_layers
        out = []
        for resident in (True, False):
            dyn, z0, t = _problem(B, sd)
            dyn = dyn.to("cuda:0")
            y0 = D.shard(z0).to("cuda:0")
            D.set_resident_sharded(resident)
            with torch.no_grad():
                sol = D.odeint_sharded(dyn, y0, t.to("cuda:0"), **KW)
            s = F.dopri5.dopri5_solve.last
            mem = [f._prev.cpu() for _, f in field_layers(dyn.net)]
            # numpy, not tensors: a tensor in the queue is a shared-memory handle the parent fetches
            # from this process, which may have exited by then
            out.append((sol.cpu().numpy(), [(a[0], a[1], a[2], a[3]) for a in s.attempts], s.nfev,
                        type(s).__name__, [x.numpy() for x in mem]))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _single(dev, B):
    import fet_ode_amd as F
    from fet_ode_amd.autograd_ops import field_layers
    from fet_ode_amd.dopri5 import ResidentSolve
    dyn, z0, t = _problem(B)
    sd = {k: v.clone() for k, v in dyn.state_dict().items()}
    dyn = dyn.to(dev)
    prev = F.dopri5.set_wide_resident_dopri5(True, gap=(0, 0))
    try:
        with torch.no_grad():
            sol = F.odeint(dyn, z0.to(dev), t.to(dev), **KW)
    finally:
        F.dopri5.set_wide_resident_dopri5(prev, gap=(512, 8192))
    s = F.dopri5.dopri5_solve.last
    assert isinstance(s, ResidentSolve)
    mem = [f._prev.cpu() for _, f in field_layers(dyn.net)]
    return sd, sol.cpu(), [(a[0], a[1], a[2], a[3]) for a in s.attempts], s.nfev, mem


def _ranks(B, sd):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, B, sd)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _unpack(res):
    """per rank: [(solution, attempts, nfev, solver, memory)] for resident = True, False"""
    return [[(torch.from_numpy(o[0]), o[1], o[2], o[3], [torch.from_numpy(x) for x in o[4]]) for o in r[1]]
            for r in res]


@pytest.mark.parametrize("B,exact", [(2048, True), (2000, False)])
def test_sharded_wide_resident_dopri5(dev, B, exact):
    sd, sol, att, nfev, mem = _single(dev, B)
    assert len(att) >= 3
    (r0, h0), (r1, h1) = _unpack(_ranks(B, sd))
    (s0, a0, n0, k0, m0), (s1, a1, n1, k1, m1) = r0, r1
    assert k0 == k1 == "ResidentSolve", (k0, k1)      # one launch per rank, norms exchanged in-kernel
    assert h0[3] == h1[3] == "_Dopri5"                  # the host-driven sharded loop
    assert a0 == a1 and n0 == n1                        # every rank takes the same attempts
    full = torch.cat([s0, s1], dim=1)
    mems = [torch.cat([x, y]) for x, y in zip(m0, m1)]
    if exact:
        assert a0 == att and n0 == nfev
        assert torch.equal(full, sol)
        assert all(torch.equal(x, y) for x, y in zip(mems, mem))
    else:
        hs, ha, hn = torch.cat([h0[0], h1[0]], dim=1), h0[1], h0[2]
        assert n0 == hn and [a[3] for a in a0] == [a[3] for a in ha]
        for (t0, dt, r, _), (t0h, dth, rh, _) in zip(a0, ha):
            assert abs(dt - dth) <= 1e-12 * abs(dth) and abs(r - rh) <= 1e-6 * max(abs(rh), 1e-30)
        scale = hs.abs().max().item()
        assert (full - hs).abs().max().item() <= 1e-6 * scale
        hm = [torch.cat([x, y]) for x, y in zip(h0[4], h1[4])]
        for x, y in zip(mems, hm):
            assert (x - y).abs().max().item() <= 1e-6 * (y.abs().max().item() + 1e-30)
