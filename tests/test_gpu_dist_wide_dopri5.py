"""Trajectory-sharded device-resident dopri5 of the wide KAN-FET field (fetode_wide_dopri5_xrank):
the ETT forecaster's solve, odeint(self.dynamics, z0, t_fut, method="dopri5") (train_kan_fet_ett.py:192)
with KANFET([64, 128, 64]), sharded over ranks (BASELINE configs[3] "sharded 8x", SURVEY §8e
caveat 2).  2 ranks on cuda:0: each rank's kernel owns its rows, the error norms are exchanged
between the two kernels through IPC-mapped inboxes (no host round trip per attempt).

* Equal shards of 64-row tiles (global B = 2048): the ranks exchange the norm's leaf sums and form
  the single device's xor tree, so attempts, solution and hysteresis memory are BITWISE the single
  device's resident solve of the global batch (whose norm order depends on the batch alone).
* Shards that split a row tile (global B = 2000): rank totals summed in rank order — the single
  device's attempts and step sizes, the solution to fp32 rounding.

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
        dyn, z0, t = _problem(B, sd)
        dyn = dyn.to("cuda:0")
        y0 = D.shard(z0).to("cuda:0")
        with torch.no_grad():
            sol = D.odeint_sharded(dyn, y0, t.to("cuda:0"), **KW)
        s = F.dopri5.dopri5_solve.last
        mem = [f._prev.cpu() for _, f in field_layers(dyn.net)]
        q.put((rank, sol.cpu(), [(a[0], a[1], a[2], a[3]) for a in s.attempts], s.nfev, type(s).__name__, mem))
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


@pytest.mark.parametrize("B,exact", [(2048, True), (2000, False)])
def test_sharded_wide_resident_dopri5(dev, B, exact):
    sd, sol, att, nfev, mem = _single(dev, B)
    assert len(att) >= 3
    (_, s0, a0, n0, k0, m0), (_, s1, a1, n1, k1, m1) = _ranks(B, sd)
    assert k0 == k1 == "ResidentSolve", (k0, k1)      # one launch per rank, norms exchanged in-kernel
    assert a0 == a1 and n0 == n1 == nfev                # every rank takes the same attempts
    full = torch.cat([s0, s1], dim=1)
    mems = [torch.cat([x, y]) for x, y in zip(m0, m1)]
    if exact:
        assert a0 == att
        assert torch.equal(full, sol)
        assert all(torch.equal(x, y) for x, y in zip(mems, mem))
    else:
        assert [a[3] for a in a0] == [a[3] for a in att]
        for (t0, dt, r, _), (t0r, dtr, rr, _) in zip(a0, att):
            assert abs(dt - dtr) <= 1e-6 * abs(dtr) and abs(r - rr) <= 1e-5 * max(abs(rr), 1e-30)
        # the shards' layers are input-sliced for their own batch (other fp32 sums than the single
        # device's): KAN-FET rounding differences, not an exchange error (attempts above are equal)
        scale = sol.abs().max().item()
        assert (full - sol).abs().max().item() <= 1e-4 * scale
