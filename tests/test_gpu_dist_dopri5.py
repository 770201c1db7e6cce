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


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import fet_ode_amd as F
    import fet_ode_amd.dist as D
    g = load_golden("traj_kanfet")
    m = _model(F, golden_sd(g))
    y0 = D.shard(torch.from_numpy(g["y0_B64"])).to("cuda:0")
    with torch.no_grad():
        sol = D.odeint_sharded(lambda tt, yy: m(yy), y0, torch.tensor(T_GRID, dtype=torch.float64),
                               rtol=1e-3, atol=1e-4)
    s = F.dopri5.dopri5_solve.last
    q.put((rank, sol.cpu(), [(a[1], a[2], a[3]) for a in s.attempts], s.nfev))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_dopri5_matches_single_device(dev):
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    m = _model(F, golden_sd(g))
    with torch.no_grad(), F.closure_fusion(False):   # the host-driven solver (its attempt record)
        ref = F.odeint(lambda tt, yy: m(yy), torch.from_numpy(g["y0_B64"]).to(dev),
                       torch.tensor(T_GRID, dtype=torch.float64), rtol=1e-3, atol=1e-4).cpu()
    s = F.dopri5.dopri5_solve.last
    ref_att = [(a[1], a[2], a[3]) for a in s.attempts]

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, s0, a0, n0), (_, s1, a1, n1) = res
    assert a0 == a1 and n0 == n1                    # both ranks took identical steps
    assert len(a0) == len(ref_att) and n0 == s.nfev
    assert [a[2] for a in a0] == [a[2] for a in ref_att]
    np.testing.assert_allclose([a[0] for a in a0], [a[0] for a in ref_att], rtol=1e-5)   # dt
    np.testing.assert_allclose([a[1] for a in a0], [a[1] for a in ref_att], rtol=1e-4)   # error ratio
    sol = torch.cat([s0, s1], dim=1)
    assert ((sol - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max() < 1e-5
