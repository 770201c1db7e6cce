"""Trajectory-sharded TRAINING on the real model (train_kanfet_node_predprey.py:254-257):
2 ranks on cuda:0 (gloo carries the collectives).  Each rank solves its shard of y0_B64, runs the
backward and all-reduces the gradients; the result must equal the single-device gradient of the
global batch.

  * fused rk4: one forward launch with tape + one reverse-sweep launch per rank, then
    allreduce_gradients(weights=B_local/B) — the fixed-grid path needs no other collective;
  * dopri5 with autograd (the reference's default method): every error norm is the global RMS
    (odeint_sharded), and its gradient is all-reduced in the backward (dopri5._NormAllReduce), so
    d loss / d theta through the adaptive step sizes is the single-device one too.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, golden_sd, load_golden

pytestmark = pytest.mark.gpu

T_RK4 = 12          # points of t35 used by the fused rk4 case
T_DOPRI = [0.0, 0.25, 0.5]


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


def _grads(m):
    return torch.cat([p.grad.detach().double().cpu().reshape(-1) for p in m.parameters()])


def _worker(rank, world, port, q, case):
    import sys
    sys.path.insert(0, REPO)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import fet_ode_amd as F
        import fet_ode_amd.dist as D
        g = load_golden("traj_kanfet")
        m = _model(F, golden_sd(g))
        y0g = torch.from_numpy(g["y0_B64"])
        y0 = D.shard(y0g).to("cuda:0")
        if case == "rk4":
            t = torch.from_numpy(g["t35"])[:T_RK4]
            sol = F.odeint(F.autonomous(m), y0, t, method="rk4")
            # per-rank mean loss, all-reduced with this shard's share: the global-mean gradient
            loss = sol.square().mean()
            loss.backward()
            D.allreduce_gradients(list(m.parameters()), weights=y0.shape[0] / y0g.shape[0])
            extra = None
        else:
            t = torch.tensor(T_DOPRI, dtype=torch.float64)
            sol = D.odeint_sharded(lambda tt, yy: m(yy), y0, t, rtol=1e-3, atol=1e-4)
            loss = sol.square().sum() / (sol.shape[0] * y0g.shape[0] * sol.shape[2])
            loss.backward()
            D.allreduce_gradients(list(m.parameters()), average=False)
            s = F.dopri5.dopri5_solve.last
            extra = [(a[1], a[3]) for a in s.attempts]
        # numpy: a tensor in the queue is a shared-memory handle served by this process, which may
        # have exited when the parent unpickles it (ConnectionRefusedError)
        q.put((rank, sol.detach().cpu().numpy(), _grads(m).numpy(), extra))
    finally:
        dist.destroy_process_group()


def _run(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [(r, torch.from_numpy(s), torch.from_numpy(g), extra) for r, s, g, extra in res]


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_sharded_fused_rk4_training_gradients(dev):
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    m = _model(F, golden_sd(g))
    t = torch.from_numpy(g["t35"])[:T_RK4]
    sol = F.odeint(F.autonomous(m), torch.from_numpy(g["y0_B64"]).to(dev), t, method="rk4")
    sol.square().mean().backward()
    ref = _grads(m)
    (_, s0, g0, _), (_, s1, g1, _) = _run("rk4")
    assert torch.equal(g0, g1)                       # every rank holds the same all-reduced gradient
    assert torch.equal(torch.cat([s0, s1], dim=1), sol.detach().cpu())   # shards: bitwise the same solve
    assert _rel(g0, ref) <= 1e-5, _rel(g0, ref)


def _dopri5_grads(F, g, dev, flip=False, roll=0):
    m = _model(F, golden_sd(g))
    y0 = torch.from_numpy(g["y0_B64"]).to(dev)
    if flip:      # the same global loss with the batch in reverse order: only fp32 sums reorder
        y0 = y0.flip(0)
    if roll:      # ... or rotated
        y0 = y0.roll(roll, 0)
    # the host-driven autograd path, as the sharded solve takes (the single-device resident
    # training path evaluates the field with another kernel: other fp32 roundings)
    from fet_ode_amd.dopri5 import set_resident_dopri5_training
    prev = set_resident_dopri5_training(False)
    try:
        sol = F.odeint(lambda tt, yy: m(yy), y0, torch.tensor(T_DOPRI, dtype=torch.float64), rtol=1e-3, atol=1e-4)
        (sol.square().sum() / sol.numel()).backward()
    finally:
        set_resident_dopri5_training(prev)
    att = [(a[1], a[3]) for a in F.dopri5.dopri5_solve.last.attempts]
    if roll:
        sol = sol.roll(-roll, 1)
    return _grads(m), (sol.flip(1) if flip else sol).detach().cpu(), att


def test_sharded_dopri5_training_gradients(dev):
    """Same attempts and solution as one device; the gradient within the fp32 noise floor of the
    single-device gradient itself.  The gradient through dopri5's step-size control is
    ill-conditioned in fp32, so the floor is measured: the single-device gradient
    of the same loss with the batch reversed or rotated by 16 / 32 / 48 (the norms' summation order
    changes, nothing else): the largest of the four.
    The exact cross-rank algebra is pinned in fp64 by tests/test_dist_gloo.py
    (test_sharded_dopri5_gradient_through_step_control_fp64)."""
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    ref, sol, ref_att = _dopri5_grads(F, g, dev)
    ref_flip, _, _ = _dopri5_grads(F, g, dev, flip=True)
    rolls = [_dopri5_grads(F, g, dev, roll=r)[0] for r in (16, 32, 48)]
    floor = max([_rel(ref_flip, ref)] + [_rel(x, ref) for x in rolls])
    (_, s0, g0, a0), (_, s1, g1, a1) = _run("dopri5")
    assert [a[1] for a in a0] == [a[1] for a in ref_att] and a0 == a1   # same accept pattern, both ranks
    for (d0, _), (dr, _) in zip(a0, ref_att):
        assert abs(d0 - dr) <= 1e-5 * abs(dr)
    assert torch.equal(g0, g1)
    full = torch.cat([s0, s1], dim=1)
    assert ((full - sol).norm() / sol.norm()).item() <= 1e-5
    assert _rel(g0, ref) <= max(4 * floor, 1e-5), (_rel(g0, ref), floor)
