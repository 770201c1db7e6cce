"""v6 (small6_kernel<..., TAPE>) vs v4 (fused4_kernel taping) fixed-grid training tapes on the same
solve: which evaluations / trajectories / tape columns differ, and by how much.  env KIND=kan|kanfet,
B=64, NPTS=35, METHOD=rk4."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from fet_ode_amd.autograd_ops import build_plan, make_handle, pack_state  # noqa: E402
from fet_ode_amd.odeint import get_schedule  # noqa: E402
from oracle import torch_ref as O  # noqa: E402
from conftest import golden_sd, load_golden  # noqa: E402

kind = os.environ.get("KIND", "kan")
B = int(os.environ.get("B", "64"))
npts = int(os.environ.get("NPTS", "35"))
method = {"rk4": _lib.RK4, "rk4_classic": _lib.RK4_CLASSIC, "euler": _lib.EULER,
          "midpoint": _lib.MIDPOINT}[os.environ.get("METHOD", "rk4")]
nst = {_lib.RK4: 4, _lib.RK4_CLASSIC: 4, _lib.EULER: 1, _lib.MIDPOINT: 2}[method]
dev = torch.device("cuda:0")
lib = _lib.load()
g = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
sd = golden_sd(g)
t = torch.from_numpy(g["t35"])[:npts]
y0 = O.lv_y0(B, seed=9).to(dev)


def run(small):
    prev = lib.fetode_fused_set_small_batch_max(1 << 40 if small else 0)
    try:
        m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        sched = get_schedule(t, None, False)
        handle = make_handle(m, B, dev)
        plan = build_plan(m, handle, dev)
        state, mask = pack_state(m, B, dev)
        _, coef, ostep, omode, oslope = sched.device_arrays(dev)
        sol = torch.empty(sched.T, B, 2, device=dev)
        tape = torch.full((sched.n_steps * nst, B, 12), float("nan"), device=dev)
        _lib.check(lib.fetode_integrate_fixed(handle.ref, plan.data_ptr(), method, y0.data_ptr(), B, coef.data_ptr(),
                                              sched.n_steps, ostep.data_ptr(), omode.data_ptr(), oslope.data_ptr(),
                                              sched.T, sol.data_ptr(), _lib.ptr(state), mask, tape.data_ptr(),
                                              _lib.stream_handle(dev)), "integrate")
        torch.cuda.synchronize()
        return sol.cpu().double(), tape.cpu().double()
    finally:
        lib.fetode_fused_set_small_batch_max(prev)


s6, t6 = run(True)
s4, t4 = run(False)
print("solution max rel diff", ((s6 - s4).abs().max() / s4.abs().max()).item())
print("tape NaN (unwritten) v6:", int(torch.isnan(t6).sum()), " v4:", int(torch.isnan(t4).sum()))
d = (t6 - t4).abs()
rel = d / t4.abs().clamp_min(1e-6)
print("tape max abs diff", np.nanmax(d.numpy()), "max rel", np.nanmax(rel.numpy()))
ev_bad = torch.nonzero(torch.nan_to_num(rel, nan=1.0).amax(dim=(1, 2)) > 1e-4).flatten().tolist()
print("evaluations with rel diff > 1e-4:", ev_bad[:40], "of", t4.shape[0])
col = torch.nan_to_num(rel, nan=1.0).amax(dim=(0, 1))
print("per column max rel:", [float("%.2e" % v) for v in col.tolist()])
bb = torch.nan_to_num(rel, nan=1.0).amax(dim=(0, 2))
print("trajectories with rel diff > 1e-4:", torch.nonzero(bb > 1e-4).flatten().tolist()[:40])
if ev_bad:
    e = ev_bad[0]
    j = int(torch.nan_to_num(rel[e], nan=1.0).amax(dim=1).argmax())
    print("first bad ev", e, "traj", j, "v6", t6[e, j].tolist(), "\nv4", t4[e, j].tolist())
