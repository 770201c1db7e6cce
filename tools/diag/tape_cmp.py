"""The fixed-grid training path (taped rk4 forward + reverse sweep) with the forward on the
one-trajectory-per-wave kernel and on the two-per-wave kernel (fetode_fused_set_tpw1_range), each
from a fresh module: solutions and gradients against each other and against the fp64 oracle."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from oracle import torch_ref as O  # noqa: E402
from conftest import golden_sd, load_golden  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
B = int(os.environ.get("B", "777"))
g = load_golden("traj_kanfet")
sd = golden_sd(g)
t = torch.from_numpy(g["t35"])[:6]
y0 = O.lv_y0(B, seed=4)
res = {}
for name, hi, grad in (("one", 1 << 40, True), ("two", 0, True), ("one_nograd", 1 << 40, False), ("two_nograd", 0, False)):
    lib.fetode_fused_set_tpw1_range(0, hi)
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    yg = y0.clone().to(dev).requires_grad_(grad)
    with torch.set_grad_enabled(grad):
        sol = F.odeint(F.autonomous(m), yg, t, method="rk4")
        if grad:
            sol.square().mean().backward()
    res[name] = (sol.detach().cpu().double(), yg.grad.cpu().double() if grad else None)
lib.fetode_fused_set_tpw1_range(320, 1024)
skip = ("grid", "prev_x", "branch_sign")
ps = {k: v.clone().double().requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
ref = O.KANFETRef.from_state_dict(ps, 2)
yc = y0.clone().double().requires_grad_(True)
e = O.odeint(lambda tt, yy: ref(yy), yc, t, method="rk4")
e.square().mean().backward()
mx = lambda a, b: (a - b).abs().max().item()
out = {k: {"sol_vs_fp64": mx(v[0], e.detach()), "gy0_vs_fp64": None if v[1] is None else mx(v[1], yc.grad) / yc.grad.abs().max().item()}
       for k, v in res.items()}
print(json.dumps(out), flush=True)
