"""Which dopri5 gradient is right when the taped resident sweep and host autograd disagree?
Directional derivatives of loss = sum(w * sol) along a random parameter direction v:
  resident grad . v, host (_Dopri5Grad) grad . v, central finite differences of the resident
  forward (eps in EPS), and the oracle's fp64 CPU autograd (reference modules + restated solver).
env KIND=kanfet|kan, B=1, T=0.5, NT=3, RTOL=1e-3, FS (first_step, optional)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd.dopri5 import set_resident_dopri5_training  # noqa: E402
from oracle import torch_ref as O  # noqa: E402
from conftest import golden_sd, load_golden  # noqa: E402

kind = os.environ.get("KIND", "kanfet")
B = int(os.environ.get("B", "1"))
rtol = float(os.environ.get("RTOL", "1e-3"))
fs = os.environ.get("FS")
opts = {"first_step": float(fs)} if fs else None
dev = torch.device("cuda:0")
g = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
sd = golden_sd(g)
t = torch.tensor(np.linspace(0, float(os.environ.get("T", "0.5")), int(os.environ.get("NT", "3"))))
y0 = torch.from_numpy(g["y0_B64"]).repeat((B + 63) // 64, 1)[:B].clone()
w = torch.randn(len(t), B, 2, generator=torch.Generator().manual_seed(0))
Cls = F.KANFET if kind == "kanfet" else F.KAN


def model(delta=None, eps=0.0):
    m = Cls([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    if delta is not None:
        with torch.no_grad():
            for n, p in m.named_parameters():
                p.add_(eps * delta[n])
    return m.to(dev)


m0 = model()
names = [n for n, _ in m0.named_parameters()]
gen = torch.Generator().manual_seed(1)
v = {n: torch.randn(p.shape, generator=gen) for n, p in m0.named_parameters()}


def grad_run(resident):
    m = model()
    prev = set_resident_dopri5_training(resident)
    try:
        sol = F.odeint(F.autonomous(m), y0.to(dev), t, rtol=rtol, atol=rtol * 0.1, options=opts)
        loss = (w.to(dev) * sol).sum()
        loss.backward()
    finally:
        set_resident_dopri5_training(prev)
    s = F.dopri5.dopri5_solve.last
    gv = sum((p.grad.cpu().double() * v[n].double()).sum().item() for n, p in m.named_parameters())
    return loss.item(), gv, s.nfev, {n: p.grad.norm().item() for n, p in m.named_parameters()}


def loss_at(eps):
    m = model(v, eps)
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m), y0.to(dev), t, rtol=rtol, atol=rtol * 0.1, options=opts)
    return (w.to(dev) * sol).sum().item(), F.dopri5.dopri5_solve.last.nfev


out = {"kind": kind, "B": B, "rtol": rtol}
out["resident"] = grad_run(True)
out["host"] = grad_run(False)
fd = {}
for eps in (1e-2, 3e-3, 1e-3, 3e-4, 1e-4):
    (lp, np_), (lm, nm) = loss_at(eps), loss_at(-eps)
    fd[eps] = ((lp - lm) / (2 * eps), np_, nm)
out["fd"] = fd
# oracle fp64 autograd (CPU)
ps = {k: v_.clone().double().requires_grad_(k in names) for k, v_ in sd.items()}
ref = (O.KANFETRef.from_state_dict(ps, 2) if kind == "kanfet"
       else O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)]))
tr = O.Dopri5Trace()
sol = O.odeint(lambda tt, yy: ref(yy), y0.double(), t, rtol=rtol, atol=rtol * 0.1, trace=tr, options=opts)
lo = (w.double() * sol).sum()
gr = torch.autograd.grad(lo, [ps[n] for n in names])
out["oracle64"] = (lo.item(), sum((a * v[n].double()).sum().item() for a, n in zip(gr, names)), tr.nfev)
print(json.dumps(out, default=str), flush=True)
