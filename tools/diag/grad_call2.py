"""Diagnose the second-solve gradient: fused vs per-stage GPU vs oracle fp64, per trajectory."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch
import fet_ode_amd as F
from conftest import golden_sd, load_golden
from oracle import torch_ref as O
dev = torch.device("cuda:0")
g = load_golden("traj_kanfet"); sd = golden_sd(g)
t = torch.from_numpy(g["t35"])[:4]
B = int(os.environ.get("B", "5"))
y0 = O.lv_y0(B, seed=11)
res = {}
for mode in ("fused", "stage"):
    F.set_fused_training(mode == "fused")
    m = F.KANFET([2, 10, 2], grid_size=5); m.load_state_dict(sd); m = m.to(dev)
    out = []
    for call in range(2):
        m.zero_grad()
        yg = y0.clone().to(dev).requires_grad_(True)
        sol = F.odeint(F.autonomous(m), yg, t, method="rk4")
        sol.square().sum().backward()
        out.append((sol.detach().cpu(), yg.grad.cpu(), [p.prev_x.detach().cpu().clone() if False else None for p in []]))
    res[mode] = out
skip = ("grid", "prev_x", "branch_sign")
ps = {k: v.clone().double().requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
ref = O.KANFETRef.from_state_dict(ps, 2)
ro = []
for call in range(2):
    yc = y0.clone().double().requires_grad_(True)
    s = O.odeint(lambda tt, yy: ref(yy), yc, t, method="rk4"); s.square().sum().backward()
    ro.append((s.detach(), yc.grad.clone()))
for call in range(2):
    for mode in ("fused", "stage"):
        sol, gy, _ = res[mode][call]
        es = ((sol.double() - ro[call][0]).abs().max().item())
        eg = (gy.double() - ro[call][1]).abs().amax(dim=1)
        print(f"call {call} {mode}: sol maxabs {es:.3e}  y0grad per-traj maxabs {eg.tolist()}  scale {ro[call][1].abs().amax(dim=1).tolist()}")
