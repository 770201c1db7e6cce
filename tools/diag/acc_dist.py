"""Distribution of per-trajectory fp64 errors: GPU fused solve vs an ensemble of fp32 CPU runs
whose parameters are moved by a fraction of an ulp (equally valid fp32 roundings)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from oracle import torch_ref as O
from tests.conftest import load_golden, golden_sd

tag = os.environ.get("TAG", "t35")
g = load_golden("traj_kanfet"); sd = golden_sd(g)
y0 = torch.from_numpy(g["y0_B64"]); t = torch.from_numpy(g[tag])
ref64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
s64 = O.odeint(lambda tt, yy: ref64(yy), y0.double(), t, method="rk4")
def errs(a):
    return ((a.double() - s64).norm(dim=2) / s64.norm(dim=2).clamp_min(1e-6)).max(0).values.numpy()
def summ(name, e):
    e = np.sort(e)[::-1]
    print(f"{name:10s} n>1e-3={int((e > 1e-3).sum()):2d} n>3e-3={int((e > 3e-3).sum()):2d} n>1e-2={int((e > 1e-2).sum()):2d} "
          f"top8={' '.join('%.1e' % v for v in e[:8])}")
if torch.cuda.is_available():
    import fet_ode_amd as F
    m = F.KANFET([2, 10, 2], grid_size=5); m.load_state_dict(sd); m = m.to("cuda")
    with torch.no_grad():
        summ("gpu", errs(F.odeint(F.autonomous(m), y0.cuda(), t, method="rk4").cpu()))
summ("cpu-fix", errs(torch.from_numpy(g[f"sol_B64_{tag}"])))
gen = torch.Generator().manual_seed(0)
for trial in range(int(os.environ.get("TRIALS", "12"))):
    sdp = {k: (v * (1 + 6e-8 * torch.randn(v.shape, generator=gen)) if v.dtype == torch.float32 and "grid" not in k else v)
           for k, v in sd.items()}
    r = O.KANFETRef.from_state_dict(sdp, 2)
    with torch.no_grad():
        summ(f"cpu-p{trial}", errs(O.odeint(lambda tt, yy: r(yy), y0, t, method="rk4")))
