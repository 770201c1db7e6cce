"""Where does the ETT forecaster's dopri5 forward at B (env, 1024) go non-finite?  The latent z0,
one field evaluation, the solve on the host loop vs the resident solver vs odeint_rk4."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import ett  # noqa: E402
import fet_ode_amd.dopri5  # noqa: E402,F401

dev = torch.device("cuda:0")
B, P = int(os.environ.get("B", 1024)), int(os.environ.get("P", 24))
torch.manual_seed(0)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=P, latent_dim=64, solver="dopri5",
                                  rtol=1e-3, atol=1e-4).to(dev)
sd = {k: v.clone() for k, v in m.state_dict().items()}
g = torch.Generator().manual_seed(4)
series = torch.cumsum(torch.randn(B + 96 + P, 7, generator=g), 0) * 0.05
ds = ett.EnergyWindowDataset(series, series[:, -1], 96, P, device=dev)
xb, yb = ds.batch(torch.arange(B, device=dev))
t_fut = torch.linspace(0.0, float(P - 1) * 0.05, steps=P, device=dev)
with torch.no_grad():
    z0 = m.encoder(xb)
    print("z0 finite", bool(torch.isfinite(z0).all()), "max", z0.abs().max().item(), flush=True)
    f = m.dynamics(0.0, z0)
    print("f(z0) finite", bool(torch.isfinite(f).all()), "max", f.abs().max().item(), flush=True)
    m.dynamics.net.reset_state()
    for name, gap in (("host loop", (0, 1 << 30)), ("resident", (0, 0))):
        m.load_state_dict(sd)
        F.dopri5.set_wide_resident_dopri5(True, gap=gap)
        try:
            zt = F.odeint(m.dynamics, z0, t_fut, method="dopri5", rtol=1e-3, atol=1e-4)
            s = F.dopri5.dopri5_solve.last
            print(name, type(s).__name__, "finite", bool(torch.isfinite(zt).all()), "max", zt.abs().max().item(),
                  "attempts", s.n_attempts, flush=True)
        except AssertionError as e:
            s = F.dopri5.dopri5_solve.last
            print(name, "AssertionError", e, flush=True)
    F.dopri5.set_wide_resident_dopri5(True, gap=(512, 8192))
    m.load_state_dict(sd)
    zr = ett.odeint_rk4(m.dynamics, z0, t_fut, n_substeps=4)
    print("rk4 finite", bool(torch.isfinite(zr).all()), "max", zr.abs().max().item(), flush=True)
    bad = (~torch.isfinite(zr)).any(dim=0).any(dim=1).nonzero().flatten().tolist()
    print("non-finite rows (rk4):", bad[:20], len(bad))
