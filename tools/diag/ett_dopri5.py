"""The reference's ETT forecaster call with the KAN-FET latent field: odeint(dynamics, z0, t_fut,
method="dopri5") (train_kan_fet_ett.py:192) at torchdiffeq's defaults (rtol 1e-7, atol 1e-9) or
given tolerances, on B windows; reports attempts, nfev, wall time and the host share (wall minus
nfev x the field evaluation's own time, measured in a tight loop)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import ett  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 256))
rtol, atol = float(os.environ.get("RTOL", 1e-7)), float(os.environ.get("ATOL", 1e-9))
P = int(os.environ.get("P", 96))
torch.manual_seed(0)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=P, latent_dim=64, solver="dopri5",
                                  rtol=rtol, atol=atol).to(dev)
g = torch.Generator().manual_seed(4)
series = torch.cumsum(torch.randn(B + 96 + P, 7, generator=g), 0) * 0.05
ds = ett.EnergyWindowDataset(series, series[:, -1], 96, P, device=dev)
xb, _ = ds.batch(torch.arange(B, device=dev))
t_fut = torch.linspace(0.0, float(P - 1), steps=P, device=dev)
with torch.no_grad():
    z0 = m.encoder(xb)
    for _ in range(3):
        m.dynamics(0.0, z0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        m.dynamics(0.0, z0)
    torch.cuda.synchronize()
    ev = (time.perf_counter() - t0) / 20
    m.dynamics.net.reset_state() if hasattr(m.dynamics.net, "reset_state") else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    try:
        y = m(xb, t_fut)
        torch.cuda.synchronize()
        ok = bool(torch.isfinite(y).all())
        err = ""
    except AssertionError as e:
        ok, err = False, str(e)
    wall = time.perf_counter() - t0
s = F.dopri5.dopri5_solve.last
n_att = len(s.attempts)
print(f"B={B} P={P} rtol={rtol:g} atol={atol:g}: attempts {n_att} accepted {sum(1 for a in s.attempts if a[3])} "
      f"nfev {s.nfev}, wall {wall:.3f} s, field eval {ev * 1e3:.3f} ms -> evals {s.nfev * ev:.3f} s, "
      f"host/control share {(wall - s.nfev * ev) / wall:.3f}, finite {ok} {err}")
