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
from fet_ode_amd import dopri5, ett  # noqa: E402,F401

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
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    modes = [int(v) for v in os.environ.get("MODES", "1,0").split(",")]   # 1: resident (fetode_wide_dopri5), 0: host loop
    ys = {}
    for resident in modes:
        F.dopri5.set_wide_resident_dopri5(bool(resident), gap=(0, 0))
        m.load_state_dict(sd)
        m.dynamics.net.reset_state()
        torch.cuda.synchronize()
        print(f"solving ({'resident' if resident else 'host loop'}) ...", flush=True)
        t0 = time.perf_counter()
        try:
            y = m(xb, t_fut)
            torch.cuda.synchronize()
            ok = bool(torch.isfinite(y).all())
            err = ""
            ys[resident] = y
        except AssertionError as e:
            ok, err = False, str(e)
        wall = time.perf_counter() - t0
        s = F.dopri5.dopri5_solve.last
        n_att = s.n_attempts
        print(f"B={B} P={P} rtol={rtol:g} atol={atol:g} {'resident' if resident else 'host loop'}: attempts {n_att} "
              f"nfev {s.nfev}, wall {wall:.3f} s, field eval {ev * 1e3:.3f} ms -> evals {s.nfev * ev:.3f} s, "
              f"{s.nfev / wall:.0f} evals/s, finite {ok} {err}", flush=True)
    if len(ys) == 2:
        print("same prediction:", bool(torch.equal(ys[0], ys[1])), flush=True)
