"""Where the reference's own ETT training iteration spends its time (bench.ett_reference_iteration_rate
shapes: B = 64, 32 -> 8, t_fut 0..7, KAN-FET latent field x0.1) at a looser rtol (fewer attempts):
forward / backward wall split, evaluations, and (under rocprofv3 --stats) the GPU kernel time."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import fet_ode_amd as F
from fet_ode_amd import ett

dev = torch.device("cuda:0")
rtol = float(os.environ.get("REF_RTOL", "1e-5"))
torch.manual_seed(0)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=32, pred_len=8, latent_dim=64, solver="dopri5",
                                  rtol=rtol, atol=rtol * 1e-2)
with torch.no_grad():
    for n, p_ in m.dynamics.net.named_parameters():
        if n.endswith(("coef", "base_weight", "spline_weight", "logistic_weight")):
            p_.mul_(0.1)
m = m.to(dev)
g = torch.Generator().manual_seed(4)
series = torch.cumsum(torch.randn(64 + 40, 7, generator=g), 0) * 0.05
ds = ett.EnergyWindowDataset(series, series[:, -1], 32, 8, device=dev)
xb, yb = ds.batch(torch.arange(64, device=dev))
t_fut = torch.linspace(0.0, 7.0, steps=8, device=dev)
for it in range(2):
    m.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = torch.nn.functional.mse_loss(m(xb, t_fut), yb)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    loss.backward()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    s = F.dopri5.dopri5_solve.last
    print(json.dumps({"rtol": rtol, "it": it, "fwd_ms": (t1 - t0) * 1e3, "bwd_ms": (t2 - t1) * 1e3,
                      "attempts": s.n_attempts, "nfev": s.nfev,
                      "fwd_us_per_eval": (t1 - t0) * 1e6 / s.nfev, "bwd_us_per_eval": (t2 - t1) * 1e6 / s.nfev}),
          flush=True)
