"""ETT forecaster training step (KAN-FET latent field [64, 128, 64], rk4 x SUB substeps over P
outputs): forward with autograd + MSE + backward, at batch B; wall time per step."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402,F401
from fet_ode_amd import ett  # noqa: E402

dev = torch.device("cuda:0")
B, P, SUB = int(os.environ.get("B", 1024)), int(os.environ.get("P", 24)), int(os.environ.get("SUB", 4))
torch.manual_seed(0)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=P, latent_dim=64, solver="rk4").to(dev)
g = torch.Generator().manual_seed(4)
series = torch.cumsum(torch.randn(B + 96 + P, 7, generator=g), 0) * 0.05
ds = ett.EnergyWindowDataset(series, series[:, -1], 96, P, device=dev)
xb, yb = ds.batch(torch.arange(B, device=dev))
t_fut = torch.linspace(0.0, float(P - 1), steps=P, device=dev)
opt = torch.optim.Adam(m.parameters(), lr=1e-3)


def step():
    opt.zero_grad(set_to_none=True)
    loss = torch.nn.functional.mse_loss(m(xb, t_fut, rk4_substeps=SUB), yb)
    loss.backward()
    opt.step()
    return loss


step()
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.no_grad():
    m(xb, t_fut, rk4_substeps=SUB)
torch.cuda.synchronize()
fwd = time.perf_counter() - t0
t0 = time.perf_counter()
loss = step()
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"ETT train B={B} P={P} sub={SUB} ({(P - 1) * SUB * 4} evals): fwd(no_grad) {fwd * 1e3:.1f} ms, "
      f"train step {el * 1e3:.1f} ms, loss {loss.item():.4f}", flush=True)
