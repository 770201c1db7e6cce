"""ETT forecaster training through its own dopri5 call (train_kan_fet_ett.py:192, 320-335): forward
with autograd + MSE + backward + Adam at batch B, P outputs, rtol RTOL; the time split into the
taped forward and the backward, plus the no-grad forward for scale.  env B, P, RTOL, ITERS."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import ett  # noqa: E402

dev = torch.device("cuda:0")
B, P = int(os.environ.get("B", 1024)), int(os.environ.get("P", 24))
rtol = float(os.environ.get("RTOL", "1e-3"))
iters = int(os.environ.get("ITERS", "2"))
torch.manual_seed(0)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=P, latent_dim=64, solver="dopri5",
                                  rtol=rtol, atol=rtol * 0.1).to(dev)
g = torch.Generator().manual_seed(4)
series = torch.cumsum(torch.randn(B + 96 + P, 7, generator=g), 0) * 0.05
ds = ett.EnergyWindowDataset(series, series[:, -1], 96, P, device=dev)
xb, yb = ds.batch(torch.arange(B, device=dev))
t_fut = torch.linspace(0.0, float(P - 1) * float(os.environ.get("TSCALE", "1")), steps=P, device=dev)
opt = torch.optim.Adam(m.parameters(), lr=1e-4)


def sync():
    torch.cuda.synchronize(dev)
    return time.perf_counter()


for it in range(iters):
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    t0 = sync()
    with torch.no_grad():
        m(xb, t_fut)
    t1 = sync()
    m.load_state_dict(sd)
    opt.zero_grad(set_to_none=True)
    t2 = sync()
    pred = m(xb, t_fut)
    loss = torch.nn.functional.mse_loss(pred, yb)
    t3 = sync()
    loss.backward()
    t4 = sync()
    opt.step()
    t5 = sync()
    s = F.dopri5.dopri5_solve.last
    gn = sum(p.grad.norm().item() ** 2 for p in m.parameters() if p.grad is not None) ** 0.5
    print(f"ETT dopri5 train B={B} P={P} rtol={rtol:g}: attempts {s.n_attempts} nfev {s.nfev} | fwd(no_grad) "
          f"{(t1 - t0) * 1e3:.1f} ms | taped fwd {(t3 - t2) * 1e3:.1f} ms, bwd {(t4 - t3) * 1e3:.1f} ms, "
          f"Adam {(t5 - t4) * 1e3:.1f} ms | loss {loss.item():.4f} |grad| {gn:.3e} path {type(s).__name__}",
          flush=True)
