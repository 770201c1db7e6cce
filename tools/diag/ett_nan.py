"""Where does the ETT training-step loss go non-finite?  The latent trajectory's max |z| per output
time on the GPU, and the oracle's (fp32 CPU, two samples) for the same model and inputs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402,F401
from fet_ode_amd import ett  # noqa: E402
from oracle import ett_ref as E  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

dev = torch.device("cuda:0")
B, P, SUB = int(os.environ.get("B", 1024)), int(os.environ.get("P", 24)), int(os.environ.get("SUB", 4))
torch.manual_seed(0)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=P, latent_dim=64, solver="rk4").to(dev)
g = torch.Generator().manual_seed(4)
series = torch.cumsum(torch.randn(B + 96 + P, 7, generator=g), 0) * 0.05
ds = ett.EnergyWindowDataset(series, series[:, -1], 96, P, device=dev)
xb, yb = ds.batch(torch.arange(B, device=dev))
t_fut = torch.linspace(0.0, float(P - 1), steps=P, device=dev)
sd = {k: v.detach().cpu().clone() for k, v in m.dynamics.net.state_dict().items()}
with torch.no_grad():
    z0 = m.encoder(xb)
    zt = ett.odeint_rk4(m.dynamics, z0, t_fut, n_substeps=SUB)
print("z0 max", z0.abs().max().item())
print("gpu max|z| per t:", [f"{v:.3g}" for v in zt.abs().amax(dim=(1, 2)).tolist()])
print("gpu nonfinite rows at last t:", (~torch.isfinite(zt[-1]).all(-1)).sum().item())
ref = O.KANFETRef.from_state_dict(sd, 2)
zr = E.odeint_rk4(lambda tt, zz: ref(zz), z0[:2].cpu(), t_fut.cpu(), n_substeps=SUB)
print("oracle max|z| per t:", [f"{v:.3g}" for v in zr.abs().amax(dim=(1, 2)).tolist()])
