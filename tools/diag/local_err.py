"""Local (one-step) error of the GPU fused rk4 step vs the CPU oracle's fp32 step, both against
an fp64 step from the SAME fp32 state, along the bench workload's fp64 trajectory
(B = 4096, t = linspace(0, 3.5, 35), seed-0 weights).  Separates per-step arithmetic accuracy
from trajectory amplification."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import fet_ode_amd as F  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5)
sd = {k: v.clone() for k, v in m.state_dict().items()}
m = m.to(dev)
B = int(os.environ.get("LE_B", "4096"))
y0 = (0.5 + 2.5 * torch.rand(4096, 2, generator=torch.Generator().manual_seed(0))).to(torch.float32)[:B]
t = torch.tensor(np.linspace(0, 3.5, 35))
r64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
with torch.no_grad():
    _, recs = O.rk4_with_states(r64, y0.double(), t)


def ref_step(dtype, y, prevs, j):
    r = O.KANFETRef.from_state_dict(sd, 2).to(dtype)
    if j > 0:
        for st, p in zip(r.states, prevs):
            st.prev_x = p.to(dtype)[:, :, None, None].expand(-1, -1, st.branch_sign.shape[2], st.branch_sign.shape[3]).clone()
            st.branch_sign = torch.ones_like(st.prev_x)
    return O.odeint(lambda tt, yy: r(yy), y.to(dtype), t[j:j + 2], method="rk4")[1]


eg, eo = [], []
with torch.no_grad():
    for j, (y, prevs) in enumerate(recs):
        y32 = y.float()
        p32 = [p.float() for p in prevs]
        s64 = ref_step(torch.float64, y32.double(), [p.double() for p in p32], j)
        s32 = ref_step(torch.float32, y32, p32, j)
        mm = F.KANFET([2, 10, 2], grid_size=5)
        mm.load_state_dict(sd)
        mm = mm.to(dev)
        if j > 0:
            for layer, p in zip(mm.layers, p32):
                layer.ferro._prev = p.clone().to(dev)
        g = F.odeint(F.autonomous(mm), y32.to(dev), t[j:j + 2], method="rk4")[1].cpu()
        den = s64.norm(dim=1).clamp_min(1e-30)
        eg.append(((g.double() - s64).norm(dim=1) / den))
        eo.append(((s32.double() - s64).norm(dim=1) / den))
eg, eo = torch.stack(eg), torch.stack(eo)
q = [0.5, 0.9, 0.99, 0.999, 1.0]
res = {"gpu_local_err_quantiles": np.quantile(eg.numpy(), q).tolist(),
       "oracle_local_err_quantiles": np.quantile(eo.numpy(), q).tolist(),
       "gpu_mean": eg.mean().item(), "oracle_mean": eo.mean().item(),
       "ratio_mean": (eg.mean() / eo.mean()).item(), "quantiles": q, "B": B}
print(res)
torch.save({"eg": eg, "eo": eo}, os.path.join(REPO, "gpurun_out", "local_err.pt"))
