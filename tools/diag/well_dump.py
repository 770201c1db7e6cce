"""Dump GPU KAN-FET trajectories (bench config B=4096 t35; golden B=64 t35/t140) for offline
well-conditioned-subset analysis against the oracle (tools/diag/well_analyse.py)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import fet_ode_amd as F  # noqa: E402
from conftest import golden_sd, load_golden  # noqa: E402

dev = torch.device("cuda:0")
out = {}
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5)
sd = {k: v.clone() for k, v in m.state_dict().items()}
y0 = (0.5 + 2.5 * torch.rand(4096, 2, generator=torch.Generator().manual_seed(0))).to(torch.float32)
t = torch.tensor(np.linspace(0, 3.5, 35))
tag = os.environ.get("FETODE_FACTOR_LIMIT", "default")
with torch.no_grad():
    mm = F.KANFET([2, 10, 2], grid_size=5)
    mm.load_state_dict(sd)
    out["bench"] = F.odeint(F.autonomous(mm.to(dev)), y0.to(dev), t, method="rk4").cpu()
    g = load_golden("traj_kanfet")
    for tt in ("t35", "t140"):
        mm = F.KANFET([2, 10, 2], grid_size=5)
        mm.load_state_dict(golden_sd(g))
        out[tt] = F.odeint(F.autonomous(mm.to(dev)), torch.from_numpy(g["y0_B64"]).to(dev),
                           torch.from_numpy(g[tt]), method="rk4").cpu()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
torch.save(out, os.path.join(REPO, "gpurun_out", f"well_dump_{tag}.pt"))
print("saved", tag)
