"""Does the resident dopri5 read memory it did not write?  The same solve after the caching
allocator's free blocks were filled with different garbage (0, NaN, 1e30, random)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import dopri5 as D5  # noqa: E402

B = int(os.environ.get("B", 2048))
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to("cuda:0")
sd = {k: v.clone() for k, v in m.state_dict().items()}
g = torch.Generator().manual_seed(0)
y0 = (0.5 + 2.5 * torch.rand(B, 2, generator=g)).to(torch.float32).to("cuda:0")
t = torch.tensor(np.linspace(0, 3.5, 35))
for fill in (0.0, float("nan"), 1e30, -7.0, "rand"):
    D5._T_DEV.clear()
    m._fetode_plan = None
    m._fetode_handle = None
    m.__dict__.pop("_fetode_state", None)
    torch.cuda.synchronize()
    junk = torch.empty(64 << 20, device="cuda:0")
    if fill == "rand":
        junk.uniform_(-1e3, 1e3)
    else:
        junk.fill_(fill)
    del junk
    m.load_state_dict(sd)
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m), y0, t, rtol=1e-7, atol=1e-9)
    s = F.dopri5.dopri5_solve.last
    a = s.attempts
    print(f"fill {fill}: attempts {s.n_attempts} first {a[0][1]!r} {a[0][2]!r} sum {float(sol.double().sum())!r}",
          flush=True)
