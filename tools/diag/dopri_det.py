"""Run-to-run / process-to-process determinism of the single-device resident dopri5: prints the
first attempts and a checksum of the solution for B in (2048, 4096)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

for B in (2048, 4096):
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to("cuda:0")
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(0)
    y0 = (0.5 + 2.5 * torch.rand(B, 2, generator=g)).to(torch.float32).to("cuda:0")
    t = torch.tensor(np.linspace(0, 3.5, 35))
    for rep in range(2):
        m.load_state_dict(sd)
        with torch.no_grad():
            sol = F.odeint(F.autonomous(m), y0, t, rtol=1e-7, atol=1e-9)
        s = F.dopri5.dopri5_solve.last
        a = s.attempts
        print(f"pid {os.getpid()} B={B} rep {rep}: attempts {s.n_attempts} nfev {s.nfev} first {a[0][1]!r} {a[0][2]!r} "
              f"second {a[1][1]!r} sum {float(sol.double().sum())!r}", flush=True)
