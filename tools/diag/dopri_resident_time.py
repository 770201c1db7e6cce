"""Per-attempt cost of the resident dopri5 (fetode_integrate_dopri5) vs batch, next to the rk4
fused kernel's per-evaluation time: separates the field cost from the grid-reduction cost."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m0 = F.KANFET([2, 10, 2], grid_size=5)
sd = {k: v.clone() for k, v in m0.state_dict().items()}
t = torch.tensor(np.linspace(0, 3.5, 35))
for rt, at in ((1e-7, 1e-9), (1e-3, 1e-4)):
    for B in (2, 64, 512, 2048, 4096):
        y0 = bench.lv_y0(B, 0).to(dev)
        m = F.KANFET([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        with torch.no_grad():
            F.odeint(F.autonomous(m), y0, t, rtol=rt, atol=at)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            F.odeint(F.autonomous(m), y0, t, rtol=rt, atol=at)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        s = F.dopri5.dopri5_solve.last
        n_att = (s.nfev - 2) / 6
        k_ms = bench.kernel_time_ms(m, y0, t, reps=5)
        print(f"rtol {rt:g} B={B}: {type(s).__name__} {el*1e3:.2f} ms nfev {s.nfev} attempts {n_att:.0f}: "
              f"{el / n_att * 1e6:.2f} us/attempt | rk4 kernel {k_ms*1e3/136:.2f} us/eval -> "
              f"barrier+control ~{el / n_att * 1e6 - 6 * k_ms * 1e3 / 136:.2f} us", flush=True)
