"""Training iteration (odeint forward + loss.backward()) of a depth-2 field of another width —
KANFET([2, 16, 2], K = 12) and KAN([4, 32, 4]) — at B = 4096 over the bench horizon (34 rk4 steps):
the fused pair (fieldn forward with tape + fieldn_adj_kernel + per-module parameter VJPs) vs the
per-stage path (F.set_fused_training(False)); HIP events, env B, N.  SECT=1|2|3 runs one section;
FUSED_ONLY=1 skips the per-stage / host-loop legs (for a rocprof kernel split)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
B, N = int(os.environ.get("B", "4096")), int(os.environ.get("N", "5"))
t = torch.tensor(np.linspace(0, 3.5, 35))
SECT = os.environ.get("SECT", "123")
FUSED_ONLY = os.environ.get("FUSED_ONLY", "0") == "1"


def ev_ms(fn, n):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for name, mk in (("KANFET[2,16,2] K=12", lambda: F.KANFET([2, 16, 2], grid_size=5, num_fet_basis=12)),
                 ("KAN[4,32,4]", lambda: F.KAN([4, 32, 4], grid_size=5))):
    if "1" not in SECT:
        break
    torch.manual_seed(0)
    m = mk().to(dev)
    D = m.layers[0].kan.in_features if hasattr(m.layers[0], "kan") else m.layers[0].in_features
    y0 = (0.5 + 2.0 * torch.rand(B, D, device=dev))
    func = F.autonomous(m)

    def it():
        m.zero_grad(set_to_none=True)
        F.odeint(func, y0, t, method="rk4").square().mean().backward()

    out = []
    for fused in ((True,) if FUSED_ONLY else (True, False)):
        prev = F.set_fused_training(fused)
        try:
            out.append(ev_ms(it, N if fused else 1))
        finally:
            F.set_fused_training(prev)
    with torch.no_grad():
        fwd = ev_ms(lambda: F.odeint(func, y0, t, method="rk4"), N)
    if FUSED_ONLY:
        print(f"{name} B={B}: inference solve {fwd:.2f} ms | training iteration fused {out[0]:.2f} ms", flush=True)
        continue
    print(f"{name} B={B}: inference solve {fwd:.2f} ms | training iteration fused {out[0]:.2f} ms, "
          f"per-stage {out[1]:.1f} ms ({out[1] / out[0]:.1f}x)", flush=True)

# dopri5 (rtol 1e-4) inference: fieldn's resident driver vs the host loop, at a batch one grid holds
from fet_ode_amd.dopri5 import set_resident_dopri5  # noqa: E402
B2 = int(os.environ.get("B2", "2048"))
t2 = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
for name, mk in (("KANFET[2,16,2] K=12", lambda: F.KANFET([2, 16, 2], grid_size=5, num_fet_basis=12)),
                 ("KAN[4,32,4]", lambda: F.KAN([4, 32, 4], grid_size=5))):
    if "2" not in SECT:
        break
    torch.manual_seed(0)
    m = mk().to(dev)
    D = m.layers[0].kan.in_features if hasattr(m.layers[0], "kan") else m.layers[0].in_features
    y0 = (0.5 + 2.0 * torch.rand(B2, D, device=dev))
    func = F.autonomous(m)
    res = []
    for resident in (True, False):
        prev = set_resident_dopri5(resident)
        try:
            with torch.no_grad():
                res.append(ev_ms(lambda: F.odeint(func, y0, t2, rtol=1e-4, atol=1e-6), 3))
        finally:
            set_resident_dopri5(prev)
    print(f"{name} dopri5 B={B2}: resident {res[0]:.2f} ms, host loop {res[1]:.2f} ms "
          f"(nfev {F.dopri5.dopri5_solve.last.nfev})", flush=True)

# dopri5 TRAINING (rtol 1e-3): the taped resident solve + fieldn_dopri_bwd_kernel vs _Dopri5Grad
from fet_ode_amd.dopri5 import set_resident_dopri5_training  # noqa: E402
B3 = int(os.environ.get("B3", "1024"))
t3 = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
for name, mk in (("KANFET[3,8,3] K=6", lambda: F.KANFET([3, 8, 3], grid_size=5, num_fet_basis=6)),
                 ("KAN[4,32,4]", lambda: F.KAN([4, 32, 4], grid_size=5))):
    if "3" not in SECT:
        break
    torch.manual_seed(0)
    m = mk().to(dev)
    D = m.layers[0].kan.in_features if hasattr(m.layers[0], "kan") else m.layers[0].in_features
    y0 = (0.5 + 2.0 * torch.rand(B3, D, device=dev))
    func = F.autonomous(m)

    def it3():
        m.zero_grad(set_to_none=True)
        F.odeint(func, y0, t3, rtol=1e-3, atol=1e-4).square().mean().backward()

    res = []
    for resident in (True, False):
        prev = set_resident_dopri5_training(resident)
        try:
            res.append(ev_ms(it3, 3 if resident else 1))
        finally:
            set_resident_dopri5_training(prev)
    print(f"{name} dopri5 training B={B3}: resident pair {res[0]:.2f} ms, host autograd {res[1]:.1f} ms "
          f"({res[1] / res[0]:.1f}x, nfev {F.dopri5.dopri5_solve.last.nfev})", flush=True)
