"""The ETT forecaster's latent dopri5 solve (KANFET([64, 128, 64]) K = 10, t_fut = 0..P-1) resident
(fetode_wide_dopri5, one launch) vs the host-driven loop, wall time per solve, attempts, nfev."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import dopri5, ett  # noqa: E402,F401

dev = torch.device("cuda:0")
P = int(os.environ.get("P", 96))
RTOL, ATOL = float(os.environ.get("RTOL", 1e-3)), float(os.environ.get("ATOL", 1e-4))
for B in [int(b) for b in os.environ.get("BS", "256,8192").split(",")]:
    torch.manual_seed(0)
    dyn = ett.KANFETDynamics(64, hidden=128).to(dev)
    sd = {k: v.clone() for k, v in dyn.state_dict().items()}
    g = torch.Generator().manual_seed(3)
    z0 = (torch.randn(B, 64, generator=g) * 0.6).to(dev)
    t = torch.linspace(0.0, float(P - 1), steps=P, device=dev)
    res = {}
    for resident in (True, False):
        F.dopri5.set_wide_resident_dopri5(resident, gap=(0, 0))
        times = []
        for rep in range(2):
            dyn.load_state_dict(sd)
            dyn.net.reset_state()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.no_grad():
                sol = F.odeint(dyn, z0, t, method="dopri5", rtol=RTOL, atol=ATOL)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        s = F.dopri5.dopri5_solve.last
        res[resident] = sol
        print(f"B={B} {'resident' if resident else 'host loop'}: {min(times) * 1e3:.1f} ms per solve "
              f"(runs {[round(x * 1e3, 1) for x in times]}), attempts {s.n_attempts}, nfev {s.nfev}, "
              f"{s.nfev / min(times):.0f} evals/s", flush=True)
    d = (res[True] - res[False]).abs().max().item() / (res[False].abs().max().item() + 1e-30)
    print(f"B={B} max |resident - host| / scale = {d:.3e}", flush=True)
    F.dopri5.set_wide_resident_dopri5(True)
