"""Training iterations through dopri5 (fwd + bwd): the taped resident path vs host autograd
(_Dopri5Grad).  Cases: the reference's own iteration (X0 (1, 2), 35 points, rtol 1e-7 / atol
1e-9), and the bench batch B = 4096 at rtol 1e-3 and at the default tolerances.
env CASES=ref,b4096,b4096d (default all), HOST=0 skips the host path."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd.dopri5 import set_resident_dopri5_training  # noqa: E402
from oracle import torch_ref as O  # noqa: E402


def run(B, rtol, atol, resident, iters):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    y0 = torch.tensor([[1.0, 1.0]], device=dev) if B == 1 else O.lv_y0(B, 0).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    _, soln = O.lotka_volterra_truth()
    target = torch.tensor(soln, dtype=torch.float32)[:35].to(dev)
    prev = set_resident_dopri5_training(resident)
    ts, fw = [], []
    try:
        for _ in range(iters):
            m.zero_grad(set_to_none=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pred = F.odeint(F.autonomous(m), y0, t, rtol=rtol, atol=atol)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            loss = torch.mean((pred[:, 0, :] - target[:, None, :]) ** 2) if B > 1 else \
                torch.mean((pred[:, 0, :] - target) ** 2)
            loss.backward()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            ts.append(t2 - t0)
            fw.append(t1 - t0)
    finally:
        set_resident_dopri5_training(prev)
    s = F.dopri5.dopri5_solve.last
    g = torch.cat([p.grad.flatten() for p in m.parameters()])
    return {"B": B, "rtol": rtol, "resident": resident, "iter_ms": 1e3 * float(np.median(ts)),
            "fwd_ms": 1e3 * float(np.median(fw)), "all_ms": [round(1e3 * x, 2) for x in ts],
            "nfev": s.nfev, "attempts": len(s.attempts), "loss": loss.item(), "gnorm": g.norm().item(),
            "finite": bool(torch.isfinite(g).all())}


cases = os.environ.get("CASES", "ref,b4096,b4096d").split(",")
host = os.environ.get("HOST", "1") != "0"
if "ref" in cases:
    print(json.dumps(run(1, 1e-7, 1e-9, True, 6)), flush=True)
    if host:
        print(json.dumps(run(1, 1e-7, 1e-9, False, 2)), flush=True)
if "b4096" in cases:
    print(json.dumps(run(4096, 1e-3, 1e-4, True, 6)), flush=True)
    if host:
        print(json.dumps(run(4096, 1e-3, 1e-4, False, 2)), flush=True)
if "b4096d" in cases:
    print(json.dumps(run(4096, 1e-7, 1e-9, True, 3)), flush=True)
