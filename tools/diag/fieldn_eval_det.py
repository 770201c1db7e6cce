"""Bitwise run-to-run determinism of fieldn single evaluations and fixed-grid solves (B = 64)."""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import fet_ode_amd as F  # noqa: E402
from test_gpu_fieldn import _model, _y0  # noqa: E402

dev = torch.device("cuda:0")
for B in (1, 64, 1000):
    for kind, widths, K in (("kan", [4, 32, 4], 0), ("kanfet", [2, 16, 2], 12)):
        y0 = _y0(B, widths[0], seed=7).to(dev)
        evs, sols = [], []
        for rep in range(4):
            m = _model(kind, widths, K).to(dev)
            with torch.no_grad():
                evs.append(m(y0).cpu())
                m2 = _model(kind, widths, K).to(dev)
                sols.append(F.odeint(F.autonomous(m2), y0, torch.tensor(np.linspace(0, 0.5, 6)), method="rk4").cpu())
        e_ok = all(torch.equal(evs[0], e) for e in evs[1:])
        s_ok = all(torch.equal(sols[0], s) for s in sols[1:])
        ediff = max((evs[0] - e).abs().max().item() for e in evs[1:])
        sdiff = max((sols[0] - s).abs().max().item() for s in sols[1:])
        print(f"B={B} {kind}: eval bitwise {e_ok} (max diff {ediff:.3e}), rk4 solve bitwise {s_ok} ({sdiff:.3e})", flush=True)
