"""Run-to-run determinism of fieldn's dopri5 paths: the resident solve twice and the host loop
twice on the same inputs (KANFET [2, 16, 2], K = 12, B = 64), bitwise comparisons."""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd.dopri5 import set_resident_dopri5  # noqa: E402
from test_gpu_fieldn import _model, _y0  # noqa: E402

dev = torch.device("cuda:0")
t = torch.tensor([0.0, 0.3, 0.7], dtype=torch.float64)
for B, kind, widths, K in ((1, "kanfet", [2, 16, 2], 12), (64, "kan", [4, 32, 4], 0), (64, "kanfet", [2, 16, 2], 12),
                           (64, "kanfet", [3, 8, 3], 6)):
  print(f"== B={B} {kind} {widths}", flush=True)
  y0 = _y0(B, widths[0], seed=7)
  runs = {}
  for resident in (True, True, False, False, True):
    prev = set_resident_dopri5(resident)
    try:
        m = _model(kind, widths, K).to(dev)
        with torch.no_grad():
            sol = F.odeint(F.autonomous(m), y0.to(dev), t, rtol=1e-4, atol=1e-6).cpu()
    finally:
        set_resident_dopri5(prev)
    s = F.dopri5.dopri5_solve.last
    att = [(float(a[1]), float(a[2])) for a in s.attempts]
    runs.setdefault(resident, []).append((sol, att, s.nfev))
  for k, v in runs.items():
    name = "resident" if k else "host"
    for j in range(1, len(v)):
        same_sol = torch.equal(v[0][0], v[j][0])
        same_att = v[0][1] == v[j][1]
        first = next((i for i, (a, b) in enumerate(zip(v[0][1], v[j][1])) if a != b), None)
        print(f"  {name} run 0 vs {j}: solution bitwise {same_sol}, attempts bitwise {same_att}, nfev {v[0][2]} / {v[j][2]}, "
              f"first differing attempt {first}", flush=True)
  a0, a1 = runs[True][0][1], runs[False][0][1]
  first = next((i for i, (a, b) in enumerate(zip(a0, a1)) if a != b), None)
  print("  resident vs host: first differing attempt", first, a0[first] if first is not None else "",
        a1[first] if first is not None else "", flush=True)
