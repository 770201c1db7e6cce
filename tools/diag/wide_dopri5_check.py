"""Resident vs host-loop wide dopri5, side by side: the first attempts' error ratios (as fp64 bits),
the per-output-time max difference.  FETODE_WIDE_DOPRI_GRID caps the persistent grid."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import dopri5, ett  # noqa: E402,F401

dev = torch.device("cuda:0")
B = int(os.environ.get("B", 1))
torch.manual_seed(0)
dyn = ett.KANFETDynamics(64, hidden=128).to(dev)
sd = {k: v.clone() for k, v in dyn.state_dict().items()}
g = torch.Generator().manual_seed(3)
z0 = (torch.randn(B, 64, generator=g) * 0.6).to(dev)
t = torch.linspace(0.0, 3.0, steps=4, device=dev)
out = {}
for resident in (False, True):
    F.dopri5.set_wide_resident_dopri5(resident, gap=(0, 0))
    dyn.load_state_dict(sd)
    dyn.net.reset_state()
    with torch.no_grad():
        sol = F.odeint(dyn, z0, t, method="dopri5", rtol=1e-3, atol=1e-4)
    s = F.dopri5.dopri5_solve.last
    out[resident] = (sol, s.attempts, s.nfev)
(sh, ah, nh), (sr, ar, nr) = out[False], out[True]
print(f"B={B} grid cap {os.environ.get('FETODE_WIDE_DOPRI_GRID', 'auto')}: nfev {nh} / {nr}, attempts {len(ah)} / {len(ar)}")
for i, (a, b) in enumerate(zip(ah, ar)):
    if i < 8 or a[2] != b[2]:
        print(f"  att {i}: host dt {a[1]!r} ratio {a[2]!r} | res dt {b[1]!r} ratio {b[2]!r}")
    if i > 30:
        break
for j in range(sh.shape[0]):
    print(f"  t[{j}] max|diff| {(sr[j] - sh[j]).abs().max().item():.3e}  scale {sh[j].abs().max().item():.3e}")
