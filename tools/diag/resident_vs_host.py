"""Resident (one-launch) vs host-driven dopri5 on the tagged LV fields: first attempt where the
two control sequences part, with t/dt/ratio on both sides."""
import sys
import numpy as np
import torch

sys.path.insert(0, "tests")
from conftest import golden_sd, load_golden  # noqa: E402
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd.dopri5 import set_resident_dopri5  # noqa: E402

dev = torch.device("cuda:0")
for kind in ("kanfet", "kan"):
    for B in (1, 64, 1000, 4096):
        gk = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
        y0 = torch.from_numpy(gk["y0_B64"]).repeat(64, 1)[:B].to(dev)
        t = torch.tensor([0.0, 0.2, 0.5], dtype=torch.float64)
        res = []
        for resident in (True, False):
            set_resident_dopri5(resident)
            m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
            m.load_state_dict(golden_sd(gk))
            m = m.to(dev)
            with torch.no_grad():
                sol = F.odeint(F.autonomous(m), y0, t, rtol=1e-3, atol=1e-4).cpu()
            s = F.dopri5.dopri5_solve.last
            res.append((sol, list(s.attempts), s.nfev, type(s).__name__))
        set_resident_dopri5(True)
        (s0, a0, n0, k0), (s1, a1, n1, k1) = res
        first = next((i for i, (x, y) in enumerate(zip(a0, a1)) if x[3] != y[3] or abs(x[1] - y[1]) > 1e-6 * abs(y[1])), None)
        rel = ((s0 - s1).norm(dim=(1, 2)) / s1.norm(dim=(1, 2))).max().item()
        print(f"{kind} B={B}: {k0} n={len(a0)} nfev={n0} | {k1} n={len(a1)} nfev={n1} | sol rel {rel:.2e} | first diff {first}")
        if first is not None:
            for i in range(max(0, first - 2), min(first + 3, len(a0), len(a1))):
                print("   ", i, "res", tuple(float(v) for v in a0[i]), "host", tuple(float(v) for v in a1[i]))
        r0 = np.array([a[2] for a in a0[:len(a1)]])
        r1 = np.array([a[2] for a in a1[:len(a0)]])
        k = min(len(r0), len(r1), first if first is not None else 10**9)
        if k:
            print("    ratio rel diff before divergence: max %.2e" % (np.abs(r0[:k] - r1[:k]) / np.abs(r1[:k]).clip(1e-30)).max())
