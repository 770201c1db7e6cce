"""Exit-time crash under rocprofv3: run one workload, then write
/proc/self/maps to gpurun_out/maps_<mode>.txt so the PCs of a crash in exit() can be mapped to
their library (tools/diag/resolve_pcs.py).

  mode torch   : torch only (a cuda tensor, one kernel) - no fet_ode_amd at all
  mode fetode  : one fused rk4 solve through fet_ode_amd (registers its exit-time release hooks)
  mode nohooks : as fetode, with the package's atexit release hooks unregistered first
  mode rk4only : as fetode without the resident dopri5 solve (no cooperative launch)
"""
import atexit
import os
import sys

mode = sys.argv[1] if len(sys.argv) > 1 else "fetode"
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

dev = torch.device("cuda:0")
if mode == "torch":
    x = torch.randn(1 << 20, device=dev)
    print("torch sum", float((x * 2).sum()))
else:
    import fet_ode_amd as F
    if mode == "nohooks":
        from fet_ode_amd import dopri5 as D5, odeint as OD
        for fn in (D5._T_DEV.clear, D5._drop_last_solve, OD._clear_last_t):
            atexit.unregister(fn)
        print("unregistered the package's 3 exit hooks")
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    y0 = (0.5 + 2.5 * torch.rand(4096, 2)).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    with torch.no_grad():
        for _ in range(3):
            sol = F.odeint(F.autonomous(m), y0, t, method="rk4")
        sol2 = sol if mode == "rk4only" else F.odeint(F.autonomous(m), y0, t)   # resident dopri5 (cooperative)
    torch.cuda.synchronize()
    print("solve ok", float(sol[-1].abs().sum()), float(sol2[-1].abs().sum()))
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
with open(f"/proc/{os.getpid()}/maps") as f, open(os.path.join(REPO, "gpurun_out", f"maps_{mode}.txt"), "w") as o:
    o.write(f.read())
print("maps written, exiting", flush=True)
