"""ECG dopri5 timing: device-resident vs host-driven solve of No_MLP_KANODEFunc (B=200, latent 64)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import fet_ode_amd as F
from fet_ode_amd import dopri5 as D5
from fet_ode_amd import ecg

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = ecg.No_MLP_KANODEFunc(latent_dim=64, num_basis=10).to(dev)
h0 = torch.randn(int(os.environ.get("B", "200")), 64, device=dev)
t = torch.tensor([0.0, 1.0])
for resident in (True, False):
    D5.set_resident_dopri5(resident)
    with torch.no_grad():
        for _ in range(3):
            F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 20
        for _ in range(n):
            F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
        torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / n
    print(f"resident={resident}: {el * 1e3:.3f} ms per solve, nfev {D5.dopri5_solve.last.nfev}", flush=True)

# phase breakdown (s_memrealtime, 100 MHz) of workgroup 0 in one resident solve, when the
# library was built with the debug stamps hook
import ctypes
from fet_ode_amd import _lib
lib = _lib.load()
if hasattr(lib, "fetode_debug_ecg_stamps"):
    lib.fetode_debug_ecg_stamps.argtypes = [ctypes.c_void_p]
    st = torch.zeros(4, dtype=torch.int64, device=dev)
    lib.fetode_debug_ecg_stamps(st.data_ptr())
    D5.set_resident_dopri5(True)
    with torch.no_grad():
        F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
    torch.cuda.synchronize()
    lib.fetode_debug_ecg_stamps(None)
    v = [x / 100.0 for x in st.tolist()]
    print("WG0 us: features %.1f head %.1f norm+barrier %.1f rest %.1f" % tuple(v))
