"""ECG dopri5 timing: device-resident vs host-driven solve of No_MLP_KANODEFunc (B=200, latent 64).
N (default 20) timed solves per path; WARM (default 3) untimed solves first — a long WARM shows
whether short runs are measured at a low clock.  With FETODE_LIB=fet-ode_amd/libfetode_stamps.so
(make -C fet-ode_amd/csrc stamps) it also prints workgroup 0's phase shares and clock."""
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
n = int(os.environ.get("N", "20"))
warm = int(os.environ.get("WARM", "3"))
for resident in (True, False):
    D5.set_resident_dopri5(resident)
    with torch.no_grad():
        for _ in range(warm):
            F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
        torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / n
    print(f"resident={resident}: {el * 1e3:.3f} ms per solve, nfev {D5.dopri5_solve.last.nfev}", flush=True)

# phase breakdown (s_memrealtime, 100 MHz) of workgroup 0, averaged over 10 resident solves run
# right after WARM more; slots 5/6: the kernel's s_memtime / s_memrealtime totals -> shader clock
import ctypes
from fet_ode_amd import _lib
lib = _lib.load()
if hasattr(lib, "fetode_debug_ecg_stamps"):
    lib.fetode_debug_ecg_stamps.argtypes = [ctypes.c_void_p]
    st = torch.zeros(8, dtype=torch.int64, device=dev)
    D5.set_resident_dopri5(True)
    with torch.no_grad():
        for _ in range(warm):
            F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
        lib.fetode_debug_ecg_stamps(st.data_ptr())
        for _ in range(10):
            F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4)
    torch.cuda.synchronize()
    lib.fetode_debug_ecg_stamps(None)
    s = st.tolist()
    v = [x / 1000.0 for x in s[:5]]
    print("WG0 us per solve: other %.1f features %.1f head %.1f partials %.1f norms %.1f" % tuple(v))
    if s[6]:
        print(f"in-kernel clock {s[5] / s[6] * 0.1:.3f} GHz", flush=True)
