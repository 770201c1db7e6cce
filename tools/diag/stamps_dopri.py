"""Per-phase cycle attribution of the resident dopri5 (DOPRI instantiation of the v4 kernel),
per attempt and wave (build: make -C fet-ode_amd/csrc stamps).
Run: FETODE_LIB=fet-ode_amd/libfetode_stamps.so python tools/diag/stamps_dopri.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

PH = ["X feats+bar", "grid sum", "edges0+h", "H feats", "barrier2", "edges1+k", "stage combine", "control"]
dev = torch.device("cuda:0")
lib = _lib.load()
lib.fetode_debug_stamp_buffer.argtypes = [ctypes.c_void_p]
for B in [int(v) for v in os.environ.get("STAMP_B", "2,512,4096").split(",")]:
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2]).to(dev)
    f = F.autonomous(m)
    y0 = O.lv_y0(B).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    nb = (B + 1) // 2
    buf = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
    with torch.no_grad():
        F.odeint(f, y0, t, rtol=1e-3, atol=1e-4)
        torch.cuda.synchronize()
        _lib.check(lib.fetode_debug_stamp_buffer(buf.data_ptr()), "stamp buffer")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        F.odeint(f, y0, t, rtol=1e-3, atol=1e-4)
        e1.record()
        torch.cuda.synchronize()
        _lib.check(lib.fetode_debug_stamp_buffer(None), "stamp buffer")
    n_att = F.dopri5.dopri5_solve.last.n_attempts
    st = buf.view(nb, 8).double().cpu().numpy() / n_att
    tot = st.sum(1)
    print(f"B={B}: solve {e0.elapsed_time(e1):.3f} ms, {n_att} attempts; shader cycles (s_memtime) per "
          f"attempt per wave: total {tot.mean():.0f} (p10 {np.percentile(tot, 10):.0f}, p90 {np.percentile(tot, 90):.0f})")
    for p in range(8):
        print(f"   {PH[p]:14s} {st[:, p].mean():8.0f}  ({100 * st[:, p].mean() / tot.mean():4.1f}%)")
