"""Per-phase cycle attribution of the fused rk4 kernels (build: make -C fet-ode_amd/csrc stamps).
Run: FETODE_LIB=fet-ode_amd/libfetode_stamps.so STAMP_KERNEL=v7|tpw1|v6 STAMP_B=1,512 python tools/diag/stamps.py
v7 = fused4_kernel two trajectories per wave, tpw1 = fused4_kernel one per wave, v6 = small6_kernel
(wave 0 of each 3-wave workgroup).  Cycles are s_memtime ticks (shader clock)."""
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
from fet_ode_amd import _lib
from oracle import torch_ref as O

KERNEL = os.environ.get("STAMP_KERNEL", "v7")
PH = {"v8": ["L0 feats+gate+pair", "L0 fw+splines", "unit sum -> h", "L1", "wave sums", "exchange",
             "stage combine", "outputs+loop"],
      "v6": ["L0 feats+swap", "L0 pair+spline", "row sum -> h", "L1 feats+pair", "L1 spline+sums", "barrier+LDS",
             "stage combine", "outputs+loop"]}.get(
    KERNEL, ["X feats+bar", "step outputs", "edges0+h", "H feats", "barrier2", "edges1+k", "stage combine", "loop+sched"])
dev = torch.device("cuda:0")
lib = _lib.load()
lib.fetode_debug_stamp_buffer.argtypes = [ctypes.c_void_p]
BIG = 1 << 40
if KERNEL == "v7":
    lib.fetode_fused_set_tpw1_range(-1, 0)
    lib.fetode_fused_set_small_batch_max(0)
elif KERNEL == "tpw1":
    lib.fetode_fused_set_tpw1_range(0, BIG)
elif KERNEL == "v8":
    lib.fetode_fused_set_v8_range(0, BIG)
elif KERNEL == "v6":
    lib.fetode_fused_set_tpw1_range(-1, 0)
    lib.fetode_fused_set_small_batch_max(BIG)
for B in [int(v) for v in os.environ.get("STAMP_B", "4096,65536").split(",")]:
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2]).to(dev)
    f = F.autonomous(m)
    y0 = O.lv_y0(B).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    nb = (B + 1) // 2 if KERNEL == "v7" else B
    buf = torch.zeros(nb * 8, dtype=torch.int64, device=dev)
    with torch.no_grad():
        F.odeint(f, y0, t, method="rk4")
        torch.cuda.synchronize()
        _lib.check(lib.fetode_debug_stamp_buffer(buf.data_ptr()), "stamp buffer")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        F.odeint(f, y0, t, method="rk4")
        e1.record()
        torch.cuda.synchronize()
        _lib.check(lib.fetode_debug_stamp_buffer(None), "stamp buffer")
    st = buf.view(nb, 8).double().cpu().numpy() / 136.0   # per evaluation
    tot = st.sum(1)
    print(f"{KERNEL} B={B}: solve {e0.elapsed_time(e1):.3f} ms; cycles per evaluation per wave: "
          f"total {tot.mean():.0f} (p10 {np.percentile(tot, 10):.0f}, p90 {np.percentile(tot, 90):.0f})")
    for p in range(8):
        print(f"   {PH[p]:14s} {st[:, p].mean():8.0f}  ({100 * st[:, p].mean() / tot.mean():4.1f}%)")
