"""Taped (training) forward of the bench's LV KAN-FET rk4 solve (B = 4096, 34 steps) timed alone:
50 back-to-back calls under autograd between two HIP events, no backward (A/B of tape-store
variants; FETODE_LIB selects the library).  Clocks settled first."""
import json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import bench
import fet_ode_amd as F

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
y0 = bench.lv_y0(4096, 0).to(dev)
f = F.autonomous(m)
with torch.no_grad():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for _ in range(20):
            F.odeint(f, y0, t, method="rk4")
        torch.cuda.synchronize()
res = {}
for mode in ("taped", "inference"):
    ts = []
    for rep in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.set_grad_enabled(mode == "taped"):
            sols = []
            e0.record()
            for _ in range(50):
                sols.append(F.odeint(f, y0, t, method="rk4"))
            e1.record()
            torch.cuda.synchronize()
        del sols
        ts.append(e0.elapsed_time(e1) / 50 * 1e3)
    res[mode + "_us"] = float(np.median(ts))
print(json.dumps({"lib": os.path.basename(os.environ.get("FETODE_LIB", "libfetode.so")),
                  "tag": os.environ.get("AB_TAG", ""), **res}), flush=True)
