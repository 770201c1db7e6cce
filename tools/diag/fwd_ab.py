"""Kernel time of the bench's rk4 solve (LV KAN-FET) at a few batches with whatever library
FETODE_LIB names — run once per A/B library.  Clocks settled first (~1 s of B = 4096 solves)."""
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
with torch.no_grad():
    y4 = bench.lv_y0(4096, 0).to(dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for _ in range(20):
            F.odeint(F.autonomous(m), y4, t, method="rk4")
        torch.cuda.synchronize()
r = {"lib": os.path.basename(os.environ.get("FETODE_LIB", "libfetode.so")), "tag": os.environ.get("AB_TAG", "")}
for B in [int(b) for b in os.environ.get("AB_B", "512,4096").split(",")]:
    r[f"B{B}_us"] = 1e3 * bench.kernel_time_ms(m, bench.lv_y0(B, 0).to(dev), t, reps=100)
print(json.dumps(r), flush=True)
