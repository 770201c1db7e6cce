"""Training-iteration A/B for whatever library FETODE_LIB names: the bench's LV KAN-FET rk4 training
step (B = 4096, 34 steps) — forward (taped) and backward (reverse sweep) timed apart with HIP events,
clocks settled first."""
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
fw, bw = [], []
for it in range(40):
    m.zero_grad(set_to_none=True)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    loss = F.odeint(f, y0, t, method="rk4").square().mean()
    e[1].record()
    loss.backward()
    e[2].record()
    torch.cuda.synchronize()
    if it >= 10:
        fw.append(e[0].elapsed_time(e[1]))
        bw.append(e[1].elapsed_time(e[2]))
print(json.dumps({"lib": os.path.basename(os.environ.get("FETODE_LIB", "libfetode.so")), "tag": os.environ.get("AB_TAG", ""),
                  "fwd_ms": float(np.median(fw)), "bwd_ms": float(np.median(bw))}), flush=True)
