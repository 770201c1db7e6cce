"""Host-side overhead of one fused training iteration (cProfile over 30 iterations, GPU synced
per iteration) — where the time between kernels goes."""
import cProfile, os, pstats, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
from oracle import torch_ref as O

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2]).to(dev)
y0 = O.lv_y0(4096).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
fused = os.environ.get("FUSED_ADAM", "1") == "1"
opt = torch.optim.Adam(m.parameters(), lr=1e-4, fused=fused)
f = F.autonomous(m)

def it():
    opt.zero_grad(set_to_none=True)
    sol = F.odeint(f, y0, t, method="rk4")
    sol.square().mean().backward()
    opt.step()

for _ in range(5):
    it()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(30):
    it()
torch.cuda.synchronize()
print(f"ms/iter {1e3 * (time.perf_counter() - t0) / 30:.3f} (fused adam {fused})")
# host time of each phase without syncing inside the iteration
ph = {"zero": 0, "fwd": 0, "loss+bwd": 0, "step": 0}
for _ in range(30):
    a = time.perf_counter(); opt.zero_grad(set_to_none=True); b = time.perf_counter()
    sol = F.odeint(f, y0, t, method="rk4"); c = time.perf_counter()
    sol.square().mean().backward(); d = time.perf_counter()
    opt.step(); e = time.perf_counter()
    ph["zero"] += b - a; ph["fwd"] += c - b; ph["loss+bwd"] += d - c; ph["step"] += e - d
torch.cuda.synchronize()
print("host ms/iter by phase:", {k: round(1e3 * v / 30, 3) for k, v in ph.items()})
pr = cProfile.Profile()
pr.enable()
for _ in range(30):
    it()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
