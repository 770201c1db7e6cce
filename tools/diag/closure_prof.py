"""cProfile of the host side of the literal drop-in: odeint(lambda t, y: model(y), ...) at
B = 4096, rk4, 35 points (the per-stage path, bench.py lv_plain_closure)."""
import cProfile, os, pstats, sys, time
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import fet_ode_amd as F  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
func = lambda tt, yy: m(yy)  # noqa: E731
t = torch.tensor(np.linspace(0, 3.5, 35))
y0 = O.lv_y0(4096).to(dev)
with torch.no_grad():
    for _ in range(3):
        F.odeint(func, y0, t, method="rk4")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        F.odeint(func, y0, t, method="rk4")
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / 10 * 1e3:.3f} ms per plain-closure solve", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        F.odeint(func, y0, t, method="rk4")
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
