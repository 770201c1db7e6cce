"""Host issue time vs wall time of the bench's training iteration (B = 4096): if the host needs
about as long to issue an iteration as the GPU needs to run it, the loop is host-bound."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
import fet_ode_amd.dist as D
from oracle import torch_ref as O

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2]).to(dev)
y0 = O.lv_y0(4096).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
opt = torch.optim.Adam(m.parameters(), lr=1e-4, fused=True)
f = F.autonomous(m)
target = torch.zeros(35, 4096, 2, device=dev)


def it():
    opt.zero_grad(set_to_none=True)
    sol = F.odeint(f, y0, t, method="rk4")
    (sol - target).square().mean().backward()
    D.allreduce_gradients(list(m.parameters()))
    opt.step()


for _ in range(10):
    it()
torch.cuda.synchronize()
n = 50
t0 = time.perf_counter()
for _ in range(n):
    it()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host issue {1e3 * (t1 - t0) / n:.3f} ms/iter, wall {1e3 * (t2 - t0) / n:.3f} ms/iter", flush=True)
