"""The bench's training iteration (bench.train_rate: fused rk4 solve with tape, loss, reverse
sweep, gradient all-reduce, fused Adam) at B = 4096, for kernel traces: ITERS iterations."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
import fet_ode_amd.dist as D
from oracle import torch_ref as O

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = F.KANFET([2, 10, 2]).to(dev)
y0 = O.lv_y0(int(os.environ.get("B", "4096"))).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
opt = torch.optim.Adam(m.parameters(), lr=1e-4, fused=True)
f = F.autonomous(m)
target = torch.zeros(35, y0.shape[0], 2, device=dev)
n = int(os.environ.get("ITERS", "10"))
for i in range(n):
    opt.zero_grad(set_to_none=True)
    sol = F.odeint(f, y0, t, method="rk4")
    loss = (sol - target).square().mean()
    loss.backward()
    D.allreduce_gradients(list(m.parameters()))
    opt.step()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for i in range(n):
    opt.zero_grad(set_to_none=True)
    sol = F.odeint(f, y0, t, method="rk4")
    loss = (sol - target).square().mean()
    loss.backward()
    D.allreduce_gradients(list(m.parameters()))
    opt.step()
ev1.record()
torch.cuda.synchronize()
print(f"{ev0.elapsed_time(ev1) / n:.3f} ms per training iteration (B={y0.shape[0]})", flush=True)
