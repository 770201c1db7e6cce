"""Capture the LV training iteration (bench.py train_rate: fused rk4 solve with tape + loss +
reverse sweep + fused Adam) in a HIP graph (torch.cuda.CUDAGraph) and compare: time per iteration
eager vs replay, and the parameters after N iterations both ways (same math, same kernels)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
T = 35


def setup():
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    g = torch.Generator().manual_seed(0)
    y0 = (0.5 + 2.5 * torch.rand(4096, 2, generator=g)).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, T))
    opt = torch.optim.Adam(m.parameters(), lr=1e-4, fused=True, capturable=True)
    target = torch.zeros(T, 4096, 2, device=dev)
    func = F.autonomous(m)

    def it():
        opt.zero_grad(set_to_none=False)
        sol = func_solve()
        loss = (sol - target).square().mean()
        loss.backward()
        opt.step()
        return loss

    def func_solve():
        return F.odeint(func, y0, t, method="rk4")
    return m, opt, it


N = int(os.environ.get("N", 50))
# eager
m1, o1, it1 = setup()
for _ in range(3):
    it1()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    it1()
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / N
# graph
m2, o2, it2 = setup()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        it2()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
F._lib._PARAM_GEN[0] += 1       # the captured iteration must include the plan rebuild
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    it2()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    graph.replay()
torch.cuda.synchronize()
rep = (time.perf_counter() - t0) / N
# the capture did not run the iteration; m2 is 3 + N iterations in, like m1
d = max((a - b).abs().max().item() for a, b in zip(m1.parameters(), m2.parameters()))
same = all(torch.equal(a, b) for a, b in zip(m1.parameters(), m2.parameters()))
print(f"eager {eager * 1e3:.3f} ms/iter = {34 / eager:.0f} steps/s; graph replay {rep * 1e3:.3f} ms/iter = "
      f"{34 / rep:.0f} steps/s; params after {3 + N} iters: bitwise equal {same}, max diff {d:.3e}")
