"""Graph-captured training iteration vs eager, step by step from identical states: loss, gradients
and parameters after each of the first iterations (finds what a replay does not redo)."""
import copy
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
T = 35
torch.manual_seed(0)
base = F.KANFET([2, 10, 2], grid_size=5)
g = torch.Generator().manual_seed(0)
y0 = (0.5 + 2.5 * torch.rand(4096, 2, generator=g)).to(dev)
t = torch.tensor(np.linspace(0, 3.5, T))
target = torch.zeros(T, 4096, 2, device=dev)


def make():
    m = copy.deepcopy(base).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True)
    func = F.autonomous(m)
    out = {}

    def it():
        opt.zero_grad(set_to_none=False)
        sol = F.odeint(func, y0, t, method="rk4")
        loss = (sol - target).square().mean()
        loss.backward()
        opt.step()
        out["loss"] = loss
        return loss
    return m, opt, it, out


def snap(m):
    return [p.detach().clone() for p in m.parameters()], [p.grad.detach().clone() for p in m.parameters()]


m1, o1, it1, out1 = make()
m2, o2, it2, out2 = make()
for _ in range(3):
    it1()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        it2()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
p1, g1 = snap(m1)
p2, g2 = snap(m2)
print("after warmup: params equal", all(torch.equal(a, b) for a, b in zip(p1, p2)),
      "state equal", torch.equal(m1._fetode_state, m2._fetode_state))
F._lib._PARAM_GEN[0] += 1
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    it2()
torch.cuda.synchronize()
p2b, _ = snap(m2)
print("capture changed params:", not all(torch.equal(a, b) for a, b in zip(p2, p2b)),
      "state equal after capture", torch.equal(m1._fetode_state, m2._fetode_state))
for k in range(3):
    it1()
    graph.replay()
    torch.cuda.synchronize()
    p1, g1 = snap(m1)
    p2, g2 = snap(m2)
    dp = max((a - b).abs().max().item() for a, b in zip(p1, p2))
    dg = max((a - b).abs().max().item() for a, b in zip(g1, g2))
    print(f"iter {k}: loss eager {out1['loss'].item():.9g} graph {out2['loss'].item():.9g}  max|dparam| {dp:.3e} "
          f"max|dgrad| {dg:.3e} state equal {torch.equal(m1._fetode_state, m2._fetode_state)}")
