import sys, os, torch, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import fet_ode_amd as F
from fet_ode_amd import _lib
from oracle import torch_ref as O
from conftest import load_golden, golden_sd
lib = _lib.load(); dev = torch.device("cuda:0")
g = load_golden("traj_kanfet"); sd = golden_sd(g)
y0 = (torch.rand(2048, 2, generator=torch.Generator().manual_seed(8), dtype=torch.float64) * 8 - 4).float()
skip = ("grid", "prev_x", "branch_sign")
t2 = torch.from_numpy(g["t35"])[:2]
def gpu(mode, t, small=None):
    lib.fetode_backward_set_v7(mode)
    m = F.KANFET([2, 10, 2], grid_size=5); m.load_state_dict(sd); m = m.to(dev)
    yg = y0.clone().to(dev).requires_grad_(True)
    F.odeint(F.autonomous(m), yg, t, method="rk4").square().mean().backward()
    return {"y0": yg.grad.cpu().double(), **{n: p.grad.cpu().double() for n, p in m.named_parameters()}}
def oracle(dt, t):
    ps = {k: v.clone().to(dt).requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
    ref = O.KANFETRef.from_state_dict(ps, 2)
    yc = y0.clone().to(dt).requires_grad_(True)
    O.odeint(lambda tt, yy: ref(yy), yc, t, method="rk4").square().mean().backward()
    return {"y0": yc.grad.double(), **{n: ps[n].grad.double() for n in ps if ps[n].grad is not None}}
e64, e32 = oracle(torch.float64, t2), oracle(torch.float32, t2)
g0, g2 = gpu(0, t2), gpu(2, t2)
m = lambda a, b: (a - b).abs().max().item()
for n in e64:
    sc = e64[n].abs().max().item()
    print(f"{n:34s} ref32 {m(e32[n], e64[n])/sc:.2e}  one-kernel {m(g0[n], e64[n])/sc:.2e}  lane {m(g2[n], e64[n])/sc:.2e}")
