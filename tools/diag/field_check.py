"""Single-evaluation check of the fused field against the fp64 oracle (fresh state, then a
second call with carried state), for whatever variant FETODE_FUSED_LPT selects."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import fet_ode_amd as F
from oracle import torch_ref as O
from tests.conftest import load_golden, golden_sd

g = load_golden("traj_kanfet"); sd = golden_sd(g)
tag = os.environ.get("FETODE_FUSED_LPT", "auto")
for B in (1, 2, 3, 64, 1000):
    torch.manual_seed(B)
    x = 0.5 + 2.5 * torch.rand(B, 2)
    x2 = x + 0.05 * torch.randn(B, 2)
    m = F.KANFET([2, 10, 2], grid_size=5); m.load_state_dict(sd); m = m.cuda()
    r = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
    with torch.no_grad():
        f1 = m(x.cuda()).cpu().double(); r1 = r(x.double())
        f2 = m(x2.cuda()).cpu().double(); r2 = r(x2.double())
        p0 = m.layers[0].ferro._prev.cpu().double(); p1 = m.layers[1].ferro._prev.cpu().double()
    e1 = ((f1 - r1).norm(dim=1) / r1.norm(dim=1)).max().item()
    e2 = ((f2 - r2).norm(dim=1) / r2.norm(dim=1)).max().item()
    ep0 = (p0 - x2.double()).abs().max().item()
    print(f"{tag} B={B:5d}: eval1 {e1:.2e} eval2 {e2:.2e} prev0 err {ep0:.2e} prev1 shape {tuple(p1.shape)}", flush=True)
