"""Isolate a wrong fused-field term: evaluate variants of the golden field with parts zeroed."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import fet_ode_amd as F
from oracle import torch_ref as O
from tests.conftest import load_golden, golden_sd

g = load_golden("traj_kanfet"); sd0 = golden_sd(g)
tag = os.environ.get("FETODE_FUSED_LPT", "auto")
B = 8
torch.manual_seed(0)
x = 0.5 + 2.5 * torch.rand(B, 2)

def run(name, sd, kan=False):
    if kan:
        sdk = {k.replace(".kan.", "."): v for k, v in sd.items() if ".kan." in k}
        m = F.KAN([2, 10, 2], grid_size=5); m.load_state_dict(sdk); m = m.cuda()
        r = O.KANRef([O.KANLinearParams.from_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sdk.items()}, f"layers.{l}.") for l in range(2)])
    else:
        m = F.KANFET([2, 10, 2], grid_size=5); m.load_state_dict(sd); m = m.cuda()
        r = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
    with torch.no_grad():
        f = m(x.cuda()).cpu().double(); rr = r(x.double())
    print(f"{tag} {name:22s} rel {((f - rr).norm(dim=1) / rr.norm(dim=1).clamp_min(1e-9)).max().item():.2e}  gpu[0] {f[0].tolist()} ref[0] {rr[0].tolist()}", flush=True)

def zero(sd, pred):
    return {k: (torch.zeros_like(v) if pred(k) else v) for k, v in sd.items()}

run("full", sd0)
run("kan only", sd0, kan=True)
run("ferro coef=0", zero(sd0, lambda k: k.endswith("ferro.coef")))
run("kan weights=0", zero(sd0, lambda k: any(k.endswith(s) for s in ("base_weight", "spline_weight", "logistic_weight"))))
run("no logistic", zero(sd0, lambda k: k.endswith("logistic_weight")))
run("no spline", zero(sd0, lambda k: k.endswith("spline_weight")))
run("no base", zero(sd0, lambda k: k.endswith("base_weight")))
