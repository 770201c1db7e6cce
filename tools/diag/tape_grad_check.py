"""Per method, v6 / v4 fixed-grid training gradients against the fp64 oracle, next to the
reference's own fp32 error (env KIND, NPTS, B): max |gpu - fp64| / max|fp64| per parameter tensor."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from oracle import torch_ref as O  # noqa: E402
from conftest import golden_sd, load_golden  # noqa: E402

kind = os.environ.get("KIND", "kanfet")
npts = int(os.environ.get("NPTS", "6"))
B = int(os.environ.get("B", "64"))
dev = torch.device("cuda:0")
lib = _lib.load()
g = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
sd = golden_sd(g)
t = torch.from_numpy(g["t35"])[:npts]
y0 = O.lv_y0(B, seed=9)
w = torch.randn(npts, B, 2, generator=torch.Generator().manual_seed(6))
skip = ("grid", "prev_x", "branch_sign")
for method in ["rk4", "rk4_classic", "midpoint", "euler"]:
    ref = {}
    for dt in (torch.float32, torch.float64):
        ps = {k: v.clone().to(dt).requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
        r = (O.KANFETRef.from_state_dict(ps, 2) if kind == "kanfet"
             else O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)]))
        yc = y0.clone().to(dt).requires_grad_(True)
        (O.odeint(lambda tt, yy: r(yy), yc, t, method=method) * w.to(dt)).sum().backward()
        ref[dt] = {"y0": yc.grad, **{n: ps[n].grad for n in ps if ps[n].grad is not None}}
    rows = {}
    for lab, small in (("v6", 1 << 40), ("v4", 0)):
        prev = lib.fetode_fused_set_small_batch_max(small)
        m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        yg = y0.clone().to(dev).requires_grad_(True)
        (F.odeint(F.autonomous(m), yg, t, method=method) * w.to(dev)).sum().backward()
        lib.fetode_fused_set_small_batch_max(prev)
        got = {"y0": yg.grad.cpu(), **{n: p.grad.cpu() for n, p in m.named_parameters()}}
        rows[lab] = got
    print(method)
    for n in ref[torch.float64]:
        e64 = ref[torch.float64][n].double()
        sc = e64.abs().max().item() + 1e-12
        r32 = (ref[torch.float32][n].double() - e64).abs().max().item() / sc
        r6 = (rows["v6"][n].double() - e64).abs().max().item() / sc
        r4 = (rows["v4"][n].double() - e64).abs().max().item() / sc
        flag = " <--" if max(r6, r4) > 4 * r32 + 1e-5 else ""
        print(f"  {n:32s} ref32 {r32:.2e}  v6 {r6:.2e}  v4 {r4:.2e}{flag}", flush=True)
