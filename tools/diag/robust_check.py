"""Bench-config robust-subset parity of the fused forward (bench.py's `parity.robust_subset`) for
the library FETODE_LIB: the CPU references (oracle fp32 solve, fp64 solve, 5 perturbed fp32
solves) are computed once and cached in gpurun_out/robust_ref.pt; prints one JSON line."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
from oracle import torch_ref as O
from oracle import parity as P

torch.manual_seed(0)
model = F.KANFET([2, 10, 2], grid_size=5)
sd = {k: v.clone() for k, v in model.state_dict().items()}
g = torch.Generator().manual_seed(0)
y0 = (0.5 + 2.5 * torch.rand(4096, 2, generator=g)).to(torch.float32)
t = torch.tensor(np.linspace(0, 3.5, 35))
cache = "gpurun_out/robust_ref.pt"
if os.path.exists(cache):
    ref = torch.load(cache, weights_only=True)
else:
    torch.set_num_threads(16)
    with torch.no_grad():
        r32 = O.KANFETRef.from_state_dict(sd, 2)
        e32 = O.odeint(lambda tt, yy: r32(yy), y0, t, method="rk4")
        r64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
        e64 = O.odeint(lambda tt, yy: r64(yy), y0.double(), t, method="rk4")
    runs = P.perturbed_solves(sd, y0, t, 5)
    ref = {"e32": e32, "e64": e64, "runs": torch.stack(runs)}
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(ref, cache)
dev = torch.device("cuda:0")
with torch.no_grad():
    sol = F.odeint(F.autonomous(model.to(dev)), y0.to(dev), t, method="rk4").cpu()
runs = list(ref["runs"])
st = P.robust_parity(sol, ref["e32"], ref["e64"], runs[:3], runs[3:])
st["ok"] = P.robust_parity_ok(st)
st["lib"] = os.path.basename(os.environ.get("FETODE_LIB", "libfetode.so"))
print(json.dumps(st), flush=True)
