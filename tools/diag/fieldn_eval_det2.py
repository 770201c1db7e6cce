"""Where fieldn's run-to-run differences come from: the same model evaluated repeatedly (one plan)
vs fresh models (fresh plans); plan bytes compared bitwise."""
import os
import sys

import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import fet_ode_amd as F  # noqa: E402,F401
from fet_ode_amd.autograd_ops import build_plan, make_handle  # noqa: E402
from test_gpu_fieldn import _model, _y0  # noqa: E402

dev = torch.device("cuda:0")
B = 1000
y0 = _y0(B, 4, seed=7).to(dev)
m = _model("kan", [4, 32, 4], 0).to(dev)
with torch.no_grad():
    a = [m(y0).cpu() for _ in range(6)]
print("same model:", [torch.equal(a[0], x) for x in a[1:]], flush=True)
plans, outs = [], []
for rep in range(4):
    mm = _model("kan", [4, 32, 4], 0).to(dev)
    with torch.no_grad():
        outs.append(mm(y0).cpu())
    h = make_handle(mm, B, dev)
    plans.append(build_plan(mm, h, dev).cpu().clone())
print("fresh models, outputs:", [torch.equal(outs[0], x) for x in outs[1:]], flush=True)
print("fresh models, plans:", [torch.equal(plans[0], x) for x in plans[1:]], plans[0].numel(), flush=True)
for x in plans[1:]:
    d = (plans[0] != x).nonzero().flatten()
    print("  plan words differing:", d[:20].tolist(), flush=True)
for x in outs[1:]:
    d = (outs[0] != x).nonzero()
    print("  output entries differing:", d[:10].tolist(), len(d), flush=True)
torch.cuda.synchronize()
# the same inputs through per-row single launches (B = 1): which rows' values move?
