"""Fused fieldn training gradients vs the per-stage GPU path, the fp64 oracle and the oracle in
fp32 (the reference's own precision: the yardstick), per parameter: max |diff| / max |ref|."""
import os
import sys

import numpy as np
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))
import fet_ode_amd as F  # noqa: E402
from test_gpu_fieldn_train import _gpu_grads, _model, _oracle_grads, _y0  # noqa: E402

dev = torch.device("cuda:0")
for kind, widths, K in (("kan", [4, 32, 4], 0), ("kanfet", [2, 16, 2], 12), ("kanfet", [3, 8, 3], 6)):
    for method in ("rk4", "euler"):
        B, D = 48, widths[0]
        npts = int(os.environ.get("NPTS", "6"))
        t = torch.tensor(np.linspace(0, 0.5, npts))
        y0 = _y0(B, D)
        target = 0.3 * torch.ones(npts, B, D)
        sd = {k: v.clone() for k, v in _model(kind, widths, K).state_dict().items()}
        res = {}
        for fused in (True, False):
            prev = F.set_fused_training(fused)
            try:
                m = _model(kind, widths, K).to(dev)
                m.load_state_dict(sd)
                res[fused] = _gpu_grads(m, y0, t, method, target, dev)[2]
            finally:
                F.set_fused_training(prev)
        _, e64 = _oracle_grads(kind, sd, y0, t, method, target)
        sd32 = {k: v.float() for k, v in sd.items()}
        from oracle import torch_ref as O
        from test_gpu_fieldn_train import SKIP, _oracle
        ps = {k: v.detach().cpu().float().clone().requires_grad_(k.split(".")[-1] not in SKIP) for k, v in sd.items()}
        ref = _oracle(kind, ps)
        yc = y0.clone().float().requires_grad_(True)
        pr = O.odeint(lambda tt, yy: ref(yy), yc, t.float(), method=method)
        torch.mean(torch.square(pr - target.float())).backward()
        e32 = {"y0": yc.grad}
        e32.update({n: ps[n].grad for n in ps if ps[n].grad is not None})
        print(f"== {kind} {widths} K={K} {method}", flush=True)
        for n in res[True]:
            ex = e64[n].double()
            sc = ex.abs().max().item() + 1e-30

            def r(v):
                return (v.double().cpu() - ex).abs().max().item() / sc
            print(f"  {n:32s} fused {r(res[True][n]):.2e}  per-stage {r(res[False][n]):.2e}  ref-fp32 {r(e32[n]):.2e}"
                  f"  fused-vs-stage {(res[True][n] - res[False][n]).abs().max().item() / sc:.2e}", flush=True)
