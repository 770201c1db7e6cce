"""Where does the taped resident dopri5 training path lose digits on the smooth KAN field?
Per parameter tensor, the relative error against the fp64 oracle's autograd of:
  res6   the default resident path (v6 taped forward at B <= small_max, the sweep's TPW choice)
  res4   the resident path with the v4 taped forward (fetode_fused_set_small_batch_max(0))
  host   autograd through the host-driven solver (_Dopri5Grad)
  ref32  the oracle's own fp32 autograd (reference op order on CPU): the reference's fp32 error
cases: env CASES="B:rtol,..." (default the gpu test grid), t = linspace(0, 2, 9), atol = rtol/10,
loss = sum(w * sol) as tests/test_gpu_dopri5_train.py."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402
from fet_ode_amd.dopri5 import set_resident_dopri5_training  # noqa: E402
from oracle import torch_ref as O  # noqa: E402
from conftest import golden_sd, load_golden  # noqa: E402

dev = torch.device("cuda:0")
g = load_golden("traj_kan")
sd = golden_sd(g)
names = [n for n, _ in F.KAN([2, 10, 2], grid_size=5).named_parameters()]
lib = _lib.load()
t = torch.tensor(np.linspace(0, 2.0, 9))


def inputs(B):
    y0 = torch.from_numpy(g["y0_B64"]).repeat((B + 63) // 64, 1)[:B].clone()
    w = torch.randn(len(t), B, 2, generator=torch.Generator().manual_seed(0))
    return y0, w


def gpu(B, rtol, resident, small=None):
    y0, w = inputs(B)
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    y = y0.to(dev).requires_grad_(True)
    prev = set_resident_dopri5_training(resident)
    ps = lib.fetode_fused_set_small_batch_max(-1)
    if small is not None:
        lib.fetode_fused_set_small_batch_max(small)
    try:
        sol = F.odeint(F.autonomous(m), y, t, rtol=rtol, atol=rtol * 0.1)
        nfev = F.dopri5.dopri5_solve.last.nfev
        (w.to(dev) * sol).sum().backward()
    finally:
        set_resident_dopri5_training(prev)
        lib.fetode_fused_set_small_batch_max(ps)
    gr = {n: p.grad.detach().cpu().double() for n, p in m.named_parameters()}
    gr["y0"] = y.grad.cpu().double()
    return gr, nfev, sol.detach().cpu().double()


def oracle(B, rtol, dtype):
    y0, w = inputs(B)
    ps = {k: v.clone().to(dtype).requires_grad_(k in names) for k, v in sd.items()}
    ref = O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)])
    y = y0.to(dtype).requires_grad_(True)
    tr = O.Dopri5Trace()
    sol = O.odeint(lambda tt, yy: ref(yy), y, t.to(torch.float64), rtol=rtol, atol=rtol * 0.1, trace=tr)
    gr = torch.autograd.grad((w.to(dtype) * sol).sum(), [ps[n] for n in names] + [y])
    out = {n: a.detach().double() for n, a in zip(names, gr[:-1])}
    out["y0"] = gr[-1].detach().double()
    return out, tr.nfev, sol.detach().double()


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


cases = os.environ.get("CASES", "1:1e-3,16:1e-3,64:1e-3,1:1e-2,16:1e-2,64:1e-2,1:1e-1,16:1e-1,64:1e-1")
allerr = {}   # path -> list of (case, tensor, error)
for c in cases.split(","):
    B, rtol = int(c.split(":")[0]), float(c.split(":")[1])
    o64, n64, s64 = oracle(B, rtol, torch.float64)
    row = {"B": B, "rtol": rtol, "nfev64": n64}
    for lab, fn in (("res6", lambda: gpu(B, rtol, True)), ("res4", lambda: gpu(B, rtol, True, 0)),
                    ("host", lambda: gpu(B, rtol, False)), ("ref32", lambda: oracle(B, rtol, torch.float32))):
        gr, nf, sol = fn()
        errs = {n: rel(gr[n], o64[n]) for n in o64}
        allerr.setdefault(lab, []).append(errs)
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
        row[lab] = {"nfev": nf, "sol": rel(sol, s64), "worst": [(k, float("%.3g" % v)) for k, v in worst]}
    print(json.dumps(row), flush=True)

# aggregates over the grid: geometric mean of every (case, tensor) error, and of each case's worst
# tensor; ratios to the host path (the VERDICT r4 bar: res6 within 1.2x of host)
gm = lambda v: float(np.exp(np.mean(np.log(np.maximum(v, 1e-30)))))
summ = {}
for lab, rows in allerr.items():
    every = [e for r in rows for e in r.values()]
    summ[lab] = {"geomean_all": gm(every), "geomean_worst": gm([max(r.values()) for r in rows]),
                 "max": max(every)}
for lab in summ:
    summ[lab]["ratio_to_host_all"] = summ[lab]["geomean_all"] / summ["host"]["geomean_all"]
    summ[lab]["ratio_to_host_worst"] = summ[lab]["geomean_worst"] / summ["host"]["geomean_worst"]
print(json.dumps({"summary": summ}), flush=True)
