"""The small ETT forecaster of tests/test_gpu_ett.py (KANFET [8, 16, 8], dopri5 rtol 1e-3) through
fieldn (default) or the per-stage path (FETODE_FIELDN=0): error against the fp64 oracle, the fp32
oracle's spread, attempts of each."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import ett  # noqa: E402
from oracle import torch_ref as O  # noqa: E402
from test_gpu_ett import _field_sd  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(11)
m = ett.LatentNeuralODEForecaster(num_features=7, context_len=16, pred_len=6, latent_dim=8, enc_hidden=32,
                                  dec_hidden=32, dyn_hidden=16, solver="dopri5", rtol=1e-3, atol=1e-4)
sd = {k: v.clone() for k, v in m.state_dict().items()}
m = m.to(dev)
g = torch.Generator().manual_seed(13)
x = torch.randn(12, 16, 7, generator=g)
t = torch.linspace(0.0, 1.0, steps=6)
from fet_ode_amd import dopri5 as D5
_orig_f = D5._Dopri5.f
calls = []


def _f(self, t_, y_):
    out = _orig_f(self, t_, y_)
    if len(calls) < 3:
        calls.append((t_, y_.detach().double().cpu().clone(), out.detach().double().cpu().clone()))
    return out


D5._Dopri5.f = _f
with torch.no_grad():
    got = m(x.to(dev), t.to(dev)).double().cpu()
D5._Dopri5.f = _orig_f
s = F.dopri5.dopri5_solve.last
res = {"fieldn": os.environ.get("FETODE_FIELDN", "1"), "nfev": s.nfev,
       "att": [(round(a[1], 6), a[3]) for a in s.attempts][:12]}
for dt in (torch.float32, torch.float64):
    sdd = {k: v.to(dt) for k, v in sd.items()}
    field = O.KANFETRef.from_state_dict(_field_sd(sdd), 2)
    h = torch.relu(torch.nn.functional.linear(x.to(dt).flatten(1), sdd["encoder.1.weight"], sdd["encoder.1.bias"]))
    z0 = torch.nn.functional.linear(h, sdd["encoder.3.weight"], sdd["encoder.3.bias"])
    tr = O.Dopri5Trace()
    zt = O.odeint(lambda tt, zz: field(zz), z0, t.to(dt), method="dopri5", rtol=1e-3, atol=1e-4, trace=tr)
    d = torch.relu(torch.nn.functional.linear(zt, sdd["decoder.0.weight"], sdd["decoder.0.bias"]))
    o = torch.nn.functional.linear(d, sdd["decoder.2.weight"], sdd["decoder.2.bias"]).squeeze(-1).T.double()
    res[str(dt)] = {"nfev": tr.nfev, "att": [(round(a[1], 6), a[3]) for a in tr.attempts][:12], "out": o}
e64 = res["torch.float64"]["out"]
res["err_gpu"] = (got - e64).abs().max().item()
res["spread32"] = (res["torch.float32"]["out"] - e64).abs().max().item()
for k in ("torch.float32", "torch.float64"):
    del res[k]["out"]
res["first_calls"] = [(c[0], c[1].abs().max().item(), c[2].norm().item()) for c in calls]
print(json.dumps(res), flush=True)
# the same first two calls through the fp64 oracle field (fresh state)
sdd0 = {k: v.double() for k, v in sd.items()}
rf = O.KANFETRef.from_state_dict(_field_sd(sdd0), 2)
outs = []
for c in calls[:2]:
    outs.append(rf(c[1].view(12, 8)))
print(json.dumps({"call_rel": [((c[2].view(12, 8) - o).norm() / o.norm()).item() for c, o in zip(calls[:2], outs)],
                  "diff_rel": (((calls[1][2] - calls[0][2]).view(12, 8) - (outs[1] - outs[0])).norm()
                               / (outs[1] - outs[0]).norm()).item(),
                  "h0_step": ((calls[1][1] - calls[0][1]).norm() / calls[0][2].norm()).item()}), flush=True)

# single evaluations of the field at z0 (fresh state) and at the probe z0 + h f0
net = m.dynamics.net
sdd = {k: v.double() for k, v in sd.items()}
h = torch.relu(torch.nn.functional.linear(x.double().flatten(1), sdd["encoder.1.weight"], sdd["encoder.1.bias"]))
z0 = torch.nn.functional.linear(h, sdd["encoder.3.weight"], sdd["encoder.3.bias"])
ref = O.KANFETRef.from_state_dict(_field_sd(sdd), 2)
f0r = ref(z0)
step = 1e-3
f1r = ref(z0 + step * f0r)
import copy
net2 = copy.deepcopy(net)
for l in net2.layers:
    l.ferro.reset_state() if hasattr(l.ferro, "reset_state") else None
fresh = ett.LatentNeuralODEForecaster(num_features=7, context_len=16, pred_len=6, latent_dim=8, enc_hidden=32,
                                      dec_hidden=32, dyn_hidden=16, solver="dopri5").to(dev)
fresh.load_state_dict(sd)
with torch.no_grad():
    f0g = fresh.dynamics.net(z0.float().to(dev)).double().cpu()
    f1g = fresh.dynamics.net((z0 + step * f0r).float().to(dev)).double().cpu()
rel = lambda a, b: ((a - b).norm() / b.norm()).item()
print(json.dumps({"fieldn": os.environ.get("FETODE_FIELDN", "1"), "f0_rel": rel(f0g, f0r), "f1_rel": rel(f1g, f1r),
                  "diff_rel": rel(f1g - f0g, f1r - f0r), "z0_absmax": z0.abs().max().item()}), flush=True)
