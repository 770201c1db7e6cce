"""Generate tests/golden/ett_*.npz from the REFERENCE's ETT forecasting code.

Run in the survey/build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden_ett.py

train_kan_fet_ett.py cannot be imported whole (it imports pandas-era plotting, torchdiffeq and the
KAN-RNN stack), so this script reads the file as text, takes the definitions the ETT path uses out
of it with `ast` (standardize_fit :34-37, standardize_apply :40-41, odeint_rk4 :51-83,
EnergyWindowDataset :107-131, ODEDynamics :136-152, LatentNeuralODEForecaster :155-197) and
executes exactly those with numpy / torch / nn / Dataset in scope.  LatentNeuralODEForecaster.forward
calls torchdiffeq's `odeint` (absent); the namespace binds that name to the reference's
own odeint_rk4 (the alternative written next to it at :192), so the forecaster fixture pins the
encoder / decoder / odeint_rk4 composition with reference code only.  Every fixture is
cross-checked bit for bit against oracle/ett_ref.py before it is written.
"""
import ast
import os
import sys

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import Dataset

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FETODE_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import ett_ref as E  # noqa: E402

torch.set_num_threads(1)
NAMES = ("standardize_fit", "standardize_apply", "odeint_rk4", "EnergyWindowDataset", "ODEDynamics",
         "LatentNeuralODEForecaster")
SUBSTEPS = 3


def reference_defs():
    src = open(os.path.join(REF, "train_kan_fet_ett.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in NAMES]
    assert sorted(n.name for n in body) == sorted(NAMES), [n.name for n in body]
    ns = {"np": np, "torch": torch, "nn": nn, "Dataset": Dataset}
    exec(compile(ast.Module(body=body, type_ignores=[]), "train_kan_fet_ett.py", "exec"), ns)
    ns["odeint"] = lambda f, z0, t, method=None: ns["odeint_rk4"](f, z0, t, n_substeps=SUBSTEPS)
    return ns


def sd_np(module, prefix="sd/"):
    return {prefix + k: v.detach().numpy().copy() for k, v in module.state_dict().items()}


def same(a, b, what):
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    assert a.shape == b.shape and torch.equal(a, b), (what, (a.double() - b.double()).abs().max().item())


def rk4_case(R):
    torch.manual_seed(61)
    dyn = R["ODEDynamics"](latent_dim=4, hidden=16)
    g = torch.Generator().manual_seed(62)
    z0 = torch.randn(5, 4, generator=g)
    t = torch.linspace(0.0, 7.0, steps=8)
    with torch.no_grad():
        traj = R["odeint_rk4"](dyn, z0, t, n_substeps=4)
        same(traj, E.odeint_rk4(E.ode_dynamics(dyn.state_dict(), ""), z0, t, n_substeps=4), "odeint_rk4")
    out = sd_np(dyn)
    out.update({"z0": z0.numpy(), "t": t.numpy(), "traj": traj.numpy(), "n_substeps": np.int32(4)})
    return out


def windows_case(R):
    rng = np.random.default_rng(63)
    raw = rng.normal(size=(48, 7)) * np.array([1, 2, 3, 4, 5, 6, 0.5]) + 10.0
    mu, sd = R["standardize_fit"](raw)
    mu2, sd2 = E.standardize_fit(raw)
    assert np.array_equal(mu, mu2) and np.array_equal(sd, sd2)
    X = R["standardize_apply"](raw, mu, sd)
    assert np.array_equal(X, E.standardize_apply(raw, mu2, sd2))
    y = X[:, -1]
    c, p = 8, 4
    ds = R["EnergyWindowDataset"](X, y, c, p)
    idx = [0, 5, 17, len(ds) - 1]
    xs = np.stack([ds[i][0].numpy() for i in idx])
    ys = np.stack([ds[i][1].numpy() for i in idx])
    xo, yo = E.windows(X, y, c, p, idx)
    assert np.array_equal(xs, xo) and np.array_equal(ys, yo)
    try:
        R["EnergyWindowDataset"](X[:11], y[:11], c, p)
        raise AssertionError("expected ValueError")
    except ValueError:
        pass
    return {"raw": raw, "mu": mu, "sd": sd, "X": X, "y": y, "idx": np.asarray(idx, np.int64),
            "x_ctx": xs, "y_fut": ys, "len": np.int64(len(ds)), "c": np.int32(c), "p": np.int32(p)}


def forecaster_case(R):
    torch.manual_seed(64)
    m = R["LatentNeuralODEForecaster"](num_features=7, context_len=8, pred_len=4, latent_dim=6, enc_hidden=16,
                                       dec_hidden=16, dyn_hidden=16)
    g = torch.Generator().manual_seed(65)
    x = torch.randn(5, 8, 7, generator=g)
    t = torch.linspace(0.0, 3.0, steps=4)
    with torch.no_grad():
        y = m(x, t)
        sd = m.state_dict()
        ref = E.ForecasterRef(sd, E.ode_dynamics(sd))
        same(y, ref(x, t, rk4_substeps=SUBSTEPS), "forecaster")
    out = sd_np(m)
    out.update({"x": x.numpy(), "t": t.numpy(), "y": y.numpy(), "n_substeps": np.int32(SUBSTEPS)})
    return out


def main():
    R = reference_defs()
    for name, fn in (("ett_rk4", rk4_case), ("ett_windows", windows_case), ("ett_forecaster", forecaster_case)):
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **fn(R))
        print("wrote", name)


if __name__ == "__main__":
    main()
