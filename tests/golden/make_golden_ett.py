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
         "LatentNeuralODEForecaster", "LogisticBasis", "LogisticBasisLinear", "FullyNonlinearKANCell",
         "KANRNNEncoder")
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
    assert a.shape == b.shape and torch.equal(a.isnan(), b.isnan()), what
    a, b = a.nan_to_num(0.0, 7.0, -7.0), b.nan_to_num(0.0, 7.0, -7.0)   # NaN where the other is NaN
    assert torch.equal(a, b), (what, (a.double() - b.double()).abs().max().item())


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


def _grads(module, inputs, out, seed):
    """d sum(out * w) / d (every parameter, every input) through the reference's autograd."""
    w = torch.randn(out.shape, generator=torch.Generator().manual_seed(seed))
    (out * w).sum().backward()
    g = {"w": w.numpy()}
    for k, p in module.named_parameters():
        g["grad/" + k] = (p.grad if p.grad is not None else torch.zeros_like(p)).numpy().copy()
    for k, v in inputs.items():
        g["grad_in/" + k] = v.grad.numpy().copy()
    return g


def kanrnn_case(R, F_, H, latent, nb, B, Ts, seed, edit=None, x_edit=None):
    """KANRNNEncoder(F_, H, latent, nb) (train_kan_fet_ett.py:798-818) straight after
    torch.manual_seed(seed) (pins the init RNG order), then forward + gradients for each T in Ts."""
    torch.manual_seed(seed)
    enc = R["KANRNNEncoder"](num_features=F_, hidden_size=H, latent_dim=latent, num_basis=nb)
    out = sd_np(enc, "init/")
    if edit is not None:
        with torch.no_grad():
            edit(enc)
    out.update(sd_np(enc))
    for T in Ts:
        x = torch.randn(B, T, F_, generator=torch.Generator().manual_seed(seed + T))
        if x_edit is not None:
            x_edit(x)
        xr = x.clone().requires_grad_(True)
        enc.zero_grad(set_to_none=True)
        z0 = enc(xr)
        with torch.no_grad():
            ref = E.KANRNNEncoderRef({k: v.detach() for k, v in enc.state_dict().items()})
            same(z0.detach(), ref(x), f"kanrnn T={T}")
        out[f"T{T}/x"] = x.numpy()
        out[f"T{T}/z0"] = z0.detach().numpy()
        out[f"T{T}/h"] = ref.hidden(x).numpy()
        out.update({f"T{T}/" + k: v for k, v in _grads(enc, {"x": xr}, z0, seed + 100 + T).items()})
    out["dims"] = np.array([F_, H, latent, nb], np.int32)
    out["Ts"] = np.array(Ts, np.int32)
    return out


def kanrnn_prod(R):
    """The ETT encoder at its production size (num_features 7, hidden 64, latent 64, 10 bases;
    KAN_FET_LatentODE_DiffusionForecaster defaults, :822-837), context 96 and a short context."""
    return kanrnn_case(R, 7, 64, 64, 10, B=12, Ts=(96, 3), seed=71)


def kanrnn_deep(R):
    """num_features * num_basis < hidden_size: the truncated cat keeps hidden-basis columns, so h_t
    really depends on h_{t-1} (chains up to 14 steps deep at 2 x 1 -> 16); NaN inputs early in the
    context (outside every chain reaching h_T) and late (inside one)."""
    def x_edit(x):
        x[0, 1, 0] = float("nan")
        x[1, -2, 1] = float("nan")
        x[2, -1, 0] = float("inf")
    return kanrnn_case(R, 2, 16, 5, 1, B=6, Ts=(20, 5), seed=72, x_edit=x_edit)


def kanrnn_overflow(R):
    """exp(-a (v - b)) overflowing in columns the truncation drops: the forward is unaffected, but
    the reference's autograd multiplies the dropped columns' zero gradient by inf (exp backward),
    so the parameters of those bases, the inputs they read and what those inputs feed get NaN."""
    def edit(enc):
        enc.rnn_cell.hidden_basis.a[3, 2] = 500.0
        enc.rnn_cell.hidden_basis.b[3, 2] = 2.0
        enc.rnn_cell.input_basis.a[6, 9] = 300.0
        enc.rnn_cell.input_basis.b[6, 9] = 5.0
    return kanrnn_case(R, 7, 16, 8, 10, B=4, Ts=(6,), seed=73, edit=edit)


def kancell_case(R):
    """FullyNonlinearKANCell (:780-795) alone: one step from a given h_prev, with gradients to
    x_t, h_prev and the four basis parameters; and LogisticBasisLinear (:753-776)."""
    torch.manual_seed(74)
    cell = R["FullyNonlinearKANCell"](3, 8, 2)
    g = torch.Generator().manual_seed(75)
    x = torch.randn(5, 3, generator=g).requires_grad_(True)
    h = torch.rand(5, 8, generator=g).requires_grad_(True)
    out = sd_np(cell, "cell/")
    y = cell(x, h)
    same(y.detach(), E.kan_cell(x.detach(), h.detach(), *(p.detach() for p in (
        cell.input_basis.a, cell.input_basis.b, cell.hidden_basis.a, cell.hidden_basis.b))), "cell")
    out.update({"cell_x": x.detach().numpy(), "cell_h": h.detach().numpy(), "cell_y": y.detach().numpy()})
    out.update({"cell_" + k: v for k, v in _grads(cell, {"x": x, "h": h}, y, 76).items()})
    torch.manual_seed(77)
    lin = R["LogisticBasisLinear"](5, 4, 3)
    with torch.no_grad():
        lin.bias.copy_(torch.randn(4, generator=g))
    xl = torch.randn(6, 5, generator=g).requires_grad_(True)
    yl = lin(xl)
    same(yl.detach(), E.logistic_basis_linear(xl.detach(), lin.basis.a.detach(), lin.basis.b.detach(),
                                              lin.weight.detach(), lin.bias.detach()), "LogisticBasisLinear")
    out.update(sd_np(lin, "lin/"))
    out.update({"lin_x": xl.detach().numpy(), "lin_y": yl.detach().numpy()})
    out.update({"lin_" + k: v for k, v in _grads(lin, {"x": xl}, yl, 78).items()})
    return out


def main():
    R = reference_defs()
    for name, fn in (("ett_rk4", rk4_case), ("ett_windows", windows_case), ("ett_forecaster", forecaster_case),
                     ("ett_kanrnn_prod", kanrnn_prod), ("ett_kanrnn_deep", kanrnn_deep),
                     ("ett_kanrnn_overflow", kanrnn_overflow), ("ett_kancell", kancell_case)):
        if len(sys.argv) > 1 and name not in sys.argv[1:]:
            continue
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **fn(R))
        print("wrote", name)


if __name__ == "__main__":
    main()
