"""Generate tests/golden/ecg_*.npz from the REFERENCE's ECG KAN-FET NODE classes.

Run in the survey/build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden_ecg.py

train_ecg_kan_fet_nn_ode.py cannot be imported whole (it imports torchdiffeq, absent from the
image — SURVEY F5), so this script reads the file as text, takes the four class definitions the
hot path uses out of it with `ast` (LogisticBasis :54-133, KANFeatureMixer :408-421,
No_MLP_KANODEFunc :483-509, KanFet_NODE :512-572) and executes exactly those definitions with
torch / nn in scope.  KanFet_NODE.forward calls `odeint`; there the oracle's restated torchdiffeq
(oracle/torch_ref.py, parity-unpinned w.r.t. a torchdiffeq binary) is supplied, as for the
other trajectory fixtures.  Every fixture is cross-checked bit for bit against oracle/ecg_ref.py
before it is written, so that restatement is pinned to the reference classes.
"""
import ast
import os
import sys

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FETODE_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)

from oracle import ecg_ref as E  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

torch.set_num_threads(1)
CLASSES = ("LogisticBasis", "KANFeatureMixer", "No_MLP_KANODEFunc", "KanFet_NODE")


def reference_classes():
    src = open(os.path.join(REF, "train_ecg_kan_fet_nn_ode.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in CLASSES]
    assert [n.name for n in body] == list(CLASSES), [n.name for n in body]
    ns = {"torch": torch, "nn": nn, "F": F, "odeint": O.odeint}
    exec(compile(ast.Module(body=body, type_ignores=[]), "train_ecg_kan_fet_nn_ode.py", "exec"), ns)
    return ns


def sd_np(module, prefix="sd/"):
    return {prefix + k: v.detach().numpy().copy() for k, v in module.state_dict().items()}


def same(a, b, what):
    a, b = a.detach(), b.detach()
    assert a.shape == b.shape and torch.equal(a, b), (what, (a - b).abs().max().item())


def hlogistic_case(R):
    torch.manual_seed(3)
    m = R["LogisticBasis"](64, 10)
    out = sd_np(m)
    p = E.HLogisticParams.from_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    g = torch.Generator().manual_seed(4)
    xs = [torch.randn(8, 64, generator=g) * 1.5, torch.randn(8, 64, generator=g) * 1.5,
          torch.randn(5, 64, generator=g) * 1.5]
    x4 = torch.randn(6, 64, generator=g) * 1.5
    x4[2] = xs[2][-1]          # a row equal to the stored last row: dx = 0, g = 0.5 -> down branch
    xs.append(x4)
    for c, x in enumerate(xs):
        y = m(x)
        yo = E.hlogistic_forward(x, p)
        same(y, yo, f"hlogistic call {c}")
        same(m.prev_x, p.prev_x, f"prev_x {c}")
        same(m.branch_state, p.branch_state, f"branch_state {c}")
        out[f"x{c}"] = x.numpy()
        out[f"y{c}"] = y.detach().numpy()
        out[f"prev_x{c}"] = m.prev_x.numpy().copy()
        out[f"branch_state{c}"] = m.branch_state.numpy().copy()
    # gradients of a fixed loss on a fifth call
    x5 = (torch.randn(7, 64, generator=g) * 1.5).requires_grad_(True)
    w = torch.randn(7, 64, 10, generator=g)
    (m(x5) * w).sum().backward()
    out["x5"], out["w5"] = x5.detach().numpy(), w.numpy()
    out["grad/x"] = x5.grad.numpy()
    for n, prm in m.named_parameters():
        out["grad/" + n] = (prm.grad.numpy() if prm.grad is not None else np.full(prm.shape, np.nan, np.float32))
    return out


def field_case(R):
    torch.manual_seed(5)
    f = R["No_MLP_KANODEFunc"](latent_dim=64, num_basis=10, hidden=128)
    out = sd_np(f)
    ref = E.ECGFieldRef.from_state_dict({k: v.clone() for k, v in f.state_dict().items()})
    g = torch.Generator().manual_seed(6)
    h1 = torch.randn(8, 64, generator=g)
    h2 = (h1 + 0.05 * torch.randn(8, 64, generator=g)).requires_grad_(True)
    t = torch.tensor(0.0)
    y1 = f(t, h1)
    same(y1, ref(t, h1), "field call 1")
    y2 = f(t, h2)
    same(y2, ref(t, h2.detach()), "field call 2")
    w = torch.randn(8, 64, generator=g)
    (y2 * w).sum().backward()
    out.update({"h1": h1.numpy(), "h2": h2.detach().numpy(), "y1": y1.detach().numpy(),
                "y2": y2.detach().numpy(), "w": w.numpy(), "grad/h": h2.grad.numpy()})
    for n, prm in f.named_parameters():
        out["grad/" + n] = (prm.grad.numpy() if prm.grad is not None else np.full(prm.shape, np.nan, np.float32))
    return out


def node_case(R, latent, nb, rtol, atol, B, seed):
    torch.manual_seed(seed)
    m = R["KanFet_NODE"](T=96, num_classes=2, latent_dim=latent, num_basis=nb, ode_hidden=128, dropout=0.1,
                         solver="dopri5", rtol=rtol, atol=atol)
    m.eval()
    out = sd_np(m)
    ref = E.ECGNodeRef({k: v.clone() for k, v in m.state_dict().items()}, rtol=rtol, atol=atol)
    x = E.ecg_x(B, seed=seed)
    with torch.no_grad():
        logits = m(x)
        lo = ref(x)
    same(logits, lo, f"node latent={latent}")
    tr = ref.trace
    out.update({"x": x.numpy(), "logits": logits.numpy(), "nfev": np.array(tr.nfev),
                "attempts": np.array([[a[0], a[1], a[2], float(a[3])] for a in tr.attempts]),
                "prev_x_odefunc": m.odefunc.feat.basis.prev_x.numpy().copy(),
                "rtol": np.array(rtol), "atol": np.array(atol)})
    return out


def main():
    R = reference_classes()
    cases = {
        "ecg_hlogistic": hlogistic_case(R),
        "ecg_field": field_case(R),
        # KanFet_NODE defaults (latent 64, nb 10, rtol 1e-3 atol 1e-4) and the __main__ config
        # (latent 1, nb 12, rtol 1e-2 atol 1e-3, :1181-1198)
        "ecg_node64": node_case(R, 64, 10, 1e-3, 1e-4, 16, 7),
        "ecg_node1": node_case(R, 1, 12, 1e-2, 1e-3, 16, 8),
    }
    for name, d in cases.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print(name, sorted(d)[:6], "...", len(d), "arrays")


if __name__ == "__main__":
    main()
