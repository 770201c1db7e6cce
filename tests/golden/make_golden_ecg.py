"""Generate tests/golden/ecg_*.npz from the REFERENCE's ECG KAN-FET NODE classes (and the
FerroElectricNet field of train_ecg.py).

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


FERRONET_CLASSES = ("KANFetODEFunc", "KanFet_MLP_NODE")


def ferronet_classes():
    """train_ecg.py:986-1059 (KANFetODEFunc, KanFet_MLP_NODE) the same way; their
    FerroelectricBasis is the reference's own ferro_class module (importable here)."""
    sys.path.insert(0, REF)
    import ferro_class  # noqa: E402  (the reference module)
    src = open(os.path.join(REF, "train_ecg.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in FERRONET_CLASSES]
    assert [n.name for n in body] == list(FERRONET_CLASSES), [n.name for n in body]
    ns = {"torch": torch, "nn": nn, "F": F, "odeint": O.odeint, "FerroelectricBasis": ferro_class.FerroelectricBasis}
    exec(compile(ast.Module(body=body, type_ignores=[]), "train_ecg.py", "exec"), ns)
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


def ferronet_field_case(R):
    out = {}
    g = torch.Generator().manual_seed(21)
    t = torch.tensor(0.0)
    # batch calls (the B > 1 first-call rule dx = 0), then a carried-state call with gradients
    torch.manual_seed(11)
    f = R["KANFetODEFunc"](latent_dim=8, hidden_dim=16, num_basis=12)
    out.update(sd_np(f, "sd_a/"))
    ref = E.FerroNetFieldRef.from_state_dict({k: v.clone() for k, v in f.state_dict().items()})
    h1 = torch.randn(4, 8, generator=g) * 1.5
    h2 = (h1 + 0.1 * torch.randn(4, 8, generator=g)).requires_grad_(True)
    y1 = f(t, h1)
    same(y1, ref(t, h1), "ferronet call 1")
    y2 = f(t, h2)
    same(y2, ref(t, h2.detach()), "ferronet call 2")
    w = torch.randn(4, 8, generator=g)
    (y2 * w).sum().backward()
    out.update({"a/h1": h1.numpy(), "a/h2": h2.detach().numpy(), "a/y1": y1.detach().numpy(),
                "a/y2": y2.detach().numpy(), "a/w": w.numpy(), "a/grad/h": h2.grad.numpy()})
    for n, prm in f.named_parameters():
        out["a/grad/" + n] = prm.grad.numpy()
    # batch-1 calls (fresh buffers keep their (1, in, out, K) zeros: dx = x), incl. a 1-D h
    torch.manual_seed(12)
    f = R["KANFetODEFunc"](latent_dim=8, hidden_dim=16, num_basis=12)
    out.update(sd_np(f, "sd_b/"))
    ref = E.FerroNetFieldRef.from_state_dict({k: v.clone() for k, v in f.state_dict().items()})
    for c in range(3):
        h = torch.randn(8, generator=g) * 1.5 if c == 1 else torch.randn(1, 8, generator=g) * 1.5
        y = f(t, h)
        same(y, ref(t, h), f"ferronet b1 call {c}")
        out[f"b/h{c}"], out[f"b/y{c}"] = h.numpy(), y.detach().numpy()
    # saturating field: coef x 8 drives fc2 past the +-50 clamp; gradients stop there
    torch.manual_seed(13)
    f = R["KANFetODEFunc"](latent_dim=8, hidden_dim=16, num_basis=12)
    with torch.no_grad():
        f.fc2.coef.mul_(8.0)
    out.update(sd_np(f, "sd_c/"))
    ref = E.FerroNetFieldRef.from_state_dict({k: v.clone() for k, v in f.state_dict().items()})
    h = (torch.randn(5, 8, generator=g) * 2).requires_grad_(True)
    y = f(t, h)
    same(y, ref(t, h.detach()), "ferronet saturating call")
    assert bool((y.abs() == 50).any()), "clamp not exercised"
    w = torch.randn(5, 8, generator=g)
    (y * w).sum().backward()
    out.update({"c/h": h.detach().numpy(), "c/y": y.detach().numpy(), "c/w": w.numpy(), "c/grad/h": h.grad.numpy()})
    for n, prm in f.named_parameters():
        out["c/grad/" + n] = prm.grad.numpy()
    return out


def ferronet_node_case(R, solver, B, seed, rtol=1e-3, atol=1e-4):
    torch.manual_seed(seed)
    m = R["KanFet_MLP_NODE"](T=96, num_classes=2, latent_dim=8, num_basis=12, ode_hidden=16, dropout=0.1,
                             solver=solver, rtol=rtol, atol=atol)
    m.eval()
    out = sd_np(m)
    ref = E.FerroNetNodeRef({k: v.clone() for k, v in m.state_dict().items()}, solver=solver, rtol=rtol, atol=atol)
    x = E.ecg_x(B, seed=seed)
    with torch.no_grad():
        logits = m(x)
        lo = ref(x)
    same(logits, lo, f"ferronet node {solver}")
    out.update({"x": x.numpy(), "logits": logits.numpy(), "rtol": np.array(rtol), "atol": np.array(atol),
                "fc1_prev_x": m.odefunc.fc1.prev_x.numpy().copy(), "fc2_prev_x": m.odefunc.fc2.prev_x.numpy().copy()})
    return out


def main():
    R = reference_classes()
    RF = ferronet_classes()
    cases = {
        "ecg_hlogistic": hlogistic_case(R),
        "ecg_field": field_case(R),
        # KanFet_NODE defaults (latent 64, nb 10, rtol 1e-3 atol 1e-4) and the __main__ config
        # (latent 1, nb 12, rtol 1e-2 atol 1e-3, :1181-1198)
        "ecg_node64": node_case(R, 64, 10, 1e-3, 1e-4, 16, 7),
        "ecg_node1": node_case(R, 1, 12, 1e-2, 1e-3, 16, 8),
        # the FerroElectricNet field (train_ecg.py:986-1013) and its NODE (:1017-1059): __main__
        # runs it with euler (:1365); dopri5 is the class default
        "ecg_ferronet_field": ferronet_field_case(RF),
        "ecg_ferronet_euler": ferronet_node_case(RF, "euler", 3, 31),
        "ecg_ferronet_dopri5": ferronet_node_case(RF, "dopri5", 2, 32),
    }
    for name, d in cases.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print(name, sorted(d)[:6], "...", len(d), "arrays")


if __name__ == "__main__":
    main()
