"""Generate tests/golden/lv_head_step.npz: one captured training epoch of the reference's
KANFET-with-head LV script (train_kanfet_mlp_node_predprey.py:206-275).

Run in the survey/build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden_lv.py

The script's head classes (ResidualBottleneckMLPHead :192-203, KANFET_ODE_WithHead :206-220) are
taken out of the file text with `ast` (the script itself trains for 10 000 epochs on import); the
KANFET core is the SURVEY §8a A9 composition of the reference's own efficientkan.KANLinear and
ferro_class.FerroelectricBasis (make_golden.RefKANFET); torchdiffeq is absent, so the
solve is the restated 3/8-rule rk4 of oracle/torch_ref.py, as in every other trajectory fixture.
Stored: the initial state_dict, the loss, every parameter gradient and the parameters after one
torch.optim.Adam(lr=2e-3) step.
"""
import ast
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FETODE_REFERENCE", "/root/reference")
sys.path.insert(0, HERE)

import make_golden as MG  # noqa: E402  (reference efficientkan / ferro_class on sys.path)

from oracle import torch_ref as O  # noqa: E402

torch.set_num_threads(1)
CLASSES = ("ResidualBottleneckMLPHead", "KANFET_ODE_WithHead")


def reference_classes():
    src = open(os.path.join(REF, "train_kanfet_mlp_node_predprey.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in CLASSES]
    assert [n.name for n in body] == list(CLASSES), [n.name for n in body]
    ns = {"torch": torch, "nn": nn}
    exec(compile(ast.Module(body=body, type_ignores=[]), "train_kanfet_mlp_node_predprey.py", "exec"), ns)
    return ns


def main():
    R = reference_classes()
    torch.manual_seed(71)
    core = MG.RefKANFET([2, 10, 2])
    model = R["KANFET_ODE_WithHead"](core, state_dim=2, head_bottleneck=32, head_dropout=0.0)
    sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    t, soln = O.lotka_volterra_truth()
    X0 = torch.unsqueeze(torch.Tensor(np.transpose(np.array([1.0, 1.0]))), 0)
    X0.requires_grad = True
    t_learn = torch.tensor(np.linspace(0, 3.5, 35), dtype=torch.float32)
    soln_train = torch.tensor(soln, dtype=torch.float32)[:35]
    opt = torch.optim.Adam(model.parameters(), lr=2e-3)
    opt.zero_grad()
    pred = O.odeint(model.rhs, X0, t_learn, method="rk4")
    pred = model.head(pred)
    loss = torch.mean((pred[:, 0, :] - soln_train) ** 2)
    loss.backward()
    out = {"sd/" + k: v.numpy() for k, v in sd0.items()}
    for n, p in model.named_parameters():
        out["grad/" + n] = p.grad.numpy().copy()
    opt.step()
    for n, p in model.named_parameters():
        out["after/" + n] = p.detach().numpy().copy()
    out.update({"loss": np.float32(loss.item()), "pred": pred.detach().numpy()})
    np.savez_compressed(os.path.join(HERE, "lv_head_step.npz"), **out)
    print("wrote lv_head_step", loss.item())


if __name__ == "__main__":
    main()
