"""Generate tests/golden/mnist_*.npz from the REFERENCE's MNIST Kuramoto + KANLinear classes.

Run in the survey/build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden_mnist.py

mnist_kuramoto_kan.py cannot be imported whole (it imports torchvision, absent from the image), so
this script reads the file as text, takes the four class definitions out of it with `ast`
(LogisticBasis :11-22, KANLinear :25-142, Kuramoto2D :145-199, KuramotoKANClassifier :202-221)
and executes exactly those definitions with math / torch / nn / F in scope.  Every fixture is
cross-checked bit for bit against oracle/mnist_ref.py before it is written.  Image size 12 x 12
(in_dim 288) keeps the fixtures small; the kernels are size-generic and the 28 x 28 production
size is checked on the GPU against the oracle run there.
"""
import ast
import math
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

from oracle import mnist_ref as M  # noqa: E402

torch.set_num_threads(1)
CLASSES = ("LogisticBasis", "KANLinear", "Kuramoto2D", "KuramotoKANClassifier")


def reference_classes():
    src = open(os.path.join(REF, "mnist_kuramoto_kan.py")).read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in CLASSES]
    assert [n.name for n in body] == list(CLASSES), [n.name for n in body]
    ns = {"math": math, "torch": torch, "nn": nn, "F": F}
    exec(compile(ast.Module(body=body, type_ignores=[]), "mnist_kuramoto_kan.py", "exec"), ns)
    return ns


def sd_np(module, prefix="sd/"):
    return {prefix + k: v.detach().numpy().copy() for k, v in module.state_dict().items()}


def same(a, b, what):
    a, b = a.detach(), b.detach()
    assert a.shape == b.shape and torch.equal(a, b), (what, (a - b).abs().max().item())


def grads(module, out, prefix="grad/"):
    for n, p in module.named_parameters():
        out[prefix + n] = p.grad.numpy().copy() if p.grad is not None else np.full(p.shape, np.nan, np.float32)


def head_case(R):
    torch.manual_seed(51)
    m = R["KANLinear"](288, 10, grid_size=5, spline_order=3, use_logistic_basis=True, num_basis=8)
    with torch.no_grad():
        m.logistic_bias.normal_(0, 0.1)   # zero at init; make it visible in the fixture
    out = sd_np(m)
    p = M.MnistKANParams.from_state_dict({k: v.clone() for k, v in m.state_dict().items()})
    g = torch.Generator().manual_seed(52)
    x = (torch.rand(6, 288, generator=g) * 2.6 - 1.3)
    x[0, :4] = torch.tensor([-2.2, 2.2, 0.2, 3.0])    # a knot, the grid ends, outside
    x.requires_grad_(True)
    y = m(x)
    same(y, M.kanlinear_forward(x.detach(), p), "head forward")
    w = torch.randn(6, 10, generator=g)
    (y * w).sum().backward()
    out.update({"x": x.detach().numpy(), "y": y.detach().numpy(), "w": w.numpy(), "grad/x": x.grad.numpy()})
    grads(m, out)
    return out


def kuramoto_case(R):
    torch.manual_seed(53)
    m = R["Kuramoto2D"](H=12, W=12, steps=10, dt=0.15, learn_K=True, learn_omega=True)
    with torch.no_grad():
        m.omega.normal_(0, 0.5)
        m.K.fill_(0.7)
    out = sd_np(m)
    x = M.mnist_x(5, 12, 12, seed=54).requires_grad_(True)
    y = m(x)
    same(y, M.kuramoto_forward(x.detach(), m.K.detach(), m.omega.detach(), 10, 0.15), "kuramoto forward")
    g = torch.Generator().manual_seed(55)
    w = torch.randn(*y.shape, generator=g)
    (y * w).sum().backward()
    out.update({"x": x.detach().numpy(), "y": y.detach().numpy(), "w": w.numpy(), "grad/x": x.grad.numpy()})
    grads(m, out)
    return out


def classifier_case(R):
    torch.manual_seed(56)
    m = R["KuramotoKANClassifier"](H=12, W=12, num_classes=10, kuramoto_steps=10, num_basis=8)
    out = sd_np(m)
    ref = M.ClassifierRef({k: v.clone() for k, v in m.state_dict().items()})
    x = M.mnist_x(4, 12, 12, seed=57)
    y = torch.tensor([3, 1, 4, 1])
    logits = m(x)
    same(logits, ref(x), "classifier forward")
    F.cross_entropy(logits, y).backward()
    out.update({"x": x.numpy(), "labels": y.numpy(), "logits": logits.detach().numpy()})
    grads(m, out)
    return out


def main():
    R = reference_classes()
    cases = {"mnist_head": head_case(R), "mnist_kuramoto": kuramoto_case(R), "mnist_classifier": classifier_case(R)}
    for name, d in cases.items():
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
        print(name, len(d), "arrays")


if __name__ == "__main__":
    main()
