"""CPU: the MNIST Kuramoto + KANLinear oracle (oracle/mnist_ref.py) reproduces the reference's
classes bit for bit (fixtures made from the reference classes by tests/golden/make_golden_mnist.py)."""
import torch

from conftest import golden_sd, load_golden


def _one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    return n


def test_head_bitwise():
    from oracle import mnist_ref as M
    n = _one_thread()
    g = load_golden("mnist_head")
    sd = {k: v.clone().requires_grad_(k != "grid") for k, v in golden_sd(g).items()}
    p = M.MnistKANParams.from_state_dict(sd)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    y = M.kanlinear_forward(x, p)
    assert torch.equal(y.detach(), torch.from_numpy(g["y"]))
    (y * torch.from_numpy(g["w"])).sum().backward()
    assert torch.equal(x.grad, torch.from_numpy(g["grad/x"]))
    for k in ("base_weight", "spline_weight", "spline_scaler", "logistic_weight", "logistic_bias"):
        assert torch.equal(sd[k].grad, torch.from_numpy(g["grad/" + k])), k
    assert torch.equal(sd["logistic_basis.a"].grad, torch.from_numpy(g["grad/logistic_basis.a"]))
    torch.set_num_threads(n)


def test_kuramoto_bitwise():
    from oracle import mnist_ref as M
    n = _one_thread()
    g = load_golden("mnist_kuramoto")
    sd = golden_sd(g)
    K = sd["K"].clone().requires_grad_(True)
    om = sd["omega"].clone().requires_grad_(True)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    y = M.kuramoto_forward(x, K, om, 10, 0.15)
    assert torch.equal(y.detach(), torch.from_numpy(g["y"]))
    (y * torch.from_numpy(g["w"])).sum().backward()
    assert torch.equal(x.grad, torch.from_numpy(g["grad/x"]))
    assert torch.equal(K.grad, torch.from_numpy(g["grad/K"]))
    assert torch.equal(om.grad, torch.from_numpy(g["grad/omega"]))
    torch.set_num_threads(n)


def test_classifier_bitwise():
    from oracle import mnist_ref as M
    n = _one_thread()
    g = load_golden("mnist_classifier")
    ref = M.ClassifierRef(golden_sd(g))
    assert torch.equal(ref(torch.from_numpy(g["x"])), torch.from_numpy(g["logits"]))
    torch.set_num_threads(n)
