"""GPU parity of the MNIST Kuramoto + KANLinear classifier (mnist_kuramoto_kan.py; SURVEY §8f
rank 3) against fixtures made from the reference classes and the CPU oracle (oracle/mnist_ref.py)."""
import pytest
import torch

from conftest import golden_sd, load_golden

pytestmark = pytest.mark.gpu


def close(got, exp, rel, name):
    got, exp = got.detach().double().cpu(), exp.detach().double().cpu()
    scale = exp.abs().max().item() + 1e-12
    err = (got - exp).abs().max().item()
    assert err <= rel * scale, f"{name}: max|diff|={err:.3e} scale={scale:.3e}"


def test_head_forward_and_grads(dev):
    """KANLinear(288 -> 10, 8 logistic bases, logistic bias): inputs in and outside the grid incl.
    a knot and both grid ends; every parameter gradient against the reference's autograd."""
    from fet_ode_amd import mnist
    g = load_golden("mnist_head")
    m = mnist.KANLinear(288, 10, num_basis=8)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    y = m(x)
    close(y, torch.from_numpy(g["y"]), 1e-5, "y")
    (y * torch.from_numpy(g["w"]).to(dev)).sum().backward()
    close(x.grad, torch.from_numpy(g["grad/x"]), 1e-4, "grad x")
    for n, p in m.named_parameters():
        close(p.grad, torch.from_numpy(g["grad/" + n]), 2e-4, "grad " + n)


def test_kuramoto_forward_and_grads(dev):
    """Kuramoto2D(12 x 12, 10 steps, random omega, K = 0.7): features and d/dx, d/dK, d/domega."""
    from fet_ode_amd import mnist
    g = load_golden("mnist_kuramoto")
    m = mnist.Kuramoto2D(H=12, W=12, steps=10, dt=0.15)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    x = torch.from_numpy(g["x"]).to(dev).requires_grad_(True)
    y = m(x)
    close(y, torch.from_numpy(g["y"]), 1e-5, "features")
    (y * torch.from_numpy(g["w"]).to(dev)).sum().backward()
    close(x.grad, torch.from_numpy(g["grad/x"]), 1e-4, "grad x")
    close(m.K.grad, torch.from_numpy(g["grad/K"]), 1e-4, "grad K")
    close(m.omega.grad, torch.from_numpy(g["grad/omega"]), 1e-4, "grad omega")


def test_classifier_training_step(dev):
    """KuramotoKANClassifier: logits and the cross-entropy gradients of every parameter."""
    from fet_ode_amd import mnist
    g = load_golden("mnist_classifier")
    m = mnist.KuramotoKANClassifier(H=12, W=12, num_classes=10, kuramoto_steps=10, num_basis=8)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    logits = m(torch.from_numpy(g["x"]).to(dev))
    close(logits, torch.from_numpy(g["logits"]), 1e-5, "logits")
    torch.nn.functional.cross_entropy(logits, torch.from_numpy(g["labels"]).to(dev)).backward()
    for n, p in m.named_parameters():
        close(p.grad, torch.from_numpy(g["grad/" + n]), 2e-4, "grad " + n)


def test_production_size_vs_oracle(dev):
    """28 x 28 images, KANLinear(1568 -> 10): batch-64 logits and gradients against the CPU oracle
    (and its autograd) on the same seeded weights and synthetic images."""
    from fet_ode_amd import mnist
    from oracle import mnist_ref as M
    torch.manual_seed(61)
    m = mnist.KuramotoKANClassifier()
    with torch.no_grad():
        m.osc.omega.normal_(0, 0.3)
        m.head.logistic_bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    x = M.mnist_x(64, seed=62)
    y = torch.arange(64) % 10
    logits = m(x.to(dev))
    torch.nn.functional.cross_entropy(logits, y.to(dev)).backward()
    ps = {k: v.clone().requires_grad_(k not in ("osc.neighbor_kernel", "head.grid")) for k, v in sd.items()}
    ref = M.ClassifierRef(ps)
    lr = ref(x)
    close(logits, lr, 1e-5, "logits")
    torch.nn.functional.cross_entropy(lr, y).backward()
    for n, p in m.named_parameters():
        close(p.grad, ps[n].grad, 5e-4, "grad " + n)


def test_per_gpu_shard_b7500_rows_vs_oracle(dev):
    """BASELINE configs[4]: MNIST B = 60000 sharded 8x = 7 500 images per GPU
    (mnist_kuramoto_kan.py:207-283).  The whole 7 500-row batch runs on the device (every row tile
    of the Kuramoto lane kernels and of the KANLinear head, the ragged last tile included); logits
    and the parameter gradients of a loss over a 256-row subset (the first and last 64 rows and 128
    spread between) are checked against the CPU oracle on those rows, at the bars of the batch-64
    test above."""
    from fet_ode_amd import mnist
    from oracle import mnist_ref as M
    B = 7500
    torch.manual_seed(63)
    m = mnist.KuramotoKANClassifier()
    with torch.no_grad():
        m.osc.omega.normal_(0, 0.3)
        m.head.logistic_bias.normal_(0, 0.1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    x = M.mnist_x(B, seed=64)
    y = torch.arange(B) % 10
    g = torch.Generator().manual_seed(65)
    mid = torch.randperm(B - 128, generator=g)[:128] + 64
    rows = torch.cat([torch.arange(64), mid.sort().values, torch.arange(B - 64, B)])
    logits = m(x.to(dev))
    assert logits.shape == (B, 10) and torch.isfinite(logits).all()
    rd = rows.to(dev)
    torch.nn.functional.cross_entropy(logits[rd], y[rows].to(dev)).backward()
    ps = {k: v.clone().requires_grad_(k not in ("osc.neighbor_kernel", "head.grid")) for k, v in sd.items()}
    ref = M.ClassifierRef(ps)
    lr = ref(x[rows])
    close(logits[rd], lr, 1e-5, "logits B=7500 rows")
    torch.nn.functional.cross_entropy(lr, y[rows]).backward()
    for n, p in m.named_parameters():
        close(p.grad, ps[n].grad, 5e-4, "grad " + n + " (B=7500, 256-row loss)")


@pytest.mark.parametrize("W", [28, 31, 32])
def test_kuramoto_lane_kernels_match_lds_kernels(dev, W):
    """The 28 x 28 production shape runs the lane-per-column Kuramoto kernels (registers + DPP wave
    shifts, no LDS); the workgroup-per-image LDS kernels (fetode_kuramoto_set_lds(1)) are the other
    implementation of the same per-pixel arithmetic and tap order: features, the tape, d/dx and
    d/domega bitwise equal, d/dK (a per-image sum in another order) to 1e-6.  An odd batch leaves
    the last wave's second image empty.  W = 31 is the widest lane shape (lane 31 of each image
    stays empty); W = 32 would put the two images of a wave next to each other across the DPP
    shifts, so it takes the LDS kernels — checked here by images that do not couple: every image
    of the batch equals the same image integrated alone."""
    from fet_ode_amd import _lib, mnist
    lib = _lib.load()
    torch.manual_seed(5)
    m = mnist.Kuramoto2D(H=28, W=W, steps=10, dt=0.15)
    with torch.no_grad():
        m.omega.normal_(0, 0.3)
        m.K.fill_(0.8)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    x = torch.rand(37, 1, 28, W, generator=torch.Generator().manual_seed(6))
    w = torch.randn(37, 2 * 28 * W, generator=torch.Generator().manual_seed(7))
    out = []
    prev = lib.fetode_kuramoto_set_lds(-1)
    try:
        for lds in (0, 1):
            lib.fetode_kuramoto_set_lds(lds)
            mm = mnist.Kuramoto2D(H=28, W=W, steps=10, dt=0.15)
            mm.load_state_dict(sd)
            mm = mm.to(dev)
            xg = x.to(dev).requires_grad_(True)
            y = mm(xg)
            (y.reshape(37, -1) * w.to(dev)).sum().backward()
            out.append((y.detach().cpu(), xg.grad.cpu(), mm.omega.grad.cpu(), mm.K.grad.cpu()))
        lib.fetode_kuramoto_set_lds(0)
        mm = mnist.Kuramoto2D(H=28, W=W, steps=10, dt=0.15)
        mm.load_state_dict(sd)
        mm = mm.to(dev)
        with torch.no_grad():
            alone = torch.cat([mm(x[i:i + 1].to(dev)).cpu() for i in range(4)])
    finally:
        lib.fetode_kuramoto_set_lds(prev)
    (y0, gx0, go0, gk0), (y1, gx1, go1, gk1) = out
    assert torch.equal(y0, y1)
    assert torch.equal(gx0, gx1) and torch.equal(go0, go1)
    # d/dK is one fp32 sum over every pixel and step of an image, in another order on each path;
    # at 28 x 28 it agrees to 1e-6, the wider test shapes sum 10 % more terms with more cancellation
    close(gk0, gk1, 1e-6 if W == 28 else 1e-5, "grad K")
    assert torch.equal(alone, y0[:4]), "images of one wave must not couple"
