"""GPU backward parity: HIP VJP kernels vs the reference's autograd (golden fixture) and vs
autograd through the CPU oracle (train_kanfet_node_predprey.py:254-257 loss.backward())."""
import numpy as np
import pytest
import torch

from conftest import golden_sd, load_golden

pytestmark = pytest.mark.gpu


def assert_grad_close(got, exp, name, rel=2e-4):
    got, exp = got.double().cpu(), exp.double().cpu()
    scale = exp.abs().max().item() + 1e-12
    err = (got - exp).abs().max().item()
    assert err <= rel * scale, f"{name}: max|diff|={err:.3e} scale={scale:.3e}"


def test_kanfet_field_grads_vs_reference_autograd(dev):
    """Two consecutive stateful calls, loss = mean(f1^2) + sum(f2 * [-1, 1]) — the fixture's
    gradients were produced by torch autograd through the reference modules."""
    import fet_ode_amd as F
    g = load_golden("kanfet_field")
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    x = torch.from_numpy(g["y0"]).to(dev).requires_grad_(True)
    f1 = m(x)
    f2 = m(x * 1.01 + 0.05)
    loss = f1.square().mean() + (f2 * torch.linspace(-1, 1, 2, device=dev)).sum()
    loss.backward()
    assert_grad_close(x.grad, torch.from_numpy(g["grad/x"]), "x")
    for n, p in m.named_parameters():
        assert_grad_close(p.grad, torch.from_numpy(g["grad/" + n]), n)


@pytest.mark.parametrize("tag,dims", [("kanlinear_2x10", (2, 10)), ("kanlinear_10x2", (10, 2))])
def test_kanlinear_grads_vs_oracle(dev, tag, dims):
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden(tag)
    sd = golden_sd(g)
    m = F.KANLinear(*dims)
    m.load_state_dict(sd)
    m = m.to(dev)
    x = torch.from_numpy(g["x"])
    w = torch.randn(x.shape[0], dims[1], generator=torch.Generator().manual_seed(1))
    xg = x.clone().to(dev).requires_grad_(True)
    (m(xg) * w.to(dev)).sum().backward()
    # oracle autograd on CPU
    ps = {k: v.clone().requires_grad_(v.dtype.is_floating_point and k != "grid") for k, v in sd.items()}
    p = O.KANLinearParams.from_state_dict(ps)
    xc = x.clone().requires_grad_(True)
    (O.kanlinear_forward(xc, p) * w).sum().backward()
    assert_grad_close(xg.grad, xc.grad, "x")
    names = {"base_weight": "base_weight", "spline_weight": "spline_weight", "spline_scaler": "spline_scaler",
             "logistic_basis.a": "logistic_basis.a", "logistic_basis.b": "logistic_basis.b",
             "logistic_weight": "logistic_weight", "logistic_scaler": "logistic_scaler"}
    mp = dict(m.named_parameters())
    for k, n in names.items():
        assert_grad_close(mp[n].grad, ps[k].grad, n)


@pytest.mark.parametrize("tag,dims", [("ferro_2x10x10", (2, 10, 10)), ("ferro_10x2x10", (10, 2, 10))])
def test_ferro_grads_vs_oracle(dev, tag, dims):
    """Second call of a B=5 sequence (dx != 0, prev from the first call)."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden(tag)
    sd = golden_sd(g, "sd2/")
    m = F.FerroelectricBasis(*dims)
    m.load_state_dict(sd, strict=False)
    m.reset_state()
    m = m.to(dev)
    xs = torch.from_numpy(g["xs5"])
    w = torch.randn(5, dims[1], generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        m(xs[0].to(dev))
    xg = xs[1].clone().to(dev).requires_grad_(True)
    (m(xg) * w.to(dev)).sum().backward()
    ps = {k: sd[k].clone().requires_grad_(True) for k in ("k", "Ec", "Ps", "bias", "coef")}
    p = O.FerroParams(*(ps[k] for k in ("k", "Ec", "Ps", "bias", "coef")))
    st = O.FerroState(*dims)
    with torch.no_grad():
        O.ferro_forward(xs[0], p, st)
    xc = xs[1].clone().requires_grad_(True)
    (O.ferro_forward(xc, p, st) * w).sum().backward()
    assert_grad_close(xg.grad, xc.grad, "x")
    for k in ("k", "Ec", "Ps", "bias", "coef"):
        assert_grad_close(getattr(m, k).grad, ps[k].grad, k)


def _loss_grads_gpu(model, y0, t, target, dev, use_autonomous):
    import fet_ode_amd as F
    y0g = y0.clone().to(dev).requires_grad_(True)
    func = F.autonomous(model) if use_autonomous else (lambda tt, yy: model(yy))
    pred = F.odeint(func, y0g, t, method="rk4")
    loss = torch.mean(torch.square(pred[:, 0, :] - target.to(dev)))
    loss.backward()
    return loss.item(), y0g.grad.cpu(), {n: p.grad.cpu() for n, p in model.named_parameters()}


@pytest.mark.parametrize("use_autonomous", [True, False])
def test_training_grads_through_rk4_kan(dev, use_autonomous):
    """predator_prey.py:135-168 training step shape: X0 (1,2) requires_grad, MSE on pred[:,0,:],
    backward through every stage.  KAN field, 35-point t_learn (float64)."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])
    y0 = torch.tensor([[1.0, 1.0]])
    target = torch.from_numpy(load_golden("lv_lsoda")["soln"][:35]).float()
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    loss, gy0, gps = _loss_grads_gpu(m, y0, t, target, dev, use_autonomous)
    ps = {k: v.clone().requires_grad_(k.split(".")[-1] != "grid") for k, v in sd.items()}
    ref = O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)])
    y0c = y0.clone().requires_grad_(True)
    pred = O.odeint(lambda tt, yy: ref(yy), y0c, t, method="rk4")
    lref = torch.mean(torch.square(pred[:, 0, :] - target))
    lref.backward()
    assert abs(loss - lref.item()) <= 1e-5 * abs(lref.item())
    assert_grad_close(gy0, y0c.grad, "y0", rel=1e-4)
    for n, gp in gps.items():
        assert_grad_close(gp, ps[n].grad, n, rel=1e-4)


def test_training_grads_through_rk4_kanfet_short(dev):
    """KAN-FET, B=16, 6 output points: short enough to be well conditioned in fp32."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])[:6]
    y0 = O.lv_y0(16, seed=5)
    target = torch.zeros(6, 2)
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    loss, gy0, gps = _loss_grads_gpu(m, y0, t, target, dev, True)
    ps = {k: v.clone().requires_grad_(k.split(".")[-1] not in ("grid", "prev_x", "branch_sign"))
          for k, v in sd.items()}
    ref = O.KANFETRef.from_state_dict(ps, 2)
    y0c = y0.clone().requires_grad_(True)
    pred = O.odeint(lambda tt, yy: ref(yy), y0c, t, method="rk4")
    lref = torch.mean(torch.square(pred[:, 0, :] - target))
    lref.backward()
    assert abs(loss - lref.item()) <= 1e-5 * abs(lref.item())
    assert_grad_close(gy0, y0c.grad, "y0", rel=1e-3)
    for n, gp in gps.items():
        assert_grad_close(gp, ps[n].grad, n, rel=1e-3)
