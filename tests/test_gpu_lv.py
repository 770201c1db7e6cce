"""MI355X: the LV training harness (fet_ode_amd.lv; train_kanfet_node_predprey.py and
train_kanfet_mlp_node_predprey.py) — one epoch (fused rk4 solve + head + MSE + fused reverse
sweep + Adam) against the oracle."""
import numpy as np
import pytest
import torch
import torch.nn.functional as Fn

import fet_ode_amd as F
from conftest import golden_sd, load_golden
from fet_ode_amd import lv
from oracle import torch_ref as O
from test_oracle_lv import head_ref, oracle_step

pytestmark = pytest.mark.gpu


def test_kan_head_epoch_matches_oracle(dev):
    """Well-conditioned core (KAN, no hysteresis): loss 1e-5, gradients 1e-4, Adam step 1e-6."""
    torch.manual_seed(3)
    m = lv.KANFET_ODE_WithHead(F.KAN([2, 10, 2], grid_size=5), state_dim=2)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    prob = lv.lv_problem(dev, t_learn_dtype=torch.float32)
    opt = torch.optim.Adam(m.parameters(), lr=2e-3)
    loss = lv.train_epoch(m, prob, opt, method="rk4")
    names = [n for n, _ in m.named_parameters()]
    ps = {k: v.clone().requires_grad_(k in names) for k, v in sd.items()}
    ref = O.KANRef([O.KANLinearParams.from_state_dict(ps, f"kanfet.layers.{l}.") for l in range(2)])
    t, soln = O.lotka_volterra_truth()
    pred = head_ref(ps, O.odeint(lambda tt, yy: ref(yy), torch.tensor([[1.0, 1.0]]),
                                 torch.tensor(np.linspace(0, 3.5, 35), dtype=torch.float32), method="rk4"))
    l_ref = torch.mean((pred[:, 0, :] - torch.tensor(soln, dtype=torch.float32)[:35]) ** 2)
    gr = dict(zip(names, torch.autograd.grad(l_ref, [ps[n] for n in names])))
    assert abs(loss.item() - l_ref.item()) <= 1e-5 * abs(l_ref.item())
    ref_opt = torch.optim.Adam([ps[n] for n in names], lr=2e-3)
    for n in names:
        ps[n].grad = gr[n]
    ref_opt.step()
    for n, p in m.named_parameters():
        g = p.grad.cpu()
        assert ((g - gr[n]).norm() / gr[n].norm().clamp_min(1e-30)).item() <= 1e-4, n
        assert (p.detach().cpu() - ps[n].detach()).abs().max().item() <= 1e-6 + 1e-3 * 2e-3, n
    assert torch.isfinite(lv.test_loss(m, prob, method="rk4"))


def test_kanfet_head_epoch_vs_reference_fixture(dev):
    """The reference fixture (KAN-FET core, B = 1, 35 points): fp32 KAN-FET is ill-conditioned here
    (the reference's fp32 and fp64 losses are 20.2 and 23.5), so the GPU loss must lie within 4x the
    reference's own fp32-vs-fp64 distance of the fp64 oracle, and every gradient be finite."""
    g = load_golden("lv_head_step")
    sd = golden_sd(g)
    torch.manual_seed(0)
    m = lv.KANFET_ODE_WithHead(F.KANFET([2, 10, 2], grid_size=5), state_dim=2)
    m.load_state_dict(sd)
    m = m.to(dev)
    prob = lv.lv_problem(dev, t_learn_dtype=torch.float32)
    opt = torch.optim.Adam(m.parameters(), lr=2e-3)
    loss = lv.train_epoch(m, prob, opt, method="rk4").item()   # the fixture's method
    l64, _ = oracle_step(sd, torch.float64)
    spread = abs(float(g["loss"]) - l64.item())
    assert abs(loss - l64.item()) <= 4 * spread + 1e-5 * abs(l64.item()), (loss, float(g["loss"]), l64.item())
    for n, p in m.named_parameters():
        assert torch.isfinite(p.grad).all() and torch.isfinite(p).all(), n


def test_default_method_is_dopri5_like_the_reference(dev):
    """train_kanfet_node_predprey.py:252 calls torchodeint without a method: dopri5 at rtol 1e-7 /
    atol 1e-9.  One default epoch of the KAN-core harness against the oracle's dopri5 autograd.
    At rtol 1e-7 the error ratios sit at fp32 rounding level, so the two step sequences may differ
    in a few attempts: the loss must agree to 1e-4 and the gradients to 1e-2 (both solves are
    accurate to ~1e-6), and the solve must have taken the adaptive path."""
    torch.manual_seed(3)
    m = lv.KANFET_ODE_WithHead(F.KAN([2, 10, 2], grid_size=5), state_dim=2)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    prob = lv.lv_problem(dev, t_learn_dtype=torch.float32)
    opt = torch.optim.SGD(m.parameters(), lr=0.0)
    loss = lv.train_epoch(m, prob, opt)
    s = F.dopri5.dopri5_solve.last
    assert s.nfev > 6 * 5 and len(s.attempts) > 5
    names = [n for n, _ in m.named_parameters()]
    ps = {k: v.clone().requires_grad_(k in names) for k, v in sd.items()}
    ref = O.KANRef([O.KANLinearParams.from_state_dict(ps, f"kanfet.layers.{l}.") for l in range(2)])
    t, soln = O.lotka_volterra_truth()
    pred = head_ref(ps, O.odeint(lambda tt, yy: ref(yy), torch.tensor([[1.0, 1.0]]),
                                 torch.tensor(np.linspace(0, 3.5, 35), dtype=torch.float32)))
    l_ref = torch.mean((pred[:, 0, :] - torch.tensor(soln, dtype=torch.float32)[:35]) ** 2)
    gr = dict(zip(names, torch.autograd.grad(l_ref, [ps[n] for n in names])))
    assert abs(loss.item() - l_ref.item()) <= 1e-4 * abs(l_ref.item()), (loss.item(), l_ref.item())
    for n, p in m.named_parameters():
        g = p.grad.cpu()
        assert ((g - gr[n]).norm() / gr[n].norm().clamp_min(1e-30)).item() <= 1e-2, n
