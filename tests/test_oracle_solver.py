"""Known-answer tests for the restated torchdiffeq solver (nothing in the reference pins it;
SURVEY §7.1 step 2).  These pin oracle/torch_ref.odeint, which in turn pins the HIP path."""
import math

import numpy as np
import pytest
import torch

from oracle import torch_ref as O


@pytest.mark.parametrize("method,order", [("euler", 1), ("midpoint", 2), ("rk4", 4)])
def test_linear_growth_factor_is_taylor_polynomial(method, order):
    lam, h = -0.7, 0.1
    z = lam * h
    y = O.odeint(lambda t, y: lam * y, torch.ones(1, dtype=torch.float64),
                 torch.tensor([0.0, h], dtype=torch.float64), method=method)
    expect = sum(z ** k / math.factorial(k) for k in range(order + 1))
    assert abs(y[1].item() - expect) < 1e-15


def test_rk4_3_8_exact_for_cubic_in_t():
    f = lambda t, y: 3 * t ** 2 - 2 * t + 1 + 0 * y
    t = torch.linspace(0, 2, 5, dtype=torch.float64)
    sol = O.odeint(f, torch.zeros(1, dtype=torch.float64), t, method="rk4")
    exact = t ** 3 - t ** 2 + t
    assert torch.allclose(sol[:, 0], exact, atol=1e-13)


def test_classic_rk4_matches_3_8_on_linear():
    lam = 0.3
    t = torch.linspace(0, 1, 11, dtype=torch.float64)
    a = O.odeint(lambda t, y: lam * y, torch.ones(1, dtype=torch.float64), t, method="rk4")
    b = O.odeint(lambda t, y: lam * y, torch.ones(1, dtype=torch.float64), t, method="rk4",
                 classic_rk4=True)
    assert torch.allclose(a, b, atol=1e-14)


def test_lv_rk4_and_dopri5_vs_lsoda():
    """Lotka-Volterra (train_kanfet_node_predprey.py:31-52) vs the scipy LSODA truth."""
    from conftest import load_golden
    g = load_golden("lv_lsoda")
    t, soln = torch.from_numpy(g["t"]), torch.from_numpy(g["soln"])
    al, be, ga, de = 1.5, 1.0, 3.0, 1.0

    def lv(t, X):
        x, y = X[..., 0], X[..., 1]
        return torch.stack([al * x - be * x * y, de * x * y - ga * y], -1)

    y0 = torch.tensor([1.0, 1.0], dtype=torch.float64)
    rk = O.odeint(lv, y0, t, method="rk4")                      # one step per output (h~0.1)
    rk_fine = O.odeint(lv, y0, t, method="rk4", options={"step_size": 0.01})  # + linear interp
    dp = O.odeint(lv, y0, t, method="dopri5", rtol=1e-10, atol=1e-12)
    # measured: dopri5 vs LSODA 1.4e-5; rk4 at h~0.1 2.9e-3 (O(h^4) global error);
    # step_size 0.01 + torchdiffeq's linear interpolation between grid points 6e-4 (O(h^2))
    assert (dp - soln).abs().max() < 5e-5
    assert (rk - dp).abs().max() < 5e-3
    assert (rk_fine - dp).abs().max() < 1e-3


def test_fixed_grid_interpolation_and_reversal():
    f = lambda t, y: -2.0 * y
    y0 = torch.ones(3, dtype=torch.float64)
    t = torch.tensor([0.0, 0.05, 0.1, 0.25], dtype=torch.float64)
    sol = O.odeint(f, y0, t, method="rk4", options={"step_size": 0.1})
    on_grid = torch.tensor([0, 2, 3])
    assert torch.allclose(sol[on_grid, 0], torch.exp(-2 * t[on_grid]), atol=1e-5)
    # off-grid output: torchdiffeq's linear interpolation between the bracketing grid points
    assert torch.allclose(sol[1], 0.5 * (sol[0] + sol[2]), atol=1e-15)
    back = O.odeint(f, sol[-1], t.flip(0), method="rk4")
    assert torch.allclose(back[-1], y0, atol=1e-5)


def test_dopri5_interp_is_quartic_hermite():
    """interp._interp_fit: p(0)=y0, p(1)=y1, p(1/2)=y_mid, p'(0)=dt f0, p'(1)=dt f1."""
    g = torch.Generator().manual_seed(0)
    y0, y1, ym, f0, f1 = (torch.randn(4, generator=g, dtype=torch.float64) for _ in range(5))
    dt = torch.tensor(0.3, dtype=torch.float64)
    c = O._interp_fit(y0, y1, ym, f0, f1, dt)
    ev = lambda x: O._interp_evaluate(c, torch.tensor(0.0, dtype=torch.float64),
                                      torch.tensor(1.0, dtype=torch.float64), torch.tensor(x, dtype=torch.float64))
    assert torch.allclose(ev(0.0), y0) and torch.allclose(ev(1.0), y1) and torch.allclose(ev(0.5), ym)
    e = c
    d1 = e[1] + 2 * e[2] + 3 * e[3] + 4 * e[4]
    assert torch.allclose(e[1], dt * f0) and torch.allclose(d1, dt * f1)


def test_dopri5_call_order_and_counts():
    calls = []
    f = lambda t, y: (calls.append(float(t)), -y)[1]
    tr = O.Dopri5Trace()
    O.odeint(f, torch.ones(2), torch.tensor([0.0, 1.0]), method="dopri5", rtol=1e-4, atol=1e-6, trace=tr)
    assert tr.nfev == len(calls) == 2 + 6 * len(tr.attempts)
    assert calls[0] == 0.0


def test_input_errors():
    with pytest.raises(TypeError):
        O.odeint(lambda t, y: y, torch.ones(2, dtype=torch.int64), torch.tensor([0.0, 1.0]))
    with pytest.raises(ValueError):
        O.odeint(lambda t, y: y, torch.ones(2), torch.tensor([0.0, 1.0]), method="nope")
    with pytest.raises(AssertionError):
        O.odeint(lambda t, y: y, torch.ones(2), torch.tensor([0.0, 1.0, 0.5]))


def test_classic_rk4_is_option_of_fixed_grid():
    """method='rk4_classic' (fet_ode_amd extension) reproduces odeint_rk4 of
    train_kan_fet_ett.py:51-83 with n_substeps=1."""
    f = lambda t, y: torch.sin(y) - 0.3 * y
    y0 = torch.tensor([0.4, -1.2], dtype=torch.float64)
    t = torch.linspace(0, 2, 9, dtype=torch.float64)
    a = O.odeint(f, y0, t, method="rk4", classic_rk4=True)
    z = y0
    out = [z]
    for i in range(len(t) - 1):
        h = t[i + 1] - t[i]
        k1 = f(t[i], z)
        k2 = f(t[i] + 0.5 * h, z + 0.5 * h * k1)
        k3 = f(t[i] + 0.5 * h, z + 0.5 * h * k2)
        k4 = f(t[i] + h, z + h * k3)
        z = z + (h / 6.0) * (k1 + 2 * k2 + 2 * k3 + k4)
        out.append(z)
    assert torch.allclose(a, torch.stack(out), atol=1e-14)


def test_dopri5_replay_reproduces_solve_and_row_subsets():
    """options['replay'] (test infrastructure for row-subset checks of large device solves): replaying
    a solve's own attempt log gives the same solution bit for bit, and replaying the FULL batch's log
    on a row subset gives those rows of the full solution (rows are independent given the steps)."""
    W = torch.tensor([[0.3, -1.1], [0.9, 0.2]], dtype=torch.float64)
    f = lambda t, y: torch.tanh(y @ W) - 0.1 * y
    y0 = torch.linspace(-1.5, 2.0, 16, dtype=torch.float64).reshape(8, 2)
    t = torch.tensor([0.0, 0.7, 2.0], dtype=torch.float64)
    tr = O.Dopri5Trace()
    sol = O.odeint(f, y0, t, rtol=1e-6, atol=1e-8, options={"first_step": 0.05}, trace=tr)
    log = [(a[0], a[1], a[3]) for a in tr.attempts]
    assert len(log) > 5
    again = O.odeint(f, y0, t, rtol=1e-6, atol=1e-8, options={"first_step": 0.05, "replay": log})
    assert torch.equal(again, sol)
    sub = O.odeint(f, y0[2:5], t, rtol=1e-6, atol=1e-8, options={"first_step": 0.05, "replay": log})
    assert torch.equal(sub, sol[:, 2:5])
    with pytest.raises(AssertionError):
        O.odeint(f, y0, t, options={"replay": log})      # the probe is a global norm: needs first_step
