"""CPU: the ETT oracle (oracle/ett_ref.py) against the reference fixtures (tests/golden/ett_*.npz,
made from train_kan_fet_ett.py's own definitions), plus the host logic of fet_ode_amd.ett
(substep schedule, device-free window gathers, constructor / state_dict surface)."""
import numpy as np
import pytest
import torch

from conftest import golden_sd, load_golden
from oracle import ett_ref as E


def test_oracle_odeint_rk4_matches_reference_bitwise():
    g = load_golden("ett_rk4")
    sd = golden_sd(g)
    with torch.no_grad():
        traj = E.odeint_rk4(E.ode_dynamics(sd, ""), torch.from_numpy(g["z0"]), torch.from_numpy(g["t"]),
                            n_substeps=int(g["n_substeps"]))
    assert torch.equal(traj, torch.from_numpy(g["traj"]))


def test_oracle_windows_and_standardize_match_reference():
    g = load_golden("ett_windows")
    mu, sd = E.standardize_fit(g["raw"])
    assert np.array_equal(mu, g["mu"]) and np.array_equal(sd, g["sd"])
    X = E.standardize_apply(g["raw"], mu, sd)
    assert np.array_equal(X, g["X"])
    xs, ys = E.windows(g["X"], g["y"], int(g["c"]), int(g["p"]), g["idx"])
    assert np.array_equal(xs, g["x_ctx"]) and np.array_equal(ys, g["y_fut"])
    with pytest.raises(ValueError):
        E.windows(g["X"][:11], g["y"][:11], int(g["c"]), int(g["p"]), [0])


def test_oracle_forecaster_matches_reference_bitwise():
    g = load_golden("ett_forecaster")
    sd = golden_sd(g)
    with torch.no_grad():
        y = E.ForecasterRef(sd, E.ode_dynamics(sd))(torch.from_numpy(g["x"]), torch.from_numpy(g["t"]),
                                                    rk4_substeps=int(g["n_substeps"]))
    assert torch.equal(y, torch.from_numpy(g["y"]))


def test_substep_schedule_is_the_reference_grid():
    from fet_ode_amd.odeint import Schedule
    t = torch.linspace(0.0, 95.0, steps=96)
    s = Schedule.substeps(t, 4)
    assert s.n_steps == 95 * 4 and s.T == 96
    h = ((t[1:] - t[:-1]) / 4.0).numpy()
    assert np.array_equal(s.step_coef[:, 0], np.repeat(h, 4))
    assert np.array_equal(s.step_coef[:, 1], np.repeat((torch.from_numpy(h) * 0.5).numpy(), 4))
    assert np.array_equal(s.step_coef[:, 2], np.repeat((torch.from_numpy(h) / 6.0).numpy(), 4))
    assert list(s.out_step[1:4]) == [3, 7, 11] and (s.out_mode[1:] == 1).all()
    # stage times: ti accumulated with ti + h in t's dtype (train_kan_fet_ett.py:68-78)
    ti = t[0].clone()
    for k in range(4):
        ti = ti + torch.tensor(h[0])
        assert s.grid[k + 1] == ti.item()


def test_window_dataset_host_logic():
    from fet_ode_amd.ett import EnergyWindowDataset
    g = load_golden("ett_windows")
    c, p = int(g["c"]), int(g["p"])
    ds = EnergyWindowDataset(g["X"], g["y"], c, p)
    assert len(ds) == int(g["len"])
    for k, i in enumerate(g["idx"]):
        xc, yf = ds[int(i)]
        assert np.array_equal(xc.numpy(), g["x_ctx"][k]) and np.array_equal(yf.numpy(), g["y_fut"][k])
    xb, yb = ds.batch(torch.from_numpy(g["idx"]))
    assert np.array_equal(xb.numpy(), g["x_ctx"]) and np.array_equal(yb.numpy(), g["y_fut"])
    with pytest.raises(ValueError):
        EnergyWindowDataset(g["X"][:11], g["y"][:11], c, p)
    with pytest.raises(IndexError):
        ds[len(ds)]


def test_forecaster_surface_matches_reference_keys():
    from fet_ode_amd.ett import LatentNeuralODEForecaster
    g = load_golden("ett_forecaster")
    ref_keys = {k for k in golden_sd(g) if not k.startswith("dynamics.")}
    m = LatentNeuralODEForecaster(num_features=7, context_len=8, pred_len=4, latent_dim=6, enc_hidden=16,
                                  dec_hidden=16, dyn_hidden=16)
    sd = m.state_dict()
    assert ref_keys <= set(sd)
    for k in ref_keys:
        assert sd[k].shape == golden_sd(g)[k].shape
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 8, 7), torch.linspace(0, 3, 4))
    with pytest.raises(ValueError):
        LatentNeuralODEForecaster(7, 8, 4, solver="adams")


# ---------------------------------------------------------------------------------------------
# the KAN-RNN encoder (train_kan_fet_ett.py:741-818): oracle vs the reference's own classes, the
# init RNG order of the drop-ins, and the host-side cone depth of fetode_kanrnn_forward
# ---------------------------------------------------------------------------------------------

def _nan_equal(a, b):
    a, b = torch.as_tensor(a), torch.as_tensor(b)
    return a.shape == b.shape and torch.equal(a.isnan(), b.isnan()) and torch.equal(a.nan_to_num(0.0),
                                                                                     b.nan_to_num(0.0))


def _enc_grads(sd, x, w):
    ps = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    xr = x.clone().requires_grad_(True)
    z0 = E.KANRNNEncoderRef(ps)(xr)
    (z0 * w).sum().backward()
    return z0.detach(), {k: v.grad for k, v in ps.items()}, xr.grad


@pytest.mark.parametrize("name", ["ett_kanrnn_prod", "ett_kanrnn_deep", "ett_kanrnn_overflow"])
def test_oracle_kanrnn_encoder_matches_reference_bitwise(name):
    """Forward, every parameter gradient and d/dx (NaN patterns included) bit for bit."""
    g = load_golden(name)
    sd = golden_sd(g)
    for T in g["Ts"]:
        x = torch.from_numpy(g[f"T{T}/x"])
        z0, grads, gx = _enc_grads(sd, x, torch.from_numpy(g[f"T{T}/w"]))
        assert _nan_equal(z0, g[f"T{T}/z0"])
        for k, v in grads.items():
            assert _nan_equal(v, g[f"T{T}/grad/{k}"]), (T, k)
        assert _nan_equal(gx, g[f"T{T}/grad_in/x"])


def test_oracle_kancell_and_logistic_basis_linear_match_reference_bitwise():
    g = load_golden("ett_kancell")
    c = golden_sd(g, "cell/")
    ps = {k: v.clone().requires_grad_(True) for k, v in c.items()}
    x = torch.from_numpy(g["cell_x"]).requires_grad_(True)
    h = torch.from_numpy(g["cell_h"]).requires_grad_(True)
    y = E.kan_cell(x, h, ps["input_basis.a"], ps["input_basis.b"], ps["hidden_basis.a"], ps["hidden_basis.b"])
    assert torch.equal(y.detach(), torch.from_numpy(g["cell_y"]))
    (y * torch.from_numpy(g["cell_w"])).sum().backward()
    for k, v in ps.items():
        assert torch.equal(v.grad, torch.from_numpy(g[f"cell_grad/{k}"])), k
    assert torch.equal(x.grad, torch.from_numpy(g["cell_grad_in/x"]))
    assert torch.equal(h.grad, torch.from_numpy(g["cell_grad_in/h"]))
    lin = golden_sd(g, "lin/")
    yl = E.logistic_basis_linear(torch.from_numpy(g["lin_x"]), lin["basis.a"], lin["basis.b"], lin["weight"],
                                 lin["bias"])
    assert torch.equal(yl, torch.from_numpy(g["lin_y"]))


def test_kanrnn_dropins_init_rng_order_matches_reference():
    """The drop-ins consume the global RNG like the reference constructors (state_dict bitwise)."""
    from fet_ode_amd import ett
    g = load_golden("ett_kanrnn_prod")
    torch.manual_seed(71)
    enc = ett.KANRNNEncoder(num_features=7, hidden_size=64, latent_dim=64, num_basis=10)
    init = golden_sd(g, "init/")
    assert list(enc.state_dict()) == list(init)
    for k, v in enc.state_dict().items():
        assert torch.equal(v, init[k]), k
    gc = load_golden("ett_kancell")
    torch.manual_seed(74)
    cell = ett.FullyNonlinearKANCell(3, 8, 2)
    for k, v in cell.state_dict().items():
        assert torch.equal(v, torch.from_numpy(gc["cell/" + k])), k
    torch.manual_seed(77)
    lin = ett.LogisticBasisLinear(5, 4, 3)
    ref = golden_sd(gc, "lin/")
    assert set(lin.state_dict()) == set(ref)
    assert torch.equal(lin.basis.a, ref["basis.a"]) and torch.equal(lin.weight, ref["weight"])


def _depth_py(F_, H, nb):
    D = 0
    for j in range(H):
        d, c = 0, j
        while c >= F_ * nb:
            c = (c - F_ * nb) // nb
            d += 1
        D = max(D, d)
    return D


@pytest.mark.parametrize("F_,H,nb", [(7, 64, 10), (2, 16, 1), (7, 16, 10), (1, 64, 1), (3, 200, 2), (1, 256, 1)])
def test_kanrnn_cone_depth_host_logic(F_, H, nb):
    """fetode_kanrnn_depth (a host function: callable without a GPU) is the dependency depth, and
    the cone argument holds on the oracle: the last depth+1 steps from ANY h reproduce h_T of the
    whole recurrence bit for bit, NaN inputs outside the cone included."""
    from fet_ode_amd import _lib
    D = _lib.load().fetode_kanrnn_depth(F_, H, nb)
    assert D == _depth_py(F_, H, nb)
    gen = torch.Generator().manual_seed(F_ * 1000 + H + nb)
    p = [torch.randn(F_, nb, generator=gen), torch.randn(F_, nb, generator=gen), torch.randn(H, nb, generator=gen),
         torch.randn(H, nb, generator=gen)]
    T = D + 6
    x = torch.randn(5, T, F_, generator=gen)
    x[0, 0, 0] = float("nan")
    full = torch.zeros(5, H)
    for t in range(T):
        full = E.kan_cell(x[:, t], full, *p)
    cone = torch.full((5, H), float("nan"))           # anything, NaN included: no chain reads it
    for t in range(T - 1 - D, T):
        cone = E.kan_cell(x[:, t], cone, *p)
    assert _nan_equal(full, cone)
    if D > 0:   # one step fewer is NOT enough: the deepest chain reads the NaN start
        short = torch.full((5, H), float("nan"))
        for t in range(T - D, T):
            short = E.kan_cell(x[:, t], short, *p)
        assert not _nan_equal(full, short)
