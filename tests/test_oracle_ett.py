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
