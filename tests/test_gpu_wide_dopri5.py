"""MI355X: the device-resident dopri5 of the wide KAN-FET field (fetode_wide_dopri5) — the ETT
forecaster's own solve, odeint(self.dynamics, z0, t_fut, method="dopri5") (train_kan_fet_ett.py:192,
:858, :879) with KANFET([64, 128, 64]) — against the host-driven loop (dopri5.py _Dopri5: two
fetode_wide_layer_forward launches per evaluation, fetode_lincomb / fetode_scaled_rms /
fetode_interp_*, one read-back per attempt), which the ETT tests pin to the fp64 oracle.

The resident solver uses the host loop's arithmetic (each layer's input slices as the per-layer
launch picks them, the same stage sums, the fp64 step control); only the error norms' fp64
summation order differs.  So: the same attempt count, accept pattern and nfev, step sizes equal to
fp64 rounding, the solution and the hysteresis memory after the solve equal up to that."""
import numpy as np
import pytest
import torch

import fet_ode_amd as F
from fet_ode_amd import ett
from fet_ode_amd.autograd_ops import field_layers
from fet_ode_amd.dopri5 import ResidentSolve, _Dopri5

pytestmark = pytest.mark.gpu


def _dyn(dev, seed=0, K=10, latent=64, hidden=128):
    torch.manual_seed(seed)
    return ett.KANFETDynamics(latent, hidden=hidden, num_fet_basis=K).to(dev)


def _z0(B, dev, D=64, seed=3, scale=0.6):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(B, D, generator=g) * scale).to(dev)


def _solve(dyn, z0, t, resident, **kw):
    prev = F.dopri5.set_wide_resident_dopri5(resident, gap=(0, 0))   # resident at every batch
    try:
        with torch.no_grad():
            sol = F.odeint(dyn, z0, t, method="dopri5", **kw)
        s = F.dopri5.dopri5_solve.last
        if resident:
            assert isinstance(s, ResidentSolve), "the wide resident path was not taken"
        else:
            assert isinstance(s, _Dopri5)
        state = [f._prev.clone() for _, f in field_layers(dyn.net)]
        return sol, s.nfev, s.attempts, state
    finally:
        F.dopri5.set_wide_resident_dopri5(prev, gap=(512, 8192))


def _compare(host, res, what):
    (sh, nh, ah, st_h), (sr, nr, ar, st_r) = host, res
    assert nr == nh, f"{what}: nfev {nr} vs host {nh}"
    assert len(ar) == len(ah), f"{what}: {len(ar)} attempts vs host {len(ah)}"
    assert [a[3] for a in ar] == [a[3] for a in ah], f"{what}: accept pattern differs"
    for (t0r, dtr, rr, _), (t0h, dth, rh, _) in zip(ar, ah):
        assert abs(dtr - dth) <= 1e-12 * abs(dth) and abs(t0r - t0h) <= 1e-12 * max(1.0, abs(t0h)), what
        assert abs(rr - rh) <= 1e-6 * max(abs(rh), 1e-30), f"{what}: error ratio {rr} vs {rh}"
    assert torch.isfinite(sr).all()
    scale = sh.abs().max().item() + 1e-30
    err = (sr - sh).abs().max().item()
    assert err <= 1e-6 * scale, f"{what}: |resident - host| = {err:.3e} (scale {scale:.3e})"
    for a, b in zip(st_r, st_h):
        assert a.shape == b.shape
        assert (a - b).abs().max().item() <= 1e-6 * (b.abs().max().item() + 1e-30), f"{what}: hysteresis memory"
    return err / scale


# B = 100 / 256: both layers input-sliced (S0 = S1 = 2) and a partial row tile; 8192: the ETT bench
# batch (layer 0 whole, layer 1 sliced); 16384: both whole
@pytest.mark.parametrize("B", [1, 100, 256, 8192, 16384])
def test_wide_resident_dopri5_matches_host_loop(dev, B):
    dyn = _dyn(dev)
    sd = {k: v.clone() for k, v in dyn.state_dict().items()}
    z0 = _z0(B, dev)
    t = torch.linspace(0.0, 3.0, steps=4, device=dev)
    kw = dict(rtol=1e-3, atol=1e-4)
    # a fresh module (first call: prev = x, ferro_class.py:372-375), then a second solve that starts
    # from the memory the first one left
    host1 = _solve(dyn, z0, t, False, **kw)
    host2 = _solve(dyn, z0 * 0.9, t, False, **kw)
    dyn = _dyn(dev)
    dyn.load_state_dict(sd)
    res1 = _solve(dyn, z0, t, True, **kw)
    res2 = _solve(dyn, z0 * 0.9, t, True, **kw)
    _compare(host1, res1, f"B={B} first solve")
    _compare(host2, res2, f"B={B} carried state")
    assert len(res1[2]) >= 3


def test_wide_resident_dopri5_reference_defaults_and_first_step(dev):
    """torchdiffeq's default tolerances (rtol 1e-7, atol 1e-9: hundreds of attempts on a short
    horizon) and an explicit first_step / max_step, K = 12, a non-ETT width pair (32 -> 64 -> 32)."""
    dyn = _dyn(dev, seed=5, K=12, latent=32, hidden=64)
    sd = {k: v.clone() for k, v in dyn.state_dict().items()}
    z0 = _z0(64, dev, D=32, seed=9, scale=0.4)
    t = torch.tensor([0.0, 0.05, 0.1], device=dev)
    host = _solve(dyn, z0, t, False)
    dyn2 = _dyn(dev, seed=5, K=12, latent=32, hidden=64)
    dyn2.load_state_dict(sd)
    res = _solve(dyn2, z0, t, True)
    _compare(host, res, "defaults")
    assert len(res[2]) > 20
    opts = dict(rtol=1e-4, atol=1e-6, options=dict(first_step=0.01, max_step=0.02))
    t2 = torch.linspace(0.0, 0.2, steps=3, device=dev)
    host = _solve(dyn, z0, t2, False, **opts)
    res = _solve(dyn2, z0, t2, True, **opts)
    _compare(host, res, "first_step / max_step")
    assert all(a[1] <= 0.02 for a in res[2])


@pytest.mark.parametrize("first_step", [None, 0.05])
def test_wide_resident_dopri5_nonfinite_state_raises(dev, first_step):
    """A NaN start raises torchdiffeq's assertion exactly like the host loop: with the initial-step
    probe the NaN norm makes dt NaN ("underflow in dt"), with first_step the attempt's finiteness
    check fires ("non-finite values in state")."""
    z0 = _z0(64, dev)
    z0[5, 3] = float("nan")
    t = torch.linspace(0.0, 1.0, steps=3, device=dev)
    kw = dict(rtol=1e-3, atol=1e-4)
    if first_step is not None:
        kw["options"] = dict(first_step=first_step)
    msgs = []
    for resident in (False, True):
        with pytest.raises(AssertionError) as ei:
            _solve(_dyn(dev), z0, t, resident, **kw)
        msgs.append(str(ei.value))
    key = "non-finite values in state" if first_step is not None else "underflow in dt"
    assert all(m.startswith(key) for m in msgs), msgs   # (the host loop appends the dt value)


def test_forecaster_dopri5_forward_takes_resident_path(dev):
    """The forecaster's forward (the reference's dopri5 call) goes through the resident solver and
    gives the host loop's prediction."""
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=8, latent_dim=64, solver="dopri5",
                                      rtol=1e-3, atol=1e-4).to(dev)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(512 + 96 + 8, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], 96, 8, device=dev)
    xb, _ = ds.batch(torch.arange(512, device=dev))
    t_fut = torch.linspace(0.0, 7.0, steps=8, device=dev)
    prev = F.dopri5.set_wide_resident_dopri5(False)
    try:
        with torch.no_grad():
            yh = m(xb, t_fut)
    finally:
        F.dopri5.set_wide_resident_dopri5(prev)
    m.load_state_dict(sd)
    m2 = ett.LatentNeuralODEForecaster(num_features=7, context_len=96, pred_len=8, latent_dim=64, solver="dopri5",
                                       rtol=1e-3, atol=1e-4).to(dev)
    m2.load_state_dict(sd)
    with torch.no_grad():
        yr = m2(xb, t_fut)
    assert isinstance(F.dopri5.dopri5_solve.last, ResidentSolve)
    assert yr.shape == yh.shape == (512, 8)
    assert (yr - yh).abs().max().item() <= 1e-5 * (yh.abs().max().item() + 1e-30)


def test_wide_resident_dispatch_crossover(dev):
    """Between the measured crossover batches (512, 8192) the per-layer launches are faster than
    the persistent grid: the default dispatch takes the host loop there and the
    resident solver on either side."""
    t = torch.linspace(0.0, 0.5, steps=3, device=dev)
    for B, resident in ((512, True), (1024, False)):
        dyn = _dyn(dev)
        with torch.no_grad():
            F.odeint(dyn, _z0(B, dev), t, method="dopri5", rtol=1e-3, atol=1e-4)
        assert isinstance(F.dopri5.dopri5_solve.last, ResidentSolve) == resident, B
