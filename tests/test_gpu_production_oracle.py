"""MI355X: the ETT production sizes pinned to the oracle on row subsets (VERDICT r3 "next" 2).

The other production-width tests compare the device paths with each other (resident dopri5 vs the
host loop, the fused wide layer vs the per-module kernels); these compare them with the CPU oracle
(oracle/torch_ref.py + oracle/ett_ref.py, the reference's op order) at the production batch itself,
B = 8192 and KANFET[64, 128, 64] — so every tiling, input-slicing and grid-barrier case the kernels
take at that size is on the checked path — on 256 rows: the first and last row tiles and 128 rows
spread over the batch.

* fetode_wide_dopri5 (train_kan_fet_ett.py:192, the forecaster's own solve): the error norm couples
  all 8192 rows, so the oracle replays the device solve's attempt log (step sizes and accept
  decisions; oracle.torch_ref `replay`) on the subset — the rows' arithmetic is then independent of
  the other rows — with an explicit first_step (the initial-step probe is a global norm too; the
  probe path itself is pinned against the host loop in test_gpu_wide_dopri5.py).
* LatentNeuralODEForecaster forward with the KAN-FET latent field (train_kan_fet_ett.py:155-197) on
  96 -> 8 windows, odeint_rk4: rows are independent, the oracle runs the subset directly.

Bar: the fp32/fp64 envelope of tests/test_gpu_ett.py — |gpu - fp64| <= 4 |reference fp32 - fp64|
+ 1e-5 x scale, elementwise max over the subset (KAN-FET is ill-conditioned in fp32).
Horizons are short so the untrained field stays bounded (|z| < 50)."""
import pytest
import torch

import fet_ode_amd as F
from fet_ode_amd import ett
from fet_ode_amd.autograd_ops import field_layers
from fet_ode_amd.dopri5 import ResidentSolve
from oracle import ett_ref as E
from oracle import torch_ref as O

pytestmark = pytest.mark.gpu

B = 8192


def _rows():
    g = torch.Generator().manual_seed(21)
    mid = torch.randperm(B - 128, generator=g)[:128] + 64
    return torch.cat([torch.arange(64), mid.sort().values, torch.arange(B - 64, B)])


def _envelope(got, e32, e64, name, floor=1e-5, k=4.0):
    got, e32, e64 = got.detach().double().cpu(), e32.detach().double().cpu(), e64.detach().double().cpu()
    scale = e64.abs().max().item() + 1e-12
    spread = (e32 - e64).abs().max().item()
    err = (got - e64).abs().max().item()
    assert err <= k * spread + floor * scale, f"{name}: |gpu-fp64|={err:.3e} fp32 spread={spread:.3e} scale={scale:.3e}"
    return err / scale, spread / scale


def test_wide_resident_dopri5_b8192_rows_vs_oracle(dev):
    torch.manual_seed(0)
    dyn = ett.KANFETDynamics(64, hidden=128, num_fet_basis=10)
    sd = {k: v.clone() for k, v in dyn.net.state_dict().items()}
    dyn = dyn.to(dev)
    g = torch.Generator().manual_seed(3)
    z0 = torch.randn(B, 64, generator=g) * 0.6
    t = torch.linspace(0.0, 0.1, steps=3)
    kw = dict(rtol=1e-1, atol=1e-2, options=dict(first_step=0.05))
    prev = F.dopri5.set_wide_resident_dopri5(True, gap=(0, 0))
    try:
        with torch.no_grad():
            sol = F.odeint(dyn, z0.to(dev), t.to(dev), method="dopri5", **kw)
        s = F.dopri5.dopri5_solve.last
        assert isinstance(s, ResidentSolve), "the wide resident path was not taken"
    finally:
        F.dopri5.set_wide_resident_dopri5(prev, gap=(512, 8192))
    log = [(a[0], a[1], a[3]) for a in s.attempts]
    assert len(log) >= 2 and torch.isfinite(sol).all()
    mem = [f._prev.detach().cpu() for _, f in field_layers(dyn.net)]
    rows = _rows()
    outs = {}
    for dt in (torch.float32, torch.float64):
        ref = O.KANFETRef.from_state_dict({k: v.to(dt) for k, v in sd.items()}, 2)
        tr = O.Dopri5Trace()
        with torch.no_grad():
            e = O.odeint(lambda tt, zz: ref(zz), z0[rows].to(dt), t.to(torch.float64), method="dopri5",
                         rtol=kw["rtol"], atol=kw["atol"], options={**kw["options"], "replay": log}, trace=tr)
        assert tr.nfev == s.nfev, (tr.nfev, s.nfev)
        outs[dt] = (e, [st.prev_x[:, :, 0, 0].clone() for st in ref.states])
    (e32, m32), (e64, m64) = outs[torch.float32], outs[torch.float64]
    got = sol.cpu()[:, rows]
    assert got.abs().max().item() < 50
    _envelope(got, e32, e64, "wide dopri5 B=8192 solution rows")
    for l in range(2):
        _envelope(mem[l][rows], m32[l], m64[l], f"wide dopri5 B=8192 hysteresis memory layer {l}")


def test_wide_resident_dopri5_oracle_chooses_its_own_steps(dev):
    """fetode_wide_dopri5 at KANFET[64, 128, 64] (train_kan_fet_ett.py:192) against the oracle's
    OWN step-size control: no replay, no first_step — the oracle selects the initial step
    (_select_initial_step) and accepts / rejects every attempt from its own fp32 error norms.  The
    batch is one the CPU oracle can carry inside a test (B = 64: ~0.2 s per oracle evaluation at
    these widths; B = 512 is ~2.4 s, ~4 min per solve); t in [0, 0.02] at rtol 1e-3 / atol 1e-4
    gives 15 attempts (4 rejected while the probe's step shrinks, 11 accepted) whose error ratios
    all stay >= 16 % away from 1, so the decisions are not at fp32 rounding level.  The device
    solve must take the same attempts (accept pattern, nfev, dt to 1e-5 relative: the norms are
    fp64 sums on the device and fp32 torch norms in the oracle); the solution and both layers'
    hysteresis memory are checked against the fp32/fp64 envelope (the fp64 oracle's own control
    takes the same decisions; a replay would need first_step and so skip the initial-step probe,
    itself a stateful hysteresis call)."""
    torch.manual_seed(0)
    dyn = ett.KANFETDynamics(64, hidden=128, num_fet_basis=10)
    sd = {k: v.clone() for k, v in dyn.net.state_dict().items()}
    dyn = dyn.to(dev)
    g = torch.Generator().manual_seed(3)
    z0 = torch.randn(64, 64, generator=g) * 0.6
    t = torch.linspace(0.0, 0.02, steps=3)
    kw = dict(rtol=1e-3, atol=1e-4)
    prev = F.dopri5.set_wide_resident_dopri5(True, gap=(0, 0))
    try:
        with torch.no_grad():
            sol = F.odeint(dyn, z0.to(dev), t.to(dev), method="dopri5", **kw)
        s = F.dopri5.dopri5_solve.last
        assert isinstance(s, ResidentSolve), "the wide resident path was not taken"
    finally:
        F.dopri5.set_wide_resident_dopri5(prev, gap=(512, 8192))
    mem = [f._prev.detach().cpu() for _, f in field_layers(dyn.net)]
    torch.set_num_threads(min(16, torch.get_num_threads()))
    ref32 = O.KANFETRef.from_state_dict(sd, 2)
    tr = O.Dopri5Trace()
    with torch.no_grad():
        e32 = O.odeint(lambda tt, zz: ref32(zz), z0, t.to(torch.float64), method="dopri5", trace=tr, **kw)
    m32 = [st.prev_x[:, :, 0, 0].clone() for st in ref32.states]
    ours = [(a[1], a[3]) for a in s.attempts]
    theirs = [(a[1], a[3]) for a in tr.attempts]
    assert len(theirs) >= 10 and not all(acc for _, acc in theirs), theirs
    assert [acc for _, acc in ours] == [acc for _, acc in theirs], (ours, theirs)
    assert s.nfev == tr.nfev, (s.nfev, tr.nfev)
    for (d0, _), (d1, _) in zip(ours, theirs):
        assert abs(d0 - d1) <= 1e-5 * abs(d1), (ours, theirs)
    assert min(abs(a[2] - 1.0) for a in tr.attempts) > 0.1   # decisions far from rounding level
    sd64 = {k: v.to(torch.float64) for k, v in sd.items()}
    ref64 = O.KANFETRef.from_state_dict(sd64, 2)
    tr64 = O.Dopri5Trace()
    with torch.no_grad():
        e64 = O.odeint(lambda tt, zz: ref64(zz), z0.double(), t.to(torch.float64), method="dopri5", trace=tr64, **kw)
    assert [a[3] for a in tr64.attempts] == [acc for _, acc in theirs]
    m64 = [st.prev_x[:, :, 0, 0].clone() for st in ref64.states]
    _envelope(sol.cpu(), e32, e64, "wide dopri5 B=64, oracle-chosen steps: solution")
    for l in range(2):
        _envelope(mem[l], m32[l], m64[l], f"wide dopri5 B=64, oracle-chosen steps: hysteresis memory layer {l}")


def test_forecaster_latent64_b8192_rows_vs_oracle(dev):
    c, p = 96, 8
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=c, pred_len=p, latent_dim=64, solver="rk4")
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(B + c + p, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], c, p, device=dev)
    xb, _ = ds.batch(torch.arange(B, device=dev))
    t_fut = torch.linspace(0.0, float(p - 1), steps=p)
    with torch.no_grad():
        got = m(xb, t_fut.to(dev), rk4_substeps=1)
    assert got.shape == (B, p) and torch.isfinite(got).all()
    rows = _rows()
    xs = xb[rows.to(dev)].cpu()
    outs = {}
    for dt in (torch.float32, torch.float64):
        sdd = {k: v.to(dt) for k, v in sd.items()}
        field = O.KANFETRef.from_state_dict({k[len("dynamics.net."):]: v for k, v in sdd.items()
                                             if k.startswith("dynamics.net.")}, 2)
        ref = E.ForecasterRef(sdd, lambda tt, zz: field(zz))
        with torch.no_grad():
            outs[dt] = ref(xs.to(dt), t_fut.to(dt), rk4_substeps=1)
    _envelope(got.cpu()[rows], outs[torch.float32], outs[torch.float64], "forecaster latent 64, B=8192 rows")


@pytest.mark.timeout(900)   # the CPU oracle: 5 x 380 steps of the [64, 128, 64] field on 8 rows
def test_forecaster_bench_workload_96_horizon_vs_oracle(dev):
    """BASELINE config 4 at its own horizon: the bench's ETT workload exactly —
    LatentNeuralODEForecaster 96 -> 96, latent 64, KAN-FET field [64, 128, 64] scaled x 0.1,
    odeint_rk4 with the reference TrainConfig's 4 substeps over t_fut = 0..95 (380 rk4 steps),
    B = 8192, first call on fresh hysteresis state (train_kan_fet_ett.py:51-83, 155-197) — against
    oracle/ett_ref.py in fp32 and fp64 on 8 windows spread over the batch (both row-tile edges and
    4 seeded random rows).  Bar: the envelope rule above, |gpu - fp64| <= 4 |ref fp32 - fp64|
    + 1e-5 x scale over the 8 x 96 forecasts, the fp32 term the worst of the reference's own
    rounding and three re-roundings of its parameters."""
    c = p = 96
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=c, pred_len=p, latent_dim=64, solver="rk4")
    with torch.no_grad():   # bench.ett_rate's scaling of the untrained field
        for n, p_ in m.dynamics.net.named_parameters():
            if n.endswith(("coef", "base_weight", "spline_weight", "logistic_weight")):
                p_.mul_(0.1)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(B + c + p, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], c, p, device=dev)
    xb, _ = ds.batch(torch.arange(B, device=dev))
    t_fut = torch.linspace(0.0, float(p - 1), steps=p)
    with torch.no_grad():
        got = m(xb, t_fut.to(dev), rk4_substeps=4)
    assert got.shape == (B, p) and torch.isfinite(got).all()
    gr = torch.Generator().manual_seed(22)
    rows = torch.cat([torch.tensor([0, 1, B - 2, B - 1]),
                      (torch.randperm(B - 4, generator=gr)[:4] + 2).sort().values])
    xs = xb[rows.to(dev)].cpu()
    torch.set_num_threads(min(16, torch.get_num_threads()))
    outs = {}
    for dt in (torch.float32, torch.float64):
        sdd = {k: v.to(dt) for k, v in sd.items()}
        field = O.KANFETRef.from_state_dict({k[len("dynamics.net."):]: v for k, v in sdd.items()
                                             if k.startswith("dynamics.net.")}, 2)
        ref = E.ForecasterRef(sdd, lambda tt, zz: field(zz))
        with torch.no_grad():
            outs[dt] = ref(xs.to(dt), t_fut.to(dt), rk4_substeps=4)
    # the yardstick over the reference's rounding and three equally valid re-roundings of its
    # parameters (one fp32 rounding is one draw of the 380-step error; the CPU's own rounding also
    # depends on its thread count)
    e64 = outs[torch.float64].double()
    worst32 = outs[torch.float32].double()
    gen = torch.Generator().manual_seed(0)
    for _ in range(3):
        sdp = {k: (v * (1 + 6e-8 * torch.randn(v.shape, generator=gen)) if v.is_floating_point()
                   and k.startswith("dynamics.net.") and not k.endswith(("grid", "prev_x", "branch_sign"))
                   else v) for k, v in sd.items()}
        fp = O.KANFETRef.from_state_dict({k[len("dynamics.net."):]: v for k, v in sdp.items()
                                          if k.startswith("dynamics.net.")}, 2)
        with torch.no_grad():
            c32 = E.ForecasterRef(sdp, lambda tt, zz: fp(zz))(xs, t_fut, rk4_substeps=4).double()
        if (c32 - e64).abs().max() > (worst32 - e64).abs().max():
            worst32 = c32
    rel, spread = _envelope(got.cpu()[rows], worst32, e64, "forecaster 96->96 x4 substeps, B=8192, 8 windows")
    print(f"config-4 horizon: |gpu-fp64|/scale {rel:.3e}, worst fp32 rounding vs fp64 /scale {spread:.3e}")
