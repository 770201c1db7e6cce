"""GPU dopri5 (torchdiffeq's default method) vs the oracle restatement and its golden trace."""
import numpy as np
import pytest
import torch

from conftest import golden_sd, load_golden

pytestmark = pytest.mark.gpu


def lv_field(t, X):
    """train_kanfet_node_predprey.py:41-47 with alpha, beta, gamma, delta = 1.5, 1, 3, 1."""
    x, y = X[..., 0], X[..., 1]
    return torch.stack([1.5 * x - x * y, x * y - 3.0 * y], -1)


@pytest.mark.parametrize("first_step", [None, 0.1])
def test_dopri5_lv_vs_oracle_and_lsoda(dev, first_step):
    """Adaptive control in fp32: when an attempt's error ratio is itself at rounding level
    (the automatically selected first step gives ~2e-5), GPU and CPU summation orders can pick
    different next steps, so only the accuracy is compared; with first_step=0.1 every ratio is
    well above rounding noise and the attempt sequences must coincide."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("lv_lsoda")
    t = torch.from_numpy(g["t"]).float()
    y0 = torch.tensor([[1.0, 1.0]])
    opts = None if first_step is None else {"first_step": first_step}
    with torch.no_grad():
        gpu = F.odeint(lv_field, y0.to(dev), t, rtol=1e-3, atol=1e-5, options=opts).cpu()
    tr = O.Dopri5Trace()
    cpu = O.odeint(lv_field, y0, t, rtol=1e-3, atol=1e-5, trace=tr, options=opts)
    solver = F.dopri5.dopri5_solve.last
    assert solver.nfev == 2 + 6 * len(solver.attempts) - (1 if first_step else 0)
    if first_step is not None:
        # identical control decisions until fp32 noise in the ratios (~1e-4 rel) compounds
        n = 20
        assert [a[3] for a in solver.attempts[:n]] == [a[3] for a in tr.attempts[:n]]
        np.testing.assert_allclose([a[1] for a in solver.attempts[:n]], [a[1] for a in tr.attempts[:n]],
                                   rtol=1e-3)
    assert abs(len(solver.attempts) - len(tr.attempts)) <= 0.1 * len(tr.attempts)
    # as accurate as the reference CPU solve, against the LSODA truth
    truth = torch.from_numpy(g["soln"])
    e_gpu = (gpu[:, 0].double() - truth).abs().max().item()
    e_cpu = (cpu[:, 0].double() - truth).abs().max().item()
    assert e_gpu <= 2 * e_cpu + 1e-3, (e_gpu, e_cpu)


def test_dopri5_kanfet_trace(dev):
    """Golden trace (tests/golden/dopri5_kanfet.npz): same attempt sequence (accept/reject
    pattern and step sizes) and the same dense output as the reference modules + restated
    solver.  Each attempt makes 6 stateful hysteresis calls, rejected ones included."""
    import fet_ode_amd as F
    g = load_golden("dopri5_kanfet")
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    with torch.no_grad(), F.closure_fusion(False):   # the host-driven solver (its attempt record)
        sol = F.odeint(lambda tt, yy: m(yy), torch.from_numpy(g["y0"]).to(dev), torch.from_numpy(g["t"]),
                       rtol=1e-3, atol=1e-4).cpu()
    solver = F.dopri5.dopri5_solve.last
    att = np.array([[a[0], a[1], a[2], float(a[3])] for a in solver.attempts])
    exp = g["attempts"]
    assert att.shape == exp.shape, (att.shape, exp.shape)
    np.testing.assert_array_equal(att[:, 3], exp[:, 3])
    np.testing.assert_allclose(att[:, 1], exp[:, 1], rtol=1e-3)   # dt ~ ratio^-1/5
    np.testing.assert_allclose(att[:, 2], exp[:, 2], rtol=1e-2, atol=1e-6)  # ill-conditioned field
    assert solver.nfev == int(g["nfev"])
    ref = torch.from_numpy(g["sol"])
    assert ((sol - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max() < 1e-4


def test_dopri5_kan_strict(dev):
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    sd = golden_sd(g)
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    ref = O.KANRef([O.KANLinearParams.from_state_dict(sd, f"layers.{l}.") for l in range(2)])
    y0 = torch.from_numpy(g["y0_B64"])
    t = torch.tensor([0.0, 0.5, 1.0, 2.0])
    with torch.no_grad():
        gpu = F.odeint(F.autonomous(m), y0.to(dev), t, rtol=1e-5, atol=1e-7).cpu()
        cpu = O.odeint(lambda tt, yy: ref(yy), y0, t, rtol=1e-5, atol=1e-7)
    assert ((gpu - cpu).norm(dim=(1, 2)) / cpu.norm(dim=(1, 2))).max() < 1e-5


@pytest.mark.parametrize("method", ["rk4", "dopri5", "euler", "midpoint"])
def test_reversed_time(dev, method):
    """torchdiffeq integrates decreasing t by negating time and the field (_ReverseFunc)."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    y0 = torch.tensor([[1.0, 1.0], [2.0, 0.5]])
    t = torch.linspace(2.0, 0.0, 9)
    with torch.no_grad():
        gpu = F.odeint(lv_field, y0.to(dev), t, method=method).cpu()
    cpu = O.odeint(lv_field, y0, t, method=method)
    assert (gpu - cpu).abs().max() < 1e-4 * cpu.abs().max()


def test_fused_reversed_and_step_size(dev):
    """Fused single-launch path: decreasing t and options={'step_size'} with linear interpolation."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    sd = golden_sd(g)
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    ref = O.KANRef([O.KANLinearParams.from_state_dict(sd, f"layers.{l}.") for l in range(2)])
    y0 = torch.from_numpy(g["y0_B64"])
    for t, opts in ((torch.linspace(1.0, 0.0, 6), None), (torch.tensor([0.0, 0.13, 0.5, 0.77]), {"step_size": 0.1})):
        for method in ("rk4", "euler", "midpoint"):
            with torch.no_grad():
                gpu = F.odeint(F.autonomous(m), y0.to(dev), t, method=method, options=opts).cpu()
            cpu = O.odeint(lambda tt, yy: ref(yy), y0, t, method=method, options=opts)
            err = ((gpu - cpu).norm(dim=(1, 2)) / cpu.norm(dim=(1, 2))).max()
            assert err < 1e-5, (method, opts, err)


@pytest.mark.parametrize("fused", [True, False])
def test_rk4_classic_fused_and_per_stage(dev, fused):
    """method='rk4_classic' = the reference's own fixed-step RK4 helpers
    (train_ecg_kan_fet_nn_ode.py:693-705, train_kan_fet_ett.py:51-83)."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    sd = golden_sd(g)
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    ref = O.KANRef([O.KANLinearParams.from_state_dict(sd, f"layers.{l}.") for l in range(2)])
    y0 = torch.from_numpy(g["y0_B64"])
    t = torch.from_numpy(g["t35"])
    func = F.autonomous(m) if fused else (lambda tt, yy: m(yy))
    with torch.no_grad(), F.closure_fusion(fused):
        gpu = F.odeint(func, y0.to(dev), t, method="rk4_classic").cpu()
    cpu = O.odeint(lambda tt, yy: ref(yy), y0, t, method="rk4_classic")
    assert ((gpu - cpu).norm(dim=(1, 2)) / cpu.norm(dim=(1, 2))).max() < 1e-5


# ---------------------------------------------------------------------------------------------
# device-resident dopri5 for the tagged LV fields (fetode_integrate_dopri5)
# ---------------------------------------------------------------------------------------------

def test_dopri5_kanfet_trace_resident(dev):
    """The golden trace again, through the whole-solve-in-one-launch path (the tagged field)."""
    import fet_ode_amd as F
    from fet_ode_amd.dopri5 import ResidentSolve
    g = load_golden("dopri5_kanfet")
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m), torch.from_numpy(g["y0"]).to(dev), torch.from_numpy(g["t"]),
                       rtol=1e-3, atol=1e-4).cpu()
    solver = F.dopri5.dopri5_solve.last
    assert isinstance(solver, ResidentSolve)
    att = np.array([[a[0], a[1], a[2], float(a[3])] for a in solver.attempts])
    exp = g["attempts"]
    assert att.shape == exp.shape, (att.shape, exp.shape)
    np.testing.assert_array_equal(att[:, 3], exp[:, 3])
    np.testing.assert_allclose(att[:, 1], exp[:, 1], rtol=1e-3)
    np.testing.assert_allclose(att[:, 2], exp[:, 2], rtol=1e-2, atol=1e-6)
    assert solver.nfev == int(g["nfev"])
    ref = torch.from_numpy(g["sol"])
    assert ((sol - ref).norm(dim=(1, 2)) / ref.norm(dim=(1, 2))).max() < 1e-4


@pytest.mark.parametrize("B", [1, 64, 1000, 4096])
@pytest.mark.parametrize("kind", ["kanfet", "kan"])
def test_dopri5_resident_matches_host_driven(dev, kernel_switch, B, kind):
    """One cooperative launch vs the host-driven loop (one fused v4 field launch per evaluation,
    the error norm read back per attempt) on the same model and inputs.  The field arithmetic is
    the same and the norms are fp64 sums in both, so up to B = 1000 the attempt sequences and nfev
    are identical, the step sizes equal up to the last ulp of fp64 pow (device libm vs host), the
    solution and hysteresis state within 1e-6.  At B = 4096 the fp64 sums' order differs enough to
    move a ratio by an fp32 ulp now and then, which the KAN-FET hysteresis amplifies — same accept
    pattern and nfev, dt within 1e-5, solution within 1e-4.  (The host path below B = 512 would run v6, a different rounding of the same
    field: tests/test_gpu_parity.py::test_small_batch_kernel_matches_v4 covers that pair.)"""
    import fet_ode_amd as F
    from fet_ode_amd.dopri5 import ResidentSolve, set_resident_dopri5
    kernel_switch(False)
    gk = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
    y0 = torch.from_numpy(gk["y0_B64"]).repeat(64, 1)[:B].to(dev)
    t = torch.tensor([0.0, 0.2, 0.5], dtype=torch.float64)
    out = []
    for resident in (True, False):
        prev = set_resident_dopri5(resident)
        try:
            m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
            m.load_state_dict(golden_sd(gk))
            m = m.to(dev)
            with torch.no_grad():
                sol = F.odeint(F.autonomous(m), y0, t, rtol=1e-3, atol=1e-4).cpu()
        finally:
            set_resident_dopri5(prev)
        s = F.dopri5.dopri5_solve.last
        assert isinstance(s, ResidentSolve) == resident
        states = [l.ferro._prev.cpu() for l in m.layers] if kind == "kanfet" else []
        out.append((sol, [(float(a[1]), float(a[3])) for a in s.attempts], s.nfev, states))
    (s0, a0, n0, st0), (s1, a1, n1, st1) = out
    assert n0 == n1 and [a[1] for a in a0] == [a[1] for a in a1]
    if B <= 1000:   # the same fp32 arithmetic; dt differs at most by fp64 pow's last ulp
        np.testing.assert_allclose([a[0] for a in a0], [a[0] for a in a1], rtol=1e-13)
        assert ((s0 - s1).norm(dim=(1, 2)) / s1.norm(dim=(1, 2)).clamp_min(1e-30)).max() <= 1e-6
        for a, b in zip(st0, st1):
            assert ((a - b).norm() / b.norm()).item() <= 1e-6
        return
    np.testing.assert_allclose([a[0] for a in a0], [a[0] for a in a1], rtol=1e-5)
    assert ((s0 - s1).norm(dim=(1, 2)) / s1.norm(dim=(1, 2)).clamp_min(1e-30)).max() <= 1e-4
    for a, b in zip(st0, st1):
        assert ((a - b).norm() / b.norm()).item() <= 1e-4


@pytest.mark.parametrize("B", [1, 64, 300])
@pytest.mark.parametrize("kind", ["kanfet", "kan"])
def test_dopri5_resident_small_batch_kernel(dev, kernel_switch, B, kind):
    """Small batches (the reference's own X0 (1, 2)): the resident solve runs on v6 (one
    trajectory per 192-thread workgroup) — against the host-driven loop whose evaluations are v6
    too: the same attempts, dt to fp64 pow's last ulp, solution and state within 1e-6."""
    import fet_ode_amd as F
    from fet_ode_amd.dopri5 import ResidentSolve, set_resident_dopri5
    kernel_switch(True)
    gk = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
    y0 = torch.from_numpy(gk["y0_B64"]).repeat(64, 1)[:B].to(dev)
    t = torch.tensor([0.0, 0.2, 0.5], dtype=torch.float64)
    out = []
    for resident in (True, False):
        prev = set_resident_dopri5(resident)
        try:
            m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
            m.load_state_dict(golden_sd(gk))
            m = m.to(dev)
            with torch.no_grad():
                sol = F.odeint(F.autonomous(m), y0, t, rtol=1e-3, atol=1e-4).cpu()
        finally:
            set_resident_dopri5(prev)
        s = F.dopri5.dopri5_solve.last
        assert isinstance(s, ResidentSolve) == resident
        states = [l.ferro._prev.cpu() for l in m.layers] if kind == "kanfet" else []
        out.append((sol, [(float(a[1]), float(a[3])) for a in s.attempts], s.nfev, states))
    (s0, a0, n0, st0), (s1, a1, n1, st1) = out
    assert n0 == n1 and [a[1] for a in a0] == [a[1] for a in a1]
    np.testing.assert_allclose([a[0] for a in a0], [a[0] for a in a1], rtol=1e-13)
    assert ((s0 - s1).norm(dim=(1, 2)) / s1.norm(dim=(1, 2)).clamp_min(1e-30)).max() <= 1e-6
    for a, b in zip(st0, st1):
        assert ((a - b).norm() / b.norm()).item() <= 1e-6


def test_dopri5_resident_reference_tolerances(dev):
    """The north-star call itself: torchodeint(calDeriv, X0, t_learn) with torchdiffeq's default
    rtol 1e-7 / atol 1e-9 on the bench workload (B = 4096, 35 points): thousands of attempts in
    one launch (rtol 1e-7 sits at fp32 resolution), finite, every attempt 6 evaluations."""
    import fet_ode_amd as F
    from fet_ode_amd.dopri5 import ResidentSolve
    from oracle import torch_ref as O
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    y0 = O.lv_y0(4096, 0).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m), y0, t)
    s = F.dopri5.dopri5_solve.last
    assert isinstance(s, ResidentSolve)
    assert torch.isfinite(sol).all()
    assert len(s.attempts) > 100 and s.nfev > 600


def test_dopri5_resident_falls_back_beyond_one_grid(dev):
    """A batch that cannot be co-resident takes the host-driven loop (no error, same API)."""
    import fet_ode_amd as F
    from fet_ode_amd.dopri5 import ResidentSolve
    g = load_golden("traj_kanfet")
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    y0 = torch.from_numpy(g["y0_B64"]).repeat(70, 1)[:4480].to(dev)
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m), y0, torch.tensor([0.0, 0.1], dtype=torch.float64), rtol=1e-3, atol=1e-4)
    assert torch.isfinite(sol).all() and not isinstance(F.dopri5.dopri5_solve.last, ResidentSolve)


@pytest.mark.parametrize("B", [64, 4096])
def test_dopri5_resident_timeout_restores_state(dev, B):
    """The timeout path on a healthy grid (fetode_dopri5_set_spin_limit(1): the first poll that
    does not find its reduction complete gives up): the resident solve raises RuntimeError
    (status 4) and `_restorer` puts the hysteresis memory back to its pre-solve value, so the
    caller can rerun — here on the host loop — and get exactly what the host loop gives from the
    untouched state.  Then the limit is restored and the resident solve works again."""
    import fet_ode_amd as F
    from fet_ode_amd import _lib
    from fet_ode_amd.dopri5 import ResidentSolve, set_resident_dopri5
    lib = _lib.load()
    g = load_golden("traj_kanfet")
    y0 = torch.from_numpy(g["y0_B64"]).repeat(64, 1)[:B].to(dev)
    t = torch.tensor([0.0, 0.2, 0.5], dtype=torch.float64)

    def model():
        m = F.KANFET([2, 10, 2], grid_size=5)
        m.load_state_dict(golden_sd(g))
        m = m.to(dev)
        with torch.no_grad():   # a carried (non-fresh) hysteresis state before the solve under test
            F.odeint(F.autonomous(m), y0, torch.tensor([0.0, 0.05], dtype=torch.float64), method="rk4")
        return m

    m = model()
    before = [l.ferro._prev.clone() for l in m.layers]
    prev = lib.fetode_dopri5_set_spin_limit(1)
    try:
        with torch.no_grad(), pytest.raises(RuntimeError, match="timed out"):
            F.odeint(F.autonomous(m), y0, t, rtol=1e-3, atol=1e-4)
            torch.cuda.synchronize(dev)
    finally:
        lib.fetode_dopri5_set_spin_limit(prev)
    for a, b in zip(before, [l.ferro._prev for l in m.layers]):
        assert torch.equal(a, b), "the pre-solve hysteresis state must survive a timed-out solve"
    # the caller's retry on the host loop == the host loop on a fresh copy of the same state
    pr = set_resident_dopri5(False)
    try:
        with torch.no_grad():
            retry = F.odeint(F.autonomous(m), y0, t, rtol=1e-3, atol=1e-4).cpu()
            m2 = model()
            clean = F.odeint(F.autonomous(m2), y0, t, rtol=1e-3, atol=1e-4).cpu()
    finally:
        set_resident_dopri5(pr)
    assert torch.equal(retry, clean)
    for a, b in zip([l.ferro._prev for l in m.layers], [l.ferro._prev for l in m2.layers]):
        assert torch.equal(a, b)
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m2), y0, t, rtol=1e-3, atol=1e-4)
    assert isinstance(F.dopri5.dopri5_solve.last, ResidentSolve) and torch.isfinite(sol).all()
