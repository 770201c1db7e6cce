"""GPU parity of the ECG KAN-FET NODE (train_ecg_kan_fet_nn_ode.py; BASELINE configs[2]) against
fixtures made from the reference classes and against the CPU oracle (oracle/ecg_ref.py)."""
import numpy as np
import pytest
import torch

from conftest import golden_sd, load_golden

pytestmark = pytest.mark.gpu


def close(got, exp, rel, name):
    got, exp = got.detach().double().cpu(), exp.detach().double().cpu()
    scale = exp.abs().max().item() + 1e-12
    err = (got - exp).abs().max().item()
    assert err <= rel * scale, f"{name}: max|diff|={err:.3e} scale={scale:.3e}"


def test_hlogistic_call_sequence(dev):
    """Four calls with batch sizes 8, 8, 5, 6: basis values, the last-row memory prev_x and the
    rebound (B, in, nb) branch_state after every call; a row equal to the remembered last row
    (dx = 0) takes the down branch."""
    from fet_ode_amd import ecg
    g = load_golden("ecg_hlogistic")
    m = ecg.LogisticBasis(64, 10)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    with torch.no_grad():
        for c in range(4):
            y = m(torch.from_numpy(g[f"x{c}"]).to(dev))
            close(y, torch.from_numpy(g[f"y{c}"]), 2e-6, f"basis {c}")
            assert torch.equal(m.prev_x.cpu(), torch.from_numpy(g[f"prev_x{c}"])), c
            assert torch.equal(m.branch_state.cpu(), torch.from_numpy(g[f"branch_state{c}"])), c
    m.reset_state()
    assert (m.prev_x == 0).all() and (m.branch_state == 1).all()


def test_hlogistic_grads(dev):
    from fet_ode_amd import ecg
    g = load_golden("ecg_hlogistic")
    m = ecg.LogisticBasis(64, 10)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    with torch.no_grad():
        for c in range(4):
            m(torch.from_numpy(g[f"x{c}"]).to(dev))
    x = torch.from_numpy(g["x5"]).to(dev).requires_grad_(True)
    (m(x) * torch.from_numpy(g["w5"]).to(dev)).sum().backward()
    close(x.grad, torch.from_numpy(g["grad/x"]), 1e-5, "x")
    for n in ("k", "Ec", "Ps", "bias"):
        close(getattr(m, n).grad, torch.from_numpy(g["grad/" + n]), 1e-5, n)
    assert m.coef.grad is None   # coef is unused by the reference forward (:88)


def test_field_calls_and_grads(dev):
    """No_MLP_KANODEFunc: two stateful calls (mixer + Linear head in one launch) and the
    gradients of a fixed loss on the second, against the reference's autograd."""
    from fet_ode_amd import ecg
    g = load_golden("ecg_field")
    f = ecg.No_MLP_KANODEFunc(latent_dim=64, num_basis=10, hidden=128)
    f.load_state_dict(golden_sd(g))
    f = f.to(dev)
    t = torch.tensor(0.0)
    with torch.no_grad():
        y1 = f(t, torch.from_numpy(g["h1"]).to(dev))
    close(y1, torch.from_numpy(g["y1"]), 1e-5, "y1")
    h2 = torch.from_numpy(g["h2"]).to(dev).requires_grad_(True)
    y2 = f(t, h2)
    close(y2, torch.from_numpy(g["y2"]), 1e-5, "y2")
    (y2 * torch.from_numpy(g["w"]).to(dev)).sum().backward()
    close(h2.grad, torch.from_numpy(g["grad/h"]), 1e-5, "h")
    for n, p in f.named_parameters():
        exp = g["grad/" + n]
        if np.isnan(exp).all():
            assert p.grad is None, n
        else:
            close(p.grad, torch.from_numpy(exp), 1e-5, n)


@pytest.mark.parametrize("name", ["ecg_node64", "ecg_node1"])
def test_node_dopri5_vs_reference(dev, name):
    """KanFet_NODE.eval() on 16 synthetic series: the GPU dopri5 takes the reference's accept /
    reject sequence (same attempt count, same nfev incl. rejected attempts and the initial-step
    probe) and the logits match."""
    from fet_ode_amd import ecg
    g = load_golden(name)
    sd = golden_sd(g)
    latent = sd["encoder.weight"].shape[0]
    nb = sd["odefunc.feat.basis.k"].shape[1]
    m = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=latent, num_basis=nb, rtol=float(g["rtol"]),
                        atol=float(g["atol"]))
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    with torch.no_grad():
        lo = m(torch.from_numpy(g["x"]).to(dev))
    s = m.last_solve
    assert s.nfev == int(g["nfev"])
    att = np.array([[a[0], a[1], a[2], float(a[3])] for a in s.attempts])
    assert att.shape == g["attempts"].shape and (att[:, 3] == g["attempts"][:, 3]).all()
    np.testing.assert_allclose(att[:, 1], g["attempts"][:, 1], rtol=1e-4)
    close(lo, torch.from_numpy(g["logits"]), 1e-5, "logits")
    close(m.odefunc.feat.basis.prev_x, torch.from_numpy(g["prev_x_odefunc"]), 1e-5, "prev_x")


def test_node_dopri5_batch200_vs_oracle(dev):
    """BASELINE configs[2] shape: batch 200 (ECG200 train + test rows), latent 64, rtol 1e-3 /
    atol 1e-4, against the CPU oracle run here on the same seeded weights and series, in fp32 and
    fp64.  Bar (round 6): the reference-fp32 envelope of the ETT tests,
    |gpu - fp64| <= 4 |ref fp32 - fp64| + 1e-5 x scale over every logit — no row allowance.
    (The branch gate is a hard switch on x - prev_x decided close to fp32 resolution on this
    workload: the fp64 oracle's smallest gate margin is 9.1e-8, row 129, evaluation 24.  The resident
    solve the default path takes stays within 2.5e-7 of fp64 on every row; the host-driven loop of
    per-module kernels flips a basis on ~4 rows)"""
    from fet_ode_amd import ecg
    from oracle import ecg_ref as E
    torch.manual_seed(0)
    m = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=64, num_basis=10)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev).eval()
    x = E.ecg_x(200, seed=1)
    ref = E.ECGNodeRef(sd, rtol=1e-3, atol=1e-4)
    ref64 = E.ECGNodeRef({k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()},
                         rtol=1e-3, atol=1e-4)
    with torch.no_grad():
        lo = m(x.to(dev))
        le = ref(x)
        l64 = ref64(x.double())
    s = m.last_solve
    assert s.nfev == ref.trace.nfev and len(s.attempts) == len(ref.trace.attempts)
    assert ref64.trace.nfev == ref.trace.nfev
    lo, le = lo.cpu().double(), le.double()
    scale = l64.abs().max().item()
    err, spread = (lo - l64).abs().max().item(), (le - l64).abs().max().item()
    assert err <= 4 * spread + 1e-5 * scale, \
        f"logits B=200: |gpu-fp64| {err:.3e}, ref fp32 spread {spread:.3e}, scale {scale:.3e}"


def test_training_through_fixed_grid(dev):
    """The field's HIP VJP under a fixed-grid solve (rk4): gradients of every parameter match the
    oracle's autograd (dopri5: test_training_through_dopri5_vs_oracle_autograd)."""
    from fet_ode_amd import ecg
    import fet_ode_amd as F
    from oracle import ecg_ref as E
    from oracle import torch_ref as O
    torch.manual_seed(2)
    f = ecg.No_MLP_KANODEFunc(latent_dim=8, num_basis=6)
    sd = {k: v.clone() for k, v in f.state_dict().items()}
    f = f.to(dev)
    h0 = torch.randn(12, 8, generator=torch.Generator().manual_seed(3))
    t = torch.linspace(0, 1, 6, dtype=torch.float64)
    hg = h0.clone().to(dev).requires_grad_(True)
    F.odeint(f, hg, t, method="rk4").square().mean().backward()
    ps = {k: v.clone().double().requires_grad_(k.split(".")[-1] in ("k", "Ec", "Ps", "bias", "weight"))
          for k, v in sd.items()}
    ps["proj.bias"].requires_grad_(True)
    ref = E.ECGFieldRef.from_state_dict(ps)
    hc = h0.clone().double().requires_grad_(True)
    O.odeint(ref, hc, t, method="rk4").square().mean().backward()
    close(hg.grad, hc.grad, 1e-4, "h0")
    for n, p in f.named_parameters():
        if n.endswith("coef"):
            assert p.grad is None
            continue
        close(p.grad, ps[n].grad, 1e-4, n)


# rel: latent 1 (the __main__ config, :1181-1198) moves the last row by tiny amounts between
# evaluations, so the hard gate sigmoid(5 dx) > 0.5 sits at its fp32 threshold often: the
# reference's own fp32 CPU solve departs from fp64 by 4e-5 .. 1.4e-4 relative over seeds (local
# measurement), and two fp32 implementations flip different gates.  Bound: 5e-4 there, 1e-5 else.
@pytest.mark.parametrize("B,latent,nb,opts,rel0", [(200, 64, 10, None, 1e-5),
                                                  (37, 64, 10, {"first_step": 0.05}, 1e-5),
                                                  (16, 1, 12, None, 5e-4), (3, 5, 4, {"first_step": 0.3}, 1e-5),
                                                  (1000, 64, 10, None, 1e-5)])
def test_resident_dopri5_matches_host_driven(dev, B, latent, nb, opts, rel0):
    """The one-launch device-resident dopri5 (fetode_ecg_dopri5) against the host-driven dopri5
    (HIP field kernel per call, host accept/reject): identical attempt sequence and nfev, solution
    and the module state it leaves (prev_x, branch_state) equal to fp32 rounding."""
    import fet_ode_amd as F
    from fet_ode_amd import dopri5 as D5
    from fet_ode_amd import ecg
    from oracle import ecg_ref as E
    torch.manual_seed(B + latent)
    f = ecg.No_MLP_KANODEFunc(latent_dim=latent, num_basis=nb)
    sd = {k: v.clone() for k, v in f.state_dict().items()}
    h0 = (torch.randn(B, latent, generator=torch.Generator().manual_seed(9)) * 2).to(dev)
    t = torch.tensor([0.0, 0.3, 1.0], dtype=torch.float64)
    out = {}
    for resident in (True, False):
        m = ecg.No_MLP_KANODEFunc(latent_dim=latent, num_basis=nb)
        m.load_state_dict(sd)
        m = m.to(dev)
        prev = D5.set_resident_dopri5(resident)
        try:
            with torch.no_grad():
                sol = F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4, options=opts)
        finally:
            D5.set_resident_dopri5(prev)
        last = D5.dopri5_solve.last
        assert isinstance(last, D5.ResidentSolve) == resident
        out[resident] = (sol.cpu(), last.nfev, last.attempts, m.feat.basis.prev_x.cpu(),
                         m.feat.basis.branch_state.cpu())
    (s1, n1, a1, p1, b1), (s2, n2, a2, p2, b2) = out[True], out[False]
    assert n1 == n2 and len(a1) == len(a2)
    assert [a[3] for a in a1] == [a[3] for a in a2]
    np.testing.assert_allclose([a[1] for a in a1], [a[1] for a in a2], rtol=1e-5)
    # The hard branch switch makes some trajectories sensitive to fp32 rounding: where a basis'
    # dx rounds across 0 the other logistic is taken, and which implementation flips depends on
    # its roundings (the local CPU oracle's fp32 run differs from fp64 by 1.9e-4 on 4.9 for B=16,
    # latent 1; another host's CPU does not).  The bound is 1e-5 relative or twice the spread of
    # the CPU oracle's fp32 solves under 1-ulp perturbations of y0 around fp64, whichever is larger.
    from oracle import torch_ref as O
    sd64 = {k: v.double() for k, v in sd.items()}
    s64 = O.odeint(E.ECGFieldRef.from_state_dict(sd64), h0.cpu().double(), t, method="dopri5", rtol=1e-3,
                   atol=1e-4, options=opts)
    spread, se = 0.0, None
    for eps in (0.0, 2.0 ** -23, -(2.0 ** -23), 2.0 ** -22):
        s32 = O.odeint(E.ECGFieldRef.from_state_dict(sd), h0.cpu() * (1 + eps), t, method="dopri5", rtol=1e-3,
                       atol=1e-4, options=opts)
        se = s32 if se is None else se
        spread = max(spread, (s32.double() - s64).abs().max().item())
    scale = s64.abs().max().item()
    rel = max(rel0, 2.0 * spread / scale)
    close(s1, s2, rel, "solution resident vs host-driven")
    close(s1, se, rel, "solution vs oracle")
    close(p1, p2, rel, "prev_x")
    # branch flips only where dx rounds across the gate threshold: at most one row's worth where
    # the last row barely moves (latent 1)
    assert (b1 != b2).float().mean().item() <= (1e-2 if rel0 <= 1e-5 else 1.0 / B)


def test_resident_dopri5_nonfinite_raises(dev):
    import fet_ode_amd as F
    from fet_ode_amd import ecg
    torch.manual_seed(1)
    m = ecg.No_MLP_KANODEFunc(latent_dim=8, num_basis=4).to(dev)
    h0 = torch.randn(6, 8, device=dev)
    h0[3, 2] = float("nan")
    with torch.no_grad(), pytest.raises(AssertionError):
        F.odeint(m, h0, torch.tensor([0.0, 1.0]), method="dopri5", options={"first_step": 0.1})


def test_kanfet_node_forward_raises_deferred_status(dev):
    """KanFet_NODE.forward reads the resident solve's status after launching the classifier
    (dopri5.deferred_status): a non-finite state still raises AssertionError from the forward,
    and the next forward is unaffected."""
    from fet_ode_amd import ecg
    torch.manual_seed(3)
    m = ecg.KanFet_NODE(T=24, num_classes=2, latent_dim=8, num_basis=4).to(dev).eval()
    x = torch.randn(6, 24, device=dev)
    bad = x.clone()
    bad[2, 5] = float("nan")
    with torch.no_grad():
        with pytest.raises(AssertionError):
            m(bad)
        out = m(x)
    assert torch.isfinite(out).all()


# ---------------------------------------------------------------------------------------------
# The FerroElectricNet field of train_ecg.py (KANFetODEFunc)
# ---------------------------------------------------------------------------------------------

def _ferronet(sd, latent, hidden, K, dev):
    from fet_ode_amd import ecg
    f = ecg.KANFetODEFunc(latent_dim=latent, hidden_dim=hidden, num_basis=K)
    f.load_state_dict(sd)
    return f.to(dev)


def test_ferronet_field_calls_and_grads(dev):
    """KANFetODEFunc vs the reference class (fixture): batch calls (B > 1 first-call rule), a
    carried-state call with every parameter gradient, batch-1 calls incl. a 1-D h, and a field
    that saturates the +-50 clamp (clamped outputs pass no gradient)."""
    g = load_golden("ecg_ferronet_field")
    t = torch.tensor(0.0)
    f = _ferronet(golden_sd(g, "sd_a/"), 8, 16, 12, dev)
    with torch.no_grad():
        close(f(t, torch.from_numpy(g["a/h1"]).to(dev)), torch.from_numpy(g["a/y1"]), 1e-5, "a/y1")
    h2 = torch.from_numpy(g["a/h2"]).to(dev).requires_grad_(True)
    y2 = f(t, h2)
    close(y2, torch.from_numpy(g["a/y2"]), 1e-5, "a/y2")
    (y2 * torch.from_numpy(g["a/w"]).to(dev)).sum().backward()
    close(h2.grad, torch.from_numpy(g["a/grad/h"]), 1e-4, "a/grad/h")
    for n, p in f.named_parameters():
        close(p.grad, torch.from_numpy(g["a/grad/" + n]), 2e-4, "a/grad/" + n)
    f = _ferronet(golden_sd(g, "sd_b/"), 8, 16, 12, dev)
    with torch.no_grad():
        for c in range(3):
            y = f(t, torch.from_numpy(g[f"b/h{c}"]).to(dev))
            assert y.shape == (1, 8)
            close(y, torch.from_numpy(g[f"b/y{c}"]), 1e-5, f"b/y{c}")
    f = _ferronet(golden_sd(g, "sd_c/"), 8, 16, 12, dev)
    h = torch.from_numpy(g["c/h"]).to(dev).requires_grad_(True)
    y = f(t, h)
    yc = torch.from_numpy(g["c/y"])
    close(y, yc, 1e-5, "c/y")
    assert torch.equal(y.detach().cpu().abs() == 50, yc.abs() == 50)
    (y * torch.from_numpy(g["c/w"]).to(dev)).sum().backward()
    close(h.grad, torch.from_numpy(g["c/grad/h"]), 1e-4, "c/grad/h")
    for n, p in f.named_parameters():
        close(p.grad, torch.from_numpy(g["c/grad/" + n]), 2e-4, "c/grad/" + n)


@pytest.mark.parametrize("name,solver", [("ecg_ferronet_euler", "euler"), ("ecg_ferronet_dopri5", "dopri5")])
def test_ferronet_node_vs_reference(dev, name, solver):
    """KanFet_MLP_NODE.eval(): per-row batch-1 solves with the Ferro state carried across rows,
    the last row's logits and both layers' prev_x after the forward."""
    from fet_ode_amd import ecg
    g = load_golden(name)
    m = ecg.KanFet_MLP_NODE(T=96, num_classes=2, latent_dim=8, num_basis=12, ode_hidden=16, solver=solver,
                            rtol=float(g["rtol"]), atol=float(g["atol"]))
    m.load_state_dict(golden_sd(g))
    m = m.to(dev).eval()
    with torch.no_grad():
        lo = m(torch.from_numpy(g["x"]).to(dev))
    assert lo.shape == (1, 2)
    # bound: 1e-5 relative, or 4x the reference's own fp32-vs-fp64 spread (the oracle in fp64 on
    # the same weights): error-controlled dopri5 steps through the hysteresis amplify rounding
    # (fc1 prev_x: 1.9e-5 between the reference's fp32 and fp64 runs of this case)
    from oracle import ecg_ref as E
    r64 = E.FerroNetNodeRef({k: v.double() for k, v in golden_sd(g).items()}, solver=solver,
                            rtol=float(g["rtol"]), atol=float(g["atol"]))
    with torch.no_grad():
        l64 = r64(torch.from_numpy(g["x"]).double())
    for got, key, e64 in ((lo, "logits", l64), (m.odefunc.fc1.prev_x, "fc1_prev_x", r64.field.st1.prev_x),
                          (m.odefunc.fc2.prev_x, "fc2_prev_x", r64.field.st2.prev_x)):
        exp = torch.from_numpy(g[key])
        spread = (exp.double() - e64).abs().max().item() / (exp.abs().max().item() + 1e-12)
        close(got, exp, max(1e-5, 4.0 * spread), f"{name} {key}")


def _envelope_close(got, e32, e64, name, floor=1e-5, k=4.0):
    """|got - fp64| <= k * |fp32 reference - fp64| + floor * scale, elementwise maximum: the GPU
    must be as accurate as the reference's own fp32 arithmetic, within a factor k."""
    got, e32, e64 = got.detach().double().cpu(), e32.detach().double().cpu(), e64.detach().double().cpu()
    scale = e64.abs().max().item() + 1e-12
    spread = (e32 - e64).abs().max().item()
    err = (got - e64).abs().max().item()
    assert err <= k * spread + floor * scale, f"{name}: |gpu-fp64|={err:.3e} fp32 spread={spread:.3e} scale={scale:.3e}"


def test_ferronet_production_width_vs_oracle(dev):
    """The train_ecg.py __main__ widths (latent 64, hidden 128, K = 12): a batch-200 euler solve on
    [0, 0.5, 1] (stateful field calls through the solver) and the gradients of a loss on a batch-32
    call, against the oracle in fp64 with the reference's own fp32 error as the yardstick (sums of
    768 / 1536 Ferro terms of size ~3: the CPU fp32 run is 9e-4 from fp64 on a scale of 53)."""
    from fet_ode_amd import ecg
    import fet_ode_amd as F
    from oracle import ecg_ref as E
    from oracle import torch_ref as O
    torch.manual_seed(41)
    f = ecg.KANFetODEFunc(latent_dim=64, hidden_dim=128, num_basis=12)
    sd = {k: v.clone() for k, v in f.state_dict().items()}
    f = f.to(dev)
    gen = torch.Generator().manual_seed(42)
    h0 = torch.randn(200, 64, generator=gen)
    t = torch.tensor([0.0, 0.5, 1.0])
    r32 = E.FerroNetFieldRef.from_state_dict({k: v.clone() for k, v in sd.items()})
    r64 = E.FerroNetFieldRef.from_state_dict({k: v.double() for k, v in sd.items()})
    with torch.no_grad():
        sol = F.odeint(f, h0.to(dev), t, method="euler")
        s32 = O.odeint(r32, h0, t, method="euler")
        s64 = O.odeint(r64, h0.double(), t.double(), method="euler")
    _envelope_close(sol, s32, s64, "euler solution")
    _envelope_close(f.fc1.prev_x[:, :, :1, :1], r32.st1.prev_x[:, :, :1, :1], r64.st1.prev_x[:, :, :1, :1],
                    "fc1 prev_x")
    # gradients on a fresh batch-32 module pair (first call: dx = 0)
    f = ecg.KANFetODEFunc(latent_dim=64, hidden_dim=128, num_basis=12)
    f.load_state_dict(sd)
    f = f.to(dev)
    h1 = torch.randn(32, 64, generator=gen)
    w = torch.randn(32, 64, generator=gen)
    hd = h1.to(dev).requires_grad_(True)
    (f(torch.tensor(0.0), hd) * w.to(dev)).sum().backward()
    grads = {}
    for dt in (torch.float32, torch.float64):
        ps = {k: v.detach().to(dt).clone().requires_grad_("prev_x" not in k and "branch_sign" not in k)
              for k, v in sd.items()}
        hh = h1.detach().to(dt).clone().requires_grad_(True)
        (E.FerroNetFieldRef.from_state_dict(ps)(torch.tensor(0.0), hh) * w.to(dt)).sum().backward()
        grads[dt] = {"h": hh.grad, **{k: v.grad for k, v in ps.items() if v.grad is not None}}
    _envelope_close(hd.grad, grads[torch.float32]["h"], grads[torch.float64]["h"], "grad h")
    missing = [n for n, p in f.named_parameters() if p.grad is None or n not in grads[torch.float64]]
    assert not missing, (missing, sorted(grads[torch.float64]))
    for n, p in f.named_parameters():
        _envelope_close(p.grad, grads[torch.float32][n], grads[torch.float64][n], "grad " + n)


def test_training_through_dopri5_vs_oracle_autograd(dev):
    """train_ecg_kan_fet_nn_ode.py trains KanFet_NODE through dopri5: cross-entropy on the logits,
    loss.backward() through the host-driven GPU dopri5 (the resident solver is inference-only)
    with the mixer's HIP VJP, against the oracle's autograd — same attempts, every parameter
    gradient within 1e-3 relative (hysteresis gates are piecewise constant: no gradient flows
    through them in either)."""
    from fet_ode_amd import ecg
    from fet_ode_amd import dopri5 as D5
    from oracle import ecg_ref as E
    g = load_golden("ecg_node64")
    sd = golden_sd(g)
    m = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=64, num_basis=10, rtol=1e-3, atol=1e-4)
    m.load_state_dict(sd)
    m = m.to(dev).eval()
    x = torch.from_numpy(g["x"])
    y = torch.arange(x.shape[0]) % 2
    loss = torch.nn.functional.cross_entropy(m(x.to(dev)), y.to(dev))
    loss.backward()
    assert isinstance(D5.dopri5_solve.last, D5._Dopri5Grad)
    ps = {k: v.clone().requires_grad_(v.dtype.is_floating_point and "prev_x" not in k and "branch_state" not in k)
          for k, v in sd.items()}
    ref = E.ECGNodeRef(ps, rtol=1e-3, atol=1e-4)
    lref = torch.nn.functional.cross_entropy(ref(x), y)
    lref.backward()
    assert len(D5.dopri5_solve.last.attempts) == len(ref.trace.attempts)
    assert abs(loss.item() - lref.item()) <= 1e-5 * abs(lref.item())
    for n, p in m.named_parameters():
        exp = ps[n].grad
        if exp is None:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, n
            continue
        close(p.grad, exp, 1e-3, "grad " + n)
