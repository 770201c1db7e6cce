"""GPU parity: HIP kernels (through the C ABI) vs the golden fixtures / CPU oracle.

Tolerances: fp32 field maths uses hardware exp2/rcp and re-associated sums, so results
match the reference CPU values to rounding, not bitwise; the bar from BASELINE.json's
north_star is 1e-5 relative per trajectory time slice.  b_splines is bitwise.
"""
import numpy as np
import pytest
import torch

from conftest import golden_sd, load_golden

pytestmark = pytest.mark.gpu

REL = 1e-5


def slice_rel_err(a, b):
    """max over time slices of ||a_t - b_t|| / ||b_t|| (SURVEY §7.3 hard part 4 metric)."""
    a = a.double().reshape(a.shape[0], -1)
    b = b.double().reshape(b.shape[0], -1)
    return ((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-30)).max().item()


def close(a, b, rel=REL, floor=1e-6):
    a, b = a.double().cpu(), b.double().cpu()
    return bool(((a - b).abs() <= rel * b.abs() + floor).all()), (a - b).abs().max().item()


def test_bsplines_bitwise(dev):
    import fet_ode_amd as F
    for tag, (i, o) in (("kanlinear_2x10", (2, 10)), ("kanlinear_10x2", (10, 2))):
        g = load_golden(tag)
        m = F.KANLinear(i, o)
        m.load_state_dict(golden_sd(g))
        m = m.to(dev)
        x = torch.from_numpy(g["x"]).to(dev)
        b = m.b_splines(x).cpu()
        assert torch.equal(b, torch.from_numpy(g["bases"])), tag
        bo = m.b_splines(torch.from_numpy(g["x_odd"]).to(dev)).cpu()
        eo = torch.from_numpy(g["bases_odd"])
        assert torch.equal(torch.isnan(bo), torch.isnan(eo))
        assert torch.equal(torch.nan_to_num(bo), torch.nan_to_num(eo))


def test_kanlinear_forward(dev):
    import fet_ode_amd as F
    for tag, (i, o) in (("kanlinear_2x10", (2, 10)), ("kanlinear_10x2", (10, 2))):
        g = load_golden(tag)
        m = F.KANLinear(i, o)
        m.load_state_dict(golden_sd(g))
        m = m.to(dev)
        with torch.no_grad():
            y = m(torch.from_numpy(g["x"]).to(dev)).cpu()
        ok, md = close(y, torch.from_numpy(g["y"]))
        assert ok, (tag, md)


@pytest.mark.parametrize("tag,dims", [("ferro_2x10x10", (2, 10, 10)), ("ferro_10x2x10", (10, 2, 10))])
def test_ferro_sequences(dev, tag, dims):
    import fet_ode_amd as F
    g = load_golden(tag)
    i, o, K = dims
    # (a) fresh, B=1: prev_x = zeros -> dx = x ; activations returned
    m = F.FerroelectricBasis(i, o, K)
    m.load_state_dict(golden_sd(g), strict=False)
    m.reset_state()
    m = m.to(dev)
    for n in range(g["xs1"].shape[0]):
        with torch.no_grad():
            y, basis, _ = m(torch.from_numpy(g["xs1"][n]).to(dev), return_activations=True)
        ok, md = close(y.cpu(), torch.from_numpy(g["ys1"][n]))
        assert ok, ("B=1 out", n, md)
        ok, md = close(basis.cpu(), torch.from_numpy(g["basis1"][n]))
        assert ok, ("B=1 basis", n, md)
        assert torch.equal(m.prev_x[:, :, 0, 0].cpu(), torch.from_numpy(g["prev1"][n]))
    # (b) fresh, B=5: re-init rule (dx = 0 on the first call), then 4 more calls
    m2 = F.FerroelectricBasis(i, o, K)
    m2.load_state_dict(golden_sd(g, "sd2/"), strict=False)
    m2.reset_state()
    m2 = m2.to(dev)
    for n in range(g["xs5"].shape[0]):
        with torch.no_grad():
            y = m2(torch.from_numpy(g["xs5"][n]).to(dev))
        ok, md = close(y.cpu(), torch.from_numpy(g["ys5"][n]))
        assert ok, ("B=5", n, md)
        assert m2.prev_x.shape == (5, i, o, K)
    # (c) after reset_state
    m2.reset_state()
    with torch.no_grad():
        y = m2(torch.from_numpy(g["x_reset"]).to(dev))
    ok, md = close(y.cpu(), torch.from_numpy(g["y_reset"]))
    assert ok, ("reset", md)


def _kanfet_from(g, dev):
    import fet_ode_amd as F
    m = F.KANFET([2, 10, 2], grid_size=5)
    m.load_state_dict(golden_sd(g))
    return m.to(dev)


def test_kanfet_field_two_calls(dev):
    g = load_golden("kanfet_field")
    m = _kanfet_from(g, dev)
    y0 = torch.from_numpy(g["y0"]).to(dev)
    with torch.no_grad():
        f1 = m(y0).cpu()
        f2 = m(y0 * 1.01 + 0.05).cpu()
    for got, exp in ((f1, g["f1"]), (f2, g["f2"])):
        ok, md = close(got, torch.from_numpy(exp), floor=1e-5)
        assert ok, md


@pytest.mark.parametrize("B", [1, 64])
@pytest.mark.parametrize("tag", ["t35", "t140"])
def test_fused_rk4_kan_trajectories(dev, B, tag):
    """KAN field (predator_prey.py:101): well conditioned in fp32 (reference fp32 vs fp64 ~2e-7),
    so the whole trajectory must match the reference CPU odeint within 1e-5 per time slice."""
    import fet_ode_amd as F
    g = load_golden("traj_kan")
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(golden_sd(g))
    m = m.to(dev)
    y0 = torch.from_numpy(g[f"y0_B{B}"]).to(dev)
    with torch.no_grad():
        sol = F.odeint(F.autonomous(m), y0, torch.from_numpy(g[tag]), method="rk4").cpu()
    assert slice_rel_err(sol, torch.from_numpy(g[f"sol_B{B}_{tag}"])) <= REL


def _set_states(model, prevs, dev):
    for layer, p in zip(model.layers, prevs):
        layer.ferro._prev = p.clone().to(dev)
        layer.ferro._bsign = None


@pytest.mark.parametrize("B", [1, 64])
@pytest.mark.parametrize("tag", ["t35", "t140"])
def test_fused_rk4_kanfet_one_step_parity(dev, B, tag):
    """KAN-FET: teacher-forced local parity.  From the reference's own (y_j, prev_x_j) every
    fused RK4 step must land on the reference's y_{j+1} within 1e-5 (per-slice relative).
    (The reference's own fp32 one-step error vs fp64 is <= 1e-6 on these cases.)"""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    ref = O.KANFETRef.from_state_dict(sd, 2)
    y0 = torch.from_numpy(g[f"y0_B{B}"])
    t = torch.from_numpy(g[tag])
    # teacher = the oracle run on THIS host (its CPU may round transcendentals differently
    # from the fixture host; the oracle==fixture bitwise pin is tests/test_oracle_golden.py)
    sol, recs = O.rk4_with_states(ref, y0, t)
    m = _kanfet_from(g, dev)
    worst = 0.0
    for j, (y, prevs) in enumerate(recs):
        _set_states(m, prevs, dev)
        with torch.no_grad():
            out = F.odeint(F.autonomous(m), y.to(dev), t[j:j + 2], method="rk4").cpu()
        worst = max(worst, slice_rel_err(out[1:], sol[j + 1:j + 2]))
        # the hysteresis state after the step is the last stage input (ferro_class.py:409)
    assert worst <= REL, worst


def _error_stats(a, s64):
    """Per-trajectory max-over-time relative error vs fp64: 25th percentile (the well-conditioned
    majority), geomean, max, and how many
    trajectories cross 1e-3 / 1e-2 (the fp32-diverging ones)."""
    e = ((a.double() - s64).norm(dim=2) / s64.norm(dim=2).clamp_min(1e-6)).max(0).values
    return {"p25": e.quantile(0.25).item(), "gmean": e.log().mean().exp().item(), "max": e.max().item(),
            "n1e-3": int((e > 1e-3).sum()), "n1e-2": int((e > 1e-2).sum())}


def fp32_error_envelope(sd, y0, t, s64, trials=6, seed=0):
    """How far an fp32 solve of this model may land from fp64 by rounding alone.

    KAN-FET trajectories are ill-conditioned in fp32 (the hysteresis gate amplifies
    x - prev_x rounding).  Re-running the CPU fp32 oracle with every parameter moved by a
    fraction of an ulp (an equally valid fp32 rounding of the same model), 4-7 of the 64
    LV trajectories always end 1e-2..6e-2 away from fp64 and the rest stay near 3e-5 — so any
    percentile near the 90th jumps between 1e-3 and 2e-2 from rounding alone.  The envelope
    is the worst value of each statistic over the unperturbed run and `trials` perturbed runs
    (tools/diag/acc_dist.py prints the distributions)."""
    from oracle import torch_ref as O
    env = None
    gen = torch.Generator().manual_seed(seed)
    for trial in range(trials + 1):
        sdp = {k: (v * (1 + 6e-8 * torch.randn(v.shape, generator=gen)) if trial and v.dtype == torch.float32
                   and "grid" not in k else v) for k, v in sd.items()}
        r = O.KANFETRef.from_state_dict(sdp, 2)
        with torch.no_grad():
            st = _error_stats(O.odeint(lambda tt, yy: r(yy), y0, t, method="rk4"), s64)
        env = st if env is None else {k: max(env[k], st[k]) for k in env}
    return env


@pytest.mark.parametrize("tag", ["t35", "t140"])
def test_fused_rk4_kanfet_accuracy_parity(dev, tag):
    """The GPU trajectory must be as accurate as the reference's CPU fp32 odeint, measured
    against the fp64 oracle: typical error (25th percentile, geomean) within 2x of the fp32
    rounding envelope, no more fp32-diverging trajectories than that envelope (+max(2, 15%)),
    and no larger worst error (x1.5).  The committed reference fp32 run joins the envelope."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    B = 64
    y0 = torch.from_numpy(g[f"y0_B{B}"])
    t = torch.from_numpy(g[tag])
    ref64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
    s64 = O.odeint(lambda tt, yy: ref64(yy), y0.double(), t, method="rk4")
    m = _kanfet_from(g, dev)
    with torch.no_grad():
        gpu = F.odeint(F.autonomous(m), y0.to(dev), t, method="rk4").cpu().double()
    assert torch.isfinite(gpu).all()
    eg = _error_stats(gpu, s64)
    ec = _error_stats(torch.from_numpy(g[f"sol_B{B}_{tag}"]), s64)
    env = {k: max(v, ec[k]) for k, v in fp32_error_envelope(sd, y0, t, s64).items()}
    msg = (eg, env)
    assert eg["p25"] <= 2 * env["p25"] and eg["gmean"] <= 2 * env["gmean"], msg
    for k in ("n1e-2", "n1e-3"):
        assert eg[k] <= env[k] + max(2, int(0.15 * env[k])), msg
    assert eg["max"] <= 1.5 * env["max"], msg
    # final hysteresis state == last stage input of the last step, on the GPU trajectory
    assert m.layers[0].ferro.prev_x.shape == (B, 2, 10, 10)


def test_per_stage_path_matches_fused(dev):
    """calDeriv-style closure (per-stage path) == fused path, including hysteresis state."""
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    m1 = _kanfet_from(g, dev)
    m2 = _kanfet_from(g, dev)
    y0 = torch.from_numpy(g["y0_B64"]).to(dev)
    t = torch.from_numpy(g["t35"])
    with torch.no_grad():
        a = F.odeint(F.autonomous(m1), y0, t, method="rk4")
        with F.closure_fusion(False):   # the closure stage by stage
            b = F.odeint(lambda tt, yy: m2(yy), y0, t, method="rk4")
    # same kernels and op order per stage: identical up to launch-boundary effects (none expected)
    assert slice_rel_err(b.cpu(), a.cpu()) <= 1e-6
    assert torch.allclose(m1.layers[1].ferro.prev_x, m2.layers[1].ferro.prev_x, rtol=1e-5, atol=1e-6)


def test_reference_caldriv_closure_takes_fused_path(dev):
    """The reference's unchanged calDeriv (train_kanfet_node_predprey.py:159-161) is integrated on
    the fused path: bitwise the autonomous() solve, hysteresis state included; the training solve
    (tape + reverse sweep) gives bitwise the same gradients; dopri5 runs resident."""
    import fet_ode_amd as F
    from fet_ode_amd.dopri5 import ResidentSolve
    g = load_golden("traj_kanfet")
    m1 = _kanfet_from(g, dev)
    m2 = _kanfet_from(g, dev)
    y0 = torch.from_numpy(g["y0_B64"]).to(dev)
    t = torch.from_numpy(g["t35"])

    def calDeriv(t, X):
        dXdt = m2(X)
        return dXdt

    with torch.no_grad():
        a = F.odeint(F.autonomous(m1), y0, t, method="rk4")
        b = F.odeint(calDeriv, y0, t, method="rk4")
    assert torch.equal(a, b)
    for l1, l2 in zip(m1.layers, m2.layers):
        assert torch.equal(l1.ferro.prev_x, l2.ferro.prev_x)
    grads = []
    for func, m in ((F.autonomous(m1), m1), (calDeriv, m2)):
        m.reset_state()
        m.zero_grad(set_to_none=True)
        F.odeint(func, y0, t[:8], method="rk4").square().mean().backward()
        grads.append([p.grad.clone() for p in m.parameters()])
    for ga, gb in zip(*grads):
        assert torch.equal(ga, gb)
    with torch.no_grad():
        F.odeint(calDeriv, y0, t[:6], rtol=1e-3, atol=1e-4)
    assert isinstance(F.dopri5.dopri5_solve.last, ResidentSolve)


def test_state_carries_over_between_solves(dev):
    """pred_test = odeint(...) after the training solve sees the carried hysteresis state
    (train_kanfet_node_predprey.py:252,260): the second solve's first step starts from the
    state the first solve left, on GPU exactly as in the oracle."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    m = _kanfet_from(g, dev)
    ref = O.KANFETRef.from_state_dict(golden_sd(g), 2)
    y0 = torch.from_numpy(g["y0_B64"])
    t1 = torch.from_numpy(g["t35"])[:3]
    t2 = torch.linspace(0, 0.2, 3)
    with torch.no_grad():
        F.odeint(F.autonomous(m), y0.to(dev), t1, method="rk4")
        p_gpu = [l.ferro._prev.cpu() for l in m.layers]
        b = F.odeint(F.autonomous(m), y0.to(dev), t2, method="rk4").cpu()
        O.odeint(lambda tt, yy: ref(yy), y0, t1, method="rk4")
        p_ref = [s.prev_x[:, :, 0, 0].clone() for s in ref.states]
        e = O.odeint(lambda tt, yy: ref(yy), y0, t2, method="rk4")
    # two steps of an ill-conditioned field: agree to 1e-3 (fp32 amplification), and the
    # second solve continues from that carried state (a fresh state would differ by O(1))
    for a, r in zip(p_gpu, p_ref):
        assert torch.allclose(a, r, rtol=1e-3, atol=1e-4)
    assert slice_rel_err(b, e) <= 1e-3
    fresh = _kanfet_from(g, dev)
    with torch.no_grad():
        c = F.odeint(F.autonomous(fresh), y0.to(dev), t2, method="rk4").cpu()
    assert slice_rel_err(c, e) > 1e-3   # the carried state matters


def test_plan_cache_follows_parameter_updates(dev):
    """The pre-transformed plan is reused across solves only while no parameter changed: an
    in-place update (optimizer-style) or load_state_dict must show up in the next solve."""
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    y0 = torch.from_numpy(g["y0_B64"]).to(dev)
    t = torch.from_numpy(g["t35"])[:5]

    def warm():
        mm = _kanfet_from(g, dev)
        F.odeint(F.autonomous(mm), y0, t, method="rk4")   # builds and caches the plan
        return mm

    def solve(mm):
        mm.reset_state()
        return F.odeint(F.autonomous(mm), y0, t, method="rk4").cpu()

    with torch.no_grad():
        m = warm()
        for layer in m.layers:
            layer.kan.base_weight.mul_(1.5)
            layer.ferro.coef.add_(0.01)
        a = solve(m)
        fresh = warm()
        for lf, lm in zip(fresh.layers, m.layers):
            lf.kan.base_weight.copy_(lm.kan.base_weight)
            lf.ferro.coef.copy_(lm.ferro.coef)
        assert torch.equal(a, solve(fresh))
        m.load_state_dict(golden_sd(g))      # replaces weights AND the hysteresis buffers
        c = solve(m)
        assert torch.equal(c, solve(_kanfet_from(g, dev))) and not torch.equal(a, c)


@pytest.mark.parametrize("tag", ["t35", "t140"])
def test_fused_rk4_kanfet_robust_subset_b64(dev, tag):
    """B = 64 golden workload (the committed reference fp32 run is the reference solve): on the
    trajectories every equally valid reference rounding keeps within 1e-5 of fp64, the GPU stays
    within 2e-5 of the reference on >= 97 % and no farther than the reference's own re-roundings
    (oracle/parity.py)."""
    import fet_ode_amd as F
    from oracle import parity as P
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    y0 = torch.from_numpy(g["y0_B64"])
    t = torch.from_numpy(g[tag])
    ref64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
    s64 = O.odeint(lambda tt, yy: ref64(yy), y0.double(), t, method="rk4")
    m = _kanfet_from(g, dev)
    with torch.no_grad():
        gpu = F.odeint(F.autonomous(m), y0.to(dev), t, method="rk4").cpu()
    runs = P.perturbed_solves(sd, y0, t, 5)
    st = P.robust_parity(gpu, torch.from_numpy(g[f"sol_B64_{tag}"]), s64, runs[:3], runs[3:])
    print(tag, st)
    # t35: ~10 of 64 are robust; over 140 points none is (the bar reduces to the fraction test)
    assert st["n_robust"] >= (4 if tag == "t35" else 0), st
    assert P.robust_parity_ok(st), st


def test_fused_rk4_kanfet_robust_subset_bench_config(dev):
    """The bench workload itself (bench.py make_problem: B = 4096, t = linspace(0, 3.5, 35), seed-0
    weights and y0) with the same bar; measured: the reference keeps 31-46 % of the trajectories
    within 1e-5 of fp64 depending on its rounding, ~950 under all of them."""
    import numpy as np
    import fet_ode_amd as F
    from oracle import parity as P
    from oracle import torch_ref as O
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    y0 = O.lv_y0(4096, 0)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    with torch.no_grad():
        gpu = F.odeint(F.autonomous(m), y0.to(dev), t, method="rk4").cpu()
        r32 = O.KANFETRef.from_state_dict(sd, 2)
        e32 = O.odeint(lambda tt, yy: r32(yy), y0, t, method="rk4")
        r64 = O.KANFETRef.from_state_dict(sd, 2).to(torch.float64)
        e64 = O.odeint(lambda tt, yy: r64(yy), y0.double(), t, method="rk4")
    runs = P.perturbed_solves(sd, y0, t, 5)
    st = P.robust_parity(gpu, e32, e64, runs[:3], runs[3:])
    print("robust-subset parity (bench config):", st)
    assert st["n_robust"] >= 256, st
    assert P.robust_parity_ok(st), st
    # north-star 1e-5 itself: no more GPU trajectories beyond it than the worst re-rounded reference
    # (round 3 measurement: GPU 29, controls 36 / 40 of 978)
    assert P.robust_parity_at_tol_ref_ok(st), st


@pytest.mark.parametrize("B", [1, 7, 64, 512])
@pytest.mark.parametrize("method", ["rk4", "rk4_classic", "midpoint", "euler"])
def test_small_batch_kernel_matches_v4(dev, kernel_switch, B, method):
    """v6 (one trajectory per 3-wave workgroup, the strong-scaling kernel) and v4 (two per wave)
    integrate the same KAN-FET solve: 3 steps (each from its own hysteresis state, first-call rule
    included) within 1e-5 per slice, and the same final hysteresis state; KAN (no hysteresis)
    over the whole 35-point grid within 1e-5 of the reference fixture."""
    import fet_ode_amd as F
    g = load_golden("traj_kanfet")
    y0 = torch.from_numpy(g["y0_B64"]).repeat(8, 1)[:B].to(dev)
    t = torch.from_numpy(g["t35"])[:4]
    outs, states = [], []
    for small in (True, False):
        kernel_switch(small)
        m = _kanfet_from(g, dev)
        with torch.no_grad():
            outs.append(F.odeint(F.autonomous(m), y0, t, method=method).cpu())
        states.append([l.ferro._prev.cpu() for l in m.layers])
    assert slice_rel_err(outs[0], outs[1]) <= 1e-5
    for a, b in zip(*states):   # layer-1 state = hidden h (sums with cancellation): 1e-4 normwise
        assert ((a - b).norm() / b.norm()).item() <= 1e-4
    if method == "rk4":
        gk = load_golden("traj_kan")
        for small in (True, False):
            kernel_switch(small)
            m = F.KAN([2, 10, 2], grid_size=5)
            m.load_state_dict(golden_sd(gk))
            m = m.to(dev)
            yk = torch.from_numpy(gk["y0_B64"]).repeat(8, 1)[:B]
            with torch.no_grad():
                sol = F.odeint(F.autonomous(m), yk.to(dev), torch.from_numpy(gk["t35"]), method="rk4").cpu()
            # KAN is stateless: row i of the repeated batch is fixture trajectory i % 64
            exp = torch.from_numpy(gk["sol_B64_t35"])[:, torch.arange(B) % 64]
            assert slice_rel_err(sol, exp) <= REL, small


def test_small_batch_kernel_single_eval_and_reference(dev, kernel_switch):
    """fetode_field_forward on v6: two stateful KAN-FET calls against the reference fixture."""
    kernel_switch(True)
    test_kanfet_field_two_calls(dev)


def test_small_batch_kernel_nonfinite_and_offgrid_inputs(dev, kernel_switch):
    """v6 and v4 field evaluations on rows with NaN / +-inf / off-grid / on-knot inputs, two
    stateful calls (the second sees the first's non-finite hysteresis inputs): the same NaN
    pattern as the reference oracle (non-finite x -> NaN bases, efficientkan.py:34-40) and the
    same finite values (1e-5)."""
    from oracle import torch_ref as O
    g = load_golden("kanfet_field")
    nan, inf = float("nan"), float("inf")
    y = torch.tensor([[nan, 0.5], [0.5, inf], [-inf, 1.0], [12.0, -12.0], [-1.0, 1.0], [0.6, 2.2],
                      [-2.2, -0.2], [0.3, -0.7], [1.5, 1.5], [2.19, -2.19]], dtype=torch.float32)
    y2 = y.flip(0) * 0.9 + 0.05
    outs = {}
    for small in (True, False):
        kernel_switch(small)
        m = _kanfet_from(g, dev)
        with torch.no_grad():
            outs[small] = (m(y.to(dev)).cpu(), m(y2.to(dev)).cpu())
    ref = O.KANFETRef.from_state_dict(golden_sd(g), 2)
    with torch.no_grad():
        exp = (ref(y), ref(y2))
    for k in range(2):
        a, b, e = outs[True][k], outs[False][k], exp[k]
        assert torch.equal(torch.isnan(a), torch.isnan(e)), (k, a, e)
        assert torch.equal(torch.isnan(b), torch.isnan(e)), (k, b, e)
        ok, md = close(torch.nan_to_num(a), torch.nan_to_num(b), floor=1e-5)
        assert ok, (k, md)
        ok, md = close(torch.nan_to_num(a), torch.nan_to_num(e), floor=1e-5)
        assert ok, (k, md)


def _forced_kernel_vs_two_per_wave(dev, B, force):
    """KAN-FET 3 rk4 steps with odd rows (NaN / +-inf / off-grid / on-knot states) under the kernel
    `force` selects (a fused_ranges.set(...) argument dict) against the two-trajectories-per-wave
    kernel, and KAN over the 35-point grid against the fixture under the forced kernel."""
    import fet_ode_amd as F
    from conftest import fused_ranges
    g = load_golden("traj_kanfet")
    y0 = torch.from_numpy(g["y0_B64"]).repeat((B + 63) // 64, 1)[:B].clone()
    odd = torch.tensor([[float("nan"), 0.5], [0.5, float("inf")], [-float("inf"), 1.0], [12.0, -12.0],
                        [0.6, 2.2], [-2.2, -0.2], [2.19, -2.19]], dtype=torch.float32)
    y0[:min(B, 7)] = odd[:min(B, 7)]
    t = torch.from_numpy(g["t35"])[:4]
    off = dict(small=0, tpw1=(0, 0), v8=(0, 0))
    outs, states = [], []
    with fused_ranges() as fr:
        for forced in (True, False):
            fr.set(**off)
            if forced:
                fr.set(**force)
            m = _kanfet_from(g, dev)
            with torch.no_grad():
                outs.append(F.odeint(F.autonomous(m), y0.to(dev), t, method="rk4").cpu())
            states.append([l.ferro._prev.cpu() for l in m.layers])
        a, b = outs
        assert torch.equal(torch.isnan(a), torch.isnan(b)), "NaN pattern differs from the two-per-wave kernel"
        fin = torch.isfinite(b).all(-1).all(0)          # trajectories that stay finite
        if fin.any():
            err = slice_rel_err(a[:, fin], b[:, fin])
            assert err <= 1e-5, f"KAN-FET slices vs the two-per-wave kernel: {err}"
        for li, (sa, sb) in enumerate(zip(*states)):
            assert torch.equal(torch.isnan(sa), torch.isnan(sb)), f"layer {li} hysteresis NaN pattern"
            ok = torch.isfinite(sb).all(-1)
            if ok.any():
                rel = ((sa[ok] - sb[ok]).norm() / sb[ok].norm()).item()
                assert rel <= 1e-4, f"layer {li} hysteresis state vs the two-per-wave kernel: {rel}"
        gk = load_golden("traj_kan")
        yk = torch.from_numpy(gk["y0_B64"]).repeat((B + 63) // 64, 1)[:B]
        exp = torch.from_numpy(gk["sol_B64_t35"])[:, torch.arange(B) % 64]
        fr.set(**off).set(**force)
        m = F.KAN([2, 10, 2], grid_size=5)
        m.load_state_dict(golden_sd(gk))
        m = m.to(dev)
        with torch.no_grad():
            sol = F.odeint(F.autonomous(m), yk.to(dev), torch.from_numpy(gk["t35"]), method="rk4").cpu()
        err = slice_rel_err(sol, exp)
        assert err <= REL, f"KAN trajectories vs the reference fixture: {err}"


@pytest.mark.parametrize("B", [1, 7, 512, 1000, 2048])
def test_one_trajectory_per_wave_matches_two(dev, B):
    """The rk4 inference kernel at one trajectory per wave (fetode_fused_set_tpw1_range: each hidden
    unit's lane group split over both half-waves, the halves' partial sums met by a permlane32 swap;
    forced at every batch) against the two-trajectories-per-wave kernel: KAN-FET 3 steps within 1e-5
    per slice and the same hysteresis state (1e-4 normwise, as the v6 comparison above), KAN over the
    35-point grid within the fixture bar, and rows with NaN / +-inf / off-grid / on-knot states giving
    the same NaN pattern and finite values (1e-5)."""
    _forced_kernel_vs_two_per_wave(dev, B, dict(tpw1=(0, 1 << 40)))


@pytest.mark.parametrize("B", [1, 7, 512, 1000, 2048])
def test_two_waves_per_trajectory_matches_two_per_wave(dev, B):
    """v8 (fetode_fused_set_v8_range: one trajectory per two-wave workgroup, 12 lanes per hidden unit,
    spline cubics in registers, one LDS exchange of the two waves' output partials per evaluation;
    forced at every batch) under the same bars as the one-per-wave kernel above."""
    _forced_kernel_vs_two_per_wave(dev, B, dict(v8=(0, 1 << 40)))
