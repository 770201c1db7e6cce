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


@pytest.mark.parametrize("dims,nb", [((2, 16), 10), ((33, 5), 10), ((4, 64), 3), ((3, 7), 0), ((1, 12), 10),
                                     ((16, 2), 10), ((6, 4), 0), ((5, 3), 12), ((7, 1), 4)])
def test_kanlinear_grads_many_rows_vs_oracle(dev, dims, nb):
    """B = 4096 rows: the many-row parameter sums (fetode_grad.hip, B >= 2048) — the tile kernel
    (input groups of 1..4 with a ragged last group at 33 inputs, 64 outputs, no logistic basis, one
    input) and the row-owner kernel of narrow layers (out <= 4; NB 0, 4, 10, 12) — against the
    oracle's fp64 autograd (some rows off the grid on either side)."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    torch.manual_seed(3)
    m = F.KANLinear(*dims, num_basis=max(nb, 1), enable_logistic_basis=nb > 0)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    gen = torch.Generator().manual_seed(4)
    x = torch.rand(4096, dims[0], generator=gen) * 2.6 - 1.3
    w = torch.randn(4096, dims[1], generator=gen)
    xg = x.clone().to(dev).requires_grad_(True)
    (m(xg) * w.to(dev)).sum().backward()
    ps = {k: v.double().requires_grad_(k != "grid") for k, v in sd.items() if v.dtype.is_floating_point}
    p = O.KANLinearParams.from_state_dict(ps)
    xc = x.double().requires_grad_(True)
    (O.kanlinear_forward(xc, p) * w.double()).sum().backward()
    assert_grad_close(xg.grad, xc.grad, "x", rel=1e-4)
    for n, q in m.named_parameters():
        assert_grad_close(q.grad, ps[n].grad, n, rel=1e-4)


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
    with F.closure_fusion(use_autonomous):   # the closure stage by stage (HIP VJPs per stage)
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


# ---------------------------------------------------------------------------------------------
# fused training path: one forward launch with a tape + one reverse-sweep launch
# (fetode_integrate_fixed_backward) — checked against the oracle's autograd and against the
# per-stage GPU path (every stage through the per-module HIP VJPs)
# ---------------------------------------------------------------------------------------------

def _fused_and_oracle(dev, kind, method, t, y0, target, step_size=None, dtype=torch.float64):
    """(loss, grads) of the fused GPU path and of the oracle autograd in `dtype`."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
    sd = golden_sd(g)
    m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    opts = None if step_size is None else {"step_size": step_size}
    y0g = y0.clone().to(dev).requires_grad_(True)
    pred = F.odeint(F.autonomous(m), y0g, t, method=method, options=opts)
    loss = torch.mean(torch.square(pred[:, 0, :] - target.to(dev)))
    loss.backward()
    got = {"y0": y0g.grad.cpu()}
    got.update({n: p.grad.cpu() for n, p in m.named_parameters()})
    skip = ("grid", "prev_x", "branch_sign")
    ps = {k: v.clone().to(dtype).requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
    if kind == "kanfet":
        ref = O.KANFETRef.from_state_dict(ps, 2)
    else:
        ref = O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)])
    y0c = y0.clone().to(dtype).requires_grad_(True)
    pr = O.odeint(lambda tt, yy: ref(yy), y0c, t, method=method, options=opts)
    lref = torch.mean(torch.square(pr[:, 0, :] - target.to(dtype)))
    lref.backward()
    exp = {"y0": y0c.grad}
    exp.update({n: ps[n].grad for n in got if n != "y0"})
    return loss.item(), got, lref.item(), exp


@pytest.mark.parametrize("method", ["rk4", "rk4_classic", "midpoint", "euler"])
def test_fused_backward_kan_vs_oracle_fp64(dev, method):
    """KAN field (well conditioned): every gradient within 1e-4 of fp64 autograd, 35 points."""
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    t = torch.from_numpy(g["t35"])
    y0 = O.lv_y0(64, seed=3)
    target = torch.from_numpy(load_golden("lv_lsoda")["soln"][:35]).float()
    loss, got, lref, exp = _fused_and_oracle(dev, "kan", method, t, y0, target)
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    for n in got:
        assert_grad_close(got[n], exp[n], n, rel=1e-4)


@pytest.mark.parametrize("small", [True, False], ids=["v6-tape", "v4-tape"])
@pytest.mark.parametrize("method", ["rk4", "rk4_classic", "midpoint", "euler"])
def test_fused_backward_kanfet_vs_oracle_fp64(dev, bwd_split, kernel_switch, small, method):
    """KAN-FET, 6 points (short enough to be well conditioned in fp32), B=16, every method; the
    taped forward on v6 (the default at this batch) and on v4 (fetode_fused_set_small_batch_max(0))."""
    kernel_switch(small)
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    t = torch.from_numpy(g["t35"])[:6]
    y0 = O.lv_y0(16, seed=5)
    target = torch.zeros(6, 2)
    loss, got, lref, exp = _fused_and_oracle(dev, "kanfet", method, t, y0, target)
    assert abs(loss - lref) <= 1e-4 * abs(lref)
    for n in got:
        assert_grad_close(got[n], exp[n], n, rel=1e-3)


def test_fused_backward_interpolated_outputs_and_reversed_time(dev, bwd_split):
    """step_size grid with outputs between grid points (linear interpolation adjoint) and a
    decreasing t (sign-flipped steps)."""
    from oracle import torch_ref as O
    y0 = O.lv_y0(8, seed=7)
    target = torch.ones(5, 2)
    # KAN field over 1.4 time units; KAN-FET only over 0.45 (its fp32 gradients drift from fp64
    # by ~4% over 1.4: the CPU oracle's own fp32 autograd gives 88.0 vs 91.3 on y0 there)
    t = torch.tensor([0.0, 0.33, 0.5, 1.07, 1.4], dtype=torch.float64)
    loss, got, lref, exp = _fused_and_oracle(dev, "kan", "rk4", t, y0, target, step_size=0.1)
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    for n in got:
        assert_grad_close(got[n], exp[n], n, rel=1e-4)
    ts = torch.tensor([0.0, 0.13, 0.2, 0.37, 0.45], dtype=torch.float64)
    loss, got, lref, exp = _fused_and_oracle(dev, "kanfet", "rk4", ts, y0, target, step_size=0.1)
    assert abs(loss - lref) <= 1e-4 * abs(lref)
    for n in got:
        assert_grad_close(got[n], exp[n], n, rel=1e-3)
    tr = torch.flip(t, [0])
    loss, got, lref, exp = _fused_and_oracle(dev, "kan", "rk4", tr, y0, target)
    assert abs(loss - lref) <= 1e-5 * abs(lref)
    for n in got:
        assert_grad_close(got[n], exp[n], n, rel=1e-4)


def test_fused_backward_first_call_rules(dev, bwd_split):
    """B=1 fresh module (prev_x = zeros, dx = x) and B>1 fresh (dx = 0) as the backward's
    evaluation 0 (ferro_class.py:373-375), and a second solve that starts from the stored state."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])[:4]
    for B in (1, 5):
        m = F.KANFET([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        skip = ("grid", "prev_x", "branch_sign")
        ps = {k: v.clone().double().requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
        ref = O.KANFETRef.from_state_dict(ps, 2)
        y0 = O.lv_y0(B, seed=11)
        for call in range(2):  # second call: hysteresis state carried over from the first solve
            m.zero_grad()
            for p in ps.values():
                p.grad = None
            yg = y0.clone().to(dev).requires_grad_(True)
            F.odeint(F.autonomous(m), yg, t, method="rk4").square().sum().backward()
            yc = y0.clone().double().requires_grad_(True)
            O.odeint(lambda tt, yy: ref(yy), yc, t, method="rk4").square().sum().backward()
            # call 1 starts from the carried state; one B=5 trajectory's gradient is sensitive to the
            # fp32 rounding of that state (measured vs fp64: fused 2.1e-3, per-stage GPU path 3.3e-3
            # relative).  A wrong first-call rule is an O(1) change, far above either bound.
            rel = 1e-3 if call == 0 else 1e-2
            assert_grad_close(yg.grad, yc.grad, f"B={B} call={call} y0", rel=rel)
            for n, p in m.named_parameters():
                assert_grad_close(p.grad, ps[n].grad, f"B={B} call={call} {n}", rel=rel)


@pytest.mark.parametrize("kind,npts", [("kan", 35)])
def test_small_batch_tape_matches_v4(dev, kernel_switch, kind, npts):
    """At B <= small_max the taped training forward runs on v6 (small6_kernel<..., TAPE>); forcing
    the v4 kernel (fetode_fused_set_small_batch_max(0)) gives the same tape up to the two kernels'
    summation orders (tools/diag/tape_diff.py: 5.7e-6 absolute on the KAN field).  A loss over EVERY
    trajectory and output time (sum(w * sol)) makes the gradient as ill-conditioned as the batch's
    worst trajectory (d loss / d y0 up to ~2e3 here), so both are held to the fp64 oracle's autograd
    with the reference's own fp32 autograd as the yardstick: |gpu - fp64| <= 4 |ref fp32 - fp64| +
    1e-5 scale for the KAN field, every fixed-grid method, and the loss likewise.  (KAN-FET: an
    all-trajectory loss only measures the hysteresis' fp32 chaos — tools/diag/tape_grad_check.py
    finds v6, v4 and the reference's own fp32 each 1e-3 .. 5e-2 from fp64, tensor by tensor; both
    kernels take the short-horizon oracle test below, test_fused_backward_kanfet_vs_oracle_fp64.)"""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kanfet" if kind == "kanfet" else "traj_kan")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])[:npts]
    y0 = O.lv_y0(64, seed=9)
    w = torch.randn(npts, 64, 2, generator=torch.Generator().manual_seed(6))
    skip = ("grid", "prev_x", "branch_sign")
    for method in ["rk4", "rk4_classic", "midpoint", "euler"]:
        ref = {}
        for dt in (torch.float32, torch.float64):
            ps = {k: v.clone().to(dt).requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
            r = (O.KANFETRef.from_state_dict(ps, 2) if kind == "kanfet"
                 else O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)]))
            yc = y0.clone().to(dt).requires_grad_(True)
            lo = (O.odeint(lambda tt, yy: r(yy), yc, t, method=method) * w.to(dt)).sum()
            lo.backward()
            ref[dt] = (lo.item(), {"y0": yc.grad, **{n: ps[n].grad for n in ps if ps[n].grad is not None}})
        l64, g64 = ref[torch.float64]
        l32, g32 = ref[torch.float32]
        for small in (True, False):
            kernel_switch(small)
            m = (F.KANFET if kind == "kanfet" else F.KAN)([2, 10, 2], grid_size=5)
            m.load_state_dict(sd)
            m = m.to(dev)
            yg = y0.clone().to(dev).requires_grad_(True)
            loss = (F.odeint(F.autonomous(m), yg, t, method=method) * w.to(dev)).sum()
            loss.backward()
            got = {"y0": yg.grad.cpu(), **{n: p.grad.cpu() for n, p in m.named_parameters()}}
            tag = f"{method} {'v6' if small else 'v4'}"
            assert abs(loss.item() - l64) <= 4 * abs(l32 - l64) + 1e-5 * abs(l64), (tag, loss.item(), l32, l64)
            ratios = []
            for n in got:
                e64, e32, gg = g64[n].double(), g32[n].double(), got[n].double()
                scale = e64.abs().max().item() + 1e-12
                err = (gg - e64).abs().max().item()
                spread = (e32 - e64).abs().max().item() + 1e-5 * scale
                ratios.append(err / spread)
                if kind == "kan":
                    assert err <= 4 * spread, f"{tag} {n}: |gpu-fp64|={err:.3e} ref32 {spread:.3e}"



def test_fused_backward_matches_per_stage_path_large_batch(dev):
    """B=4096, the bench horizon (34 rk4 steps), KAN field: the fused reverse sweep and the
    per-stage path (autograd through every stage, per-module HIP VJPs) agree within 1e-4."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])
    y0 = O.lv_y0(4096, seed=0).to(dev)
    w = torch.randn(35, 4096, 2, generator=torch.Generator().manual_seed(4)).to(dev)
    res = []
    for fused in (True, False):
        m = F.KAN([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        prev = F.set_fused_training(fused)
        try:
            yg = y0.clone().requires_grad_(True)
            (F.odeint(F.autonomous(m), yg, t, method="rk4") * w).sum().backward()
        finally:
            F.set_fused_training(prev)
        res.append({"y0": yg.grad.cpu(), **{n: p.grad.cpu() for n, p in m.named_parameters()}})
    for n in res[0]:
        assert_grad_close(res[0][n], res[1][n], n, rel=1e-4)


@pytest.mark.parametrize("B", [4096, 777])
def test_lane_sweep_matches_one_kernel_bench_horizon(dev, B):
    """KAN-FET, the bench horizon (34 rk4 steps), the bench loss: the lane-group sweep + KAN sums
    (fetode_backward_set_v7(2)) against the one-kernel sweep (mode 0) — the same VJP algebra in a
    different lane map and summation order; B = 777 leaves the last wave half empty."""
    import fet_ode_amd as F
    from fet_ode_amd import _lib
    from oracle import torch_ref as O
    lib = _lib.load()
    sd = golden_sd(load_golden("traj_kanfet"))
    t = torch.from_numpy(load_golden("traj_kanfet")["t35"])
    y0 = O.lv_y0(B, seed=1).to(dev)
    res = []
    prev = lib.fetode_backward_set_v7(-1)
    try:
        for mode in (0, 2, 6):   # one kernel; the lane sweep; the lane sweep + kansum_kernel
            lib.fetode_backward_set_v7(mode)
            m = F.KANFET([2, 10, 2], grid_size=5)
            m.load_state_dict(sd)
            m = m.to(dev)
            yg = y0.clone().requires_grad_(True)
            F.odeint(F.autonomous(m), yg, t, method="rk4").square().mean().backward()
            res.append({"y0": yg.grad.cpu(), **{n: p.grad.cpu() for n, p in m.named_parameters()}})
    finally:
        lib.fetode_backward_set_v7(prev)
    for n in res[0]:
        assert_grad_close(res[1][n], res[0][n], n, rel=1e-4)
        assert_grad_close(res[2][n], res[0][n], n + " (kansum)", rel=1e-4)


def test_lane_sweep_off_grid_inputs(dev):
    """Initial states spread over [-4, 4] (the knots span [-2.2, 2.2]): both layers' inputs leave the
    grid on many trajectories, so the lane sweep's out-of-grid branches (zero bases, the spline
    table's zero row, the layer-0 interval from the wave ballot) run; held to the one-kernel sweep
    within 1e-4 over 5 rk4 steps, and over one step (where the reference's own fp32 autograd is within
    7.5e-4 of fp64; over 5 steps these wild states put it 26 % away) to the fp64 oracle with the
    reference's fp32 error as the yardstick: |gpu - fp64| <= 4 |ref fp32 - fp64| + 1e-4 scale (both
    sweeps measure the same errors here, at most 3.7x the reference's on layers.0.ferro.Ec —
    tools/diag/offgrid_diag.py, profiles/r05_offgrid.log — the fp32 tape of the fused forward)."""
    import fet_ode_amd as F
    from fet_ode_amd import _lib
    from oracle import torch_ref as O
    lib = _lib.load()
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    y0 = (torch.rand(2048, 2, generator=torch.Generator().manual_seed(8), dtype=torch.float64) * 8 - 4).float()
    skip = ("grid", "prev_x", "branch_sign")

    def gpu(mode, t):
        lib.fetode_backward_set_v7(mode)
        m = F.KANFET([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        yg = y0.clone().to(dev).requires_grad_(True)
        F.odeint(F.autonomous(m), yg, t, method="rk4").square().mean().backward()
        return {"y0": yg.grad.cpu(), **{n: p.grad.cpu() for n, p in m.named_parameters()}}

    def oracle(dt, t):
        ps = {k: v.clone().to(dt).requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
        ref = O.KANFETRef.from_state_dict(ps, 2)
        yc = y0.clone().to(dt).requires_grad_(True)
        O.odeint(lambda tt, yy: ref(yy), yc, t, method="rk4").square().mean().backward()
        return {"y0": yc.grad.double(), **{n: ps[n].grad.double() for n in ps if ps[n].grad is not None}}

    prev = lib.fetode_backward_set_v7(-1)
    try:
        t6 = torch.from_numpy(g["t35"])[:6]
        one, lane = gpu(0, t6), gpu(2, t6)
        t2 = torch.from_numpy(g["t35"])[:2]
        lane2 = gpu(2, t2)
    finally:
        lib.fetode_backward_set_v7(prev)
    for n in one:
        assert_grad_close(lane[n], one[n], n, rel=1e-4)
    e64, e32 = oracle(torch.float64, t2), oracle(torch.float32, t2)
    for n in e64:
        scale = e64[n].abs().max().item()
        err = (lane2[n].double() - e64[n]).abs().max().item()
        yard = (e32[n] - e64[n]).abs().max().item()
        assert err <= 4 * yard + 1e-4 * scale, f"{n}: |gpu-fp64|={err:.3e} ref32 {yard:.3e} scale {scale:.3e}"


def test_one_trajectory_per_wave_tape(dev):
    """B = 777 (inside the one-trajectory-per-wave range, fetode_fused_set_tpw1_range): the taped
    training forward on that kernel against the fp64 oracle's autograd with the reference's own
    fp32 error as the yardstick (|gpu - fp64| <= 4 |ref fp32 - fp64| + 1e-4 scale), and the
    two-per-wave kernel likewise, over one rk4 step (this batch's KAN-FET trajectories part from
    fp64 within a few steps in any fp32 implementation: over 5 steps the two kernels' y0 gradients
    are 21 % and 510 % from fp64, tools/diag/tape_cmp.py)."""
    import fet_ode_amd as F
    from fet_ode_amd import _lib
    from oracle import torch_ref as O
    lib = _lib.load()
    g = load_golden("traj_kanfet")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])[:2]
    y0 = O.lv_y0(777, seed=4)
    skip = ("grid", "prev_x", "branch_sign")

    def oracle(dt):
        ps = {k: v.clone().to(dt).requires_grad_(k.split(".")[-1] not in skip) for k, v in sd.items()}
        ref = O.KANFETRef.from_state_dict(ps, 2)
        yc = y0.clone().to(dt).requires_grad_(True)
        O.odeint(lambda tt, yy: ref(yy), yc, t, method="rk4").square().mean().backward()
        return {"y0": yc.grad.double(), **{n: ps[n].grad.double() for n in ps if ps[n].grad is not None}}

    e64, e32 = oracle(torch.float64), oracle(torch.float32)
    from conftest import fused_ranges
    with fused_ranges() as fr:
        for hi in (1 << 40, 0):
            fr.set(tpw1=(0, hi))
            m = F.KANFET([2, 10, 2], grid_size=5)
            m.load_state_dict(sd)
            m = m.to(dev)
            yg = y0.clone().to(dev).requires_grad_(True)
            F.odeint(F.autonomous(m), yg, t, method="rk4").square().mean().backward()
            got = {"y0": yg.grad.cpu().double(), **{n: p.grad.cpu().double() for n, p in m.named_parameters()}}
            for n in e64:
                scale = e64[n].abs().max().item()
                err = (got[n] - e64[n]).abs().max().item()
                yard = (e32[n] - e64[n]).abs().max().item()
                assert err <= 4 * yard + 1e-4 * scale, f"hi={hi} {n}: |gpu-fp64|={err:.3e} ref32 {yard:.3e}"


def test_fused_backward_deterministic(dev, bwd_split):
    """Two identical training solves give bitwise-identical gradients (fixed-order reductions)."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    sd = golden_sd(load_golden("traj_kanfet"))
    t = torch.from_numpy(load_golden("traj_kanfet")["t35"])
    y0 = O.lv_y0(1024, seed=2).to(dev)
    out = []
    for _ in range(2):
        m = F.KANFET([2, 10, 2], grid_size=5)
        m.load_state_dict(sd)
        m = m.to(dev)
        F.odeint(F.autonomous(m), y0, t, method="rk4").square().mean().backward()
        out.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("resident", [False, True], ids=["host-autograd", "resident-sweep"])
def test_training_grads_through_dopri5_kan(dev, resident):
    """predator_prey.py:139-145 trains through torchodeint's default dopri5: loss.backward()
    through the GPU dopri5 (every stage of every attempt, the error ratios and the step sizes,
    as torchdiffeq's direct backprop) against the oracle's autograd through the same solve.
    The gradient through the step-size control is ill-conditioned in fp32 (the oracle's own fp32
    and fp64 gradients differ by up to 9 % on the spline scalers here), so the bound is the fp64
    oracle with 4x the oracle's own fp32 error, plus 1e-4 relative."""
    import fet_ode_amd as F
    from fet_ode_amd import dopri5 as D5
    from oracle import torch_ref as O
    g = load_golden("traj_kan")
    sd = golden_sd(g)
    t = torch.from_numpy(g["t35"])[:12]
    y0 = torch.tensor([[1.0, 1.0], [0.7, 1.9]])
    target = torch.from_numpy(load_golden("lv_lsoda")["soln"][:12]).float()
    m = F.KAN([2, 10, 2], grid_size=5)
    m.load_state_dict(sd)
    m = m.to(dev)
    y0g = y0.clone().to(dev).requires_grad_(True)
    prev = D5.set_resident_dopri5_training(resident)   # _Dopri5Grad, or the taped solve + sweep (§4.10)
    try:
        pred = F.odeint(lambda tt, yy: m(yy), y0g, t, rtol=1e-5, atol=1e-7)
    finally:
        D5.set_resident_dopri5_training(prev)
    assert isinstance(D5.dopri5_solve.last, D5.ResidentSolve if resident else D5._Dopri5Grad)
    loss = torch.mean(torch.square(pred[:, 0, :] - target.to(dev)))
    loss.backward()
    ref = {}
    for dt in (torch.float32, torch.float64):
        ps = {k: v.clone().to(dt).requires_grad_(k.split(".")[-1] != "grid") for k, v in sd.items()}
        kan = O.KANRef([O.KANLinearParams.from_state_dict(ps, f"layers.{l}.") for l in range(2)])
        y0c = y0.clone().to(dt).requires_grad_(True)
        tr = O.Dopri5Trace()
        pr = O.odeint(lambda tt, yy: kan(yy), y0c, t, rtol=1e-5, atol=1e-7, trace=tr)
        lref = torch.mean(torch.square(pr[:, 0, :] - target.to(dt)))
        lref.backward()
        ref[dt] = (lref.detach(), y0c.grad, {k: v.grad for k, v in ps.items() if v.grad is not None}, tr)
    last = D5.dopri5_solve.last
    tr = ref[torch.float32][3]
    assert len(last.attempts) == len(tr.attempts) and [a[3] for a in last.attempts] == [a[3] for a in tr.attempts]

    def env(got, e32, e64, name):
        got, e32, e64 = got.detach().double().cpu(), e32.double(), e64.double()
        scale = e64.abs().max().item() + 1e-12
        err, spread = (got - e64).abs().max().item(), (e32 - e64).abs().max().item()
        assert err <= 4 * spread + 1e-4 * scale, f"{name}: |gpu-fp64|={err:.3e} fp32 spread={spread:.3e} scale={scale:.3e}"

    env(loss, ref[torch.float32][0], ref[torch.float64][0], "loss")
    env(y0g.grad, ref[torch.float32][1], ref[torch.float64][1], "y0")
    for n, p in m.named_parameters():
        env(p.grad, ref[torch.float32][2][n], ref[torch.float64][2][n], n)


def test_fused_solve_follows_fused_adam_steps(dev):
    """torch.optim.Adam(fused=True) updates parameters without bumping version counters; the
    cached descriptor / plan must still follow every step (_lib.param_generation): after each
    step the fused solve equals a solve of a fresh copy of the model with the stepped weights."""
    import fet_ode_amd as F
    from oracle import torch_ref as O
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    y0 = O.lv_y0(64).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    opt = torch.optim.Adam(m.parameters(), lr=1e-2, fused=True)
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        m.reset_state()
        F.odeint(F.autonomous(m), y0, t, method="rk4").square().mean().backward()
        opt.step()
        fresh = F.KANFET([2, 10, 2], grid_size=5).to(dev)
        fresh.load_state_dict(m.state_dict())
        with torch.no_grad():
            m.reset_state()
            fresh.reset_state()
            a = F.odeint(F.autonomous(m), y0, t, method="rk4")
            b = F.odeint(F.autonomous(fresh), y0, t, method="rk4")
        assert torch.equal(a, b)


@pytest.mark.parametrize("set_to_none", [False, True])
def test_captured_training_step_matches_eager(dev, set_to_none):
    """fet_ode_amd.training.CapturedStep: the whole iteration (fused solve with tape, MSE, the
    reverse sweep, the gradient reduction, fused capturable Adam) as one HIP graph; after the
    constructor's warm-up iterations and k replays the parameters are bitwise those of the same
    number of eager iterations (every replay re-packs the plan from the updated parameters)."""
    import copy

    import fet_ode_amd as F
    from fet_ode_amd.training import CapturedStep
    torch.manual_seed(3)
    base = F.KANFET([2, 10, 2], grid_size=5)
    g = torch.Generator().manual_seed(1)
    y0 = (0.5 + 2.5 * torch.rand(512, 2, generator=g)).to(dev)
    t = torch.linspace(0.0, 0.7, 8, dtype=torch.float64)
    target = torch.zeros(8, 512, 2, device=dev)

    def make():
        m = copy.deepcopy(base).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, fused=True, capturable=True)
        func = F.autonomous(m)

        def it():
            opt.zero_grad(set_to_none=set_to_none)
            loss = (F.odeint(func, y0, t, method="rk4") - target).square().mean()
            loss.backward()
            opt.step()
            return loss
        return m, it

    m_e, it_e = make()
    m_g, it_g = make()
    warm, k = 2, 3
    step = CapturedStep(it_g, warmup=warm, device=dev)
    losses = []
    for _ in range(k):
        losses.append(step().clone())
    for _ in range(warm + k):
        le = it_e()
    torch.cuda.synchronize(dev)
    assert torch.equal(losses[-1], le)
    for (n, a), b in zip(m_g.named_parameters(), m_e.parameters()):
        assert torch.equal(a, b), n
    assert not torch.equal(losses[0], losses[-1])   # the replays did train
