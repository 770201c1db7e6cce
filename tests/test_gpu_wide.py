"""MI355X parity at the PRODUCTION widths of BASELINE configs[3] (train_kan_fet_ett.py:136-197 with
the KAN-FET latent field KANFET([64, 128, 64], K = 10)): the kernels the ETT workload runs —
wide KANLinear (every outputs-per-wave variant the launcher picks by batch size), the wide Ferro
forward (K = 10 / 12 templated and a generic K) and the whole field — against oracle/torch_ref.py.

Edge cases the product-form coercive sigmoids must survive (ferro_class.py:390-391): rows with
|gate_slope * x| > 80 mixed into a batch of normal rows, and parameters with |gate_slope * Ec| > 80
(e^{gs Ec} would overflow / underflow in fp32)."""
import pytest
import torch

import fet_ode_amd as F
from fet_ode_amd import ett
from oracle import ett_ref as E
from oracle import torch_ref as O

pytestmark = pytest.mark.gpu


def row_rel(got, exp):
    """max over rows of ||got_b - exp_b|| / ||exp_b||."""
    got, exp = got.double().cpu(), exp.double().cpu()
    return ((got - exp).norm(dim=-1) / exp.norm(dim=-1).clamp_min(1e-30)).max().item()


def _x(B, n, seed, wild_rows=()):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, n, generator=g) * 6 - 3          # in and out of the [-2.2, 2.2) knot grid
    for r in wild_rows:                                  # |gs x| > 80 (gs = 10): the direct-form rows
        x[r] = torch.sign(torch.randn(n, generator=g)) * (8.2 + torch.rand(n, generator=g) * 3)
    return x


@pytest.mark.parametrize("i,o", [(64, 128), (128, 64)])
@pytest.mark.parametrize("B", [300, 4096, 8192, 16384])
def test_wide_kanlinear_forward(dev, i, o, B):
    """KANLinear at ETT widths; B sweeps the launcher's outputs-per-wave choice (1/2/4/8)."""
    torch.manual_seed(i + o)
    m = F.KANLinear(i, o)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    x = _x(B, i, seed=B)
    with torch.no_grad():
        got = m(x.to(dev))
    exp = O.kanlinear_forward(x, O.KANLinearParams.from_state_dict(sd))
    assert row_rel(got, exp) <= 1e-5, row_rel(got, exp)


def _ferro_with_edges(i, o, K, seed):
    torch.manual_seed(seed)
    m = F.FerroelectricBasis(i, o, K)
    with torch.no_grad():                        # a trained Ec can leave [0.5, 2.5]: |gs Ec| > 80 and < 0
        m.Ec[0, :, 0] = 9.5
        m.Ec[1, :, 1] = -9.0
        m.Ec[2, 3, :] = -0.3
    return m


@pytest.mark.parametrize("i,o,K", [(64, 128, 10), (128, 64, 10), (64, 128, 12), (48, 40, 7)])
def test_wide_ferro_forward_sequence(dev, i, o, K):
    """Three stateful calls (first-call rule dx = 0, then dx = x - prev_x) of a B = 300 batch with
    wild rows; each against the fp32 oracle (1e-5 per row) and the fp64 oracle (within 4x the fp32
    oracle's own error + 1e-6)."""
    m = _ferro_with_edges(i, o, K, seed=i * o + K)
    p = O.FerroParams(*(getattr(m, n).detach().clone() for n in ("k", "Ec", "Ps", "bias", "coef")))
    st32, st64 = O.FerroState(i, o, K), O.FerroState(i, o, K, torch.float64)
    p64 = p.to(torch.float64)
    m = m.to(dev)
    B = 300
    for call in range(3):
        x = _x(B, i, seed=100 * call + i, wild_rows=(5, 77, 140, 299)) * (1.0 + 0.05 * call)
        with torch.no_grad():
            got = m(x.to(dev))
        e32 = O.ferro_forward(x, p, st32)
        e64 = O.ferro_forward(x.double(), p64, st64)
        assert torch.isfinite(got).all()
        assert row_rel(got, e32) <= 1e-5, (call, row_rel(got, e32))
        err = row_rel(got, e64)
        assert err <= 4 * row_rel(e32, e64) + 1e-6, (call, err, row_rel(e32, e64))
        assert torch.equal(m.prev_x[:, :, 0, 0].cpu(), x)


def test_wide_kanfet_field_calls(dev):
    """KANFET([64, 128, 64], K = 10) — the ETT latent field — two stateful evaluations."""
    torch.manual_seed(5)
    m = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    ref = O.KANFETRef.from_state_dict(sd, 2)
    for call in range(2):
        x = _x(300, 64, seed=11 + call, wild_rows=(0, 150) if call else ())
        with torch.no_grad():
            got = m(x.to(dev))
        assert row_rel(got, ref(x)) <= 1e-5, (call, row_rel(got, ref(x)))


def test_ett_field_through_odeint_rk4_production_width(dev):
    """The config-4 latent ODE itself: ett.KANFETDynamics(64, hidden=128, K=10) through odeint_rk4
    (classic RK4 with substeps, train_kan_fet_ett.py:51-83) at B = 256 against the oracle, with the
    reference's own fp32 error as the yardstick (KAN-FET hysteresis is ill-conditioned in fp32)."""
    torch.manual_seed(9)
    dyn = ett.KANFETDynamics(64, hidden=128, num_fet_basis=10)
    sd = {k: v.clone() for k, v in dyn.net.state_dict().items()}
    dyn = dyn.to(dev)
    g = torch.Generator().manual_seed(10)
    z0 = torch.randn(256, 64, generator=g) * 0.8
    t = torch.linspace(0.0, 0.25, steps=2)
    with torch.no_grad():
        got = ett.odeint_rk4(dyn, z0.to(dev), t.to(dev), n_substeps=2).cpu()
    r32 = O.KANFETRef.from_state_dict(sd, 2)
    r64 = O.KANFETRef.from_state_dict({k: v.double() for k, v in sd.items()}, 2)
    e32 = E.odeint_rk4(lambda tt, zz: r32(zz), z0, t, n_substeps=2)
    e64 = E.odeint_rk4(lambda tt, zz: r64(zz), z0.double(), t.double(), n_substeps=2)
    assert got.shape == (2, 256, 64) and torch.isfinite(got).all()
    spread = row_rel(e32[1], e64[1])
    err = row_rel(got[1], e64[1])
    assert err <= 4 * spread + 1e-5, (err, spread)
    # the hysteresis state after the solve is the last stage input of each layer (ferro_class.py:409)
    assert dyn.net.layers[0].ferro.prev_x.shape == (256, 64, 128, 10)


# ---------------------------------------------------------------------------------------------
# the autograd path at production widths: under autograd the layers run the generic wide kernels
# (kanlinear_fwd_wave_kernel with its OB variants, ferro_fwd_wide_kernel<10>) and their VJPs —
# what training the config-4 forecaster executes
# ---------------------------------------------------------------------------------------------

@pytest.mark.parametrize("i,o", [(64, 128), (128, 64)])
@pytest.mark.parametrize("B", [256, 4096])
def test_wide_kanlinear_autograd_forward_and_grads(dev, i, o, B):
    """KANLinear forward + every parameter gradient and d x under autograd vs the oracle's
    autograd (B sweeps the OB = 8 / 2 launcher choice)."""
    torch.manual_seed(i * 3 + o + B)
    m = F.KANLinear(i, o)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    x = _x(B, i, seed=B + 1)
    w = torch.randn(B, o, generator=torch.Generator().manual_seed(B + 2))
    xg = x.to(dev).requires_grad_(True)
    got = m(xg)
    (got * w.to(dev)).sum().backward()
    p = O.KANLinearParams.from_state_dict(sd)
    field_of = {"base_weight": "base_weight", "spline_weight": "spline_weight", "spline_scaler": "spline_scaler",
                "logistic_basis.a": "a", "logistic_basis.b": "b", "logistic_weight": "logistic_weight",
                "logistic_scaler": "logistic_scaler"}
    ps = {}
    for name, f in field_of.items():
        v = getattr(p, f)
        if v is not None:
            ps[name] = v.clone().requires_grad_(True)
            setattr(p, f, ps[name])
    xr = x.clone().requires_grad_(True)
    exp = O.kanlinear_forward(xr, p)
    (exp * w).sum().backward()
    assert row_rel(got.detach(), exp.detach()) <= 1e-5
    gx = (xg.grad.cpu() - xr.grad).abs().max().item()
    assert gx <= 1e-4 * xr.grad.abs().max().item(), gx
    checked = 0
    for name, t in m.named_parameters():
        ref = ps.get(name)
        if ref is None or ref.grad is None:
            continue
        err = (t.grad.cpu() - ref.grad).abs().max().item()
        assert err <= 2e-4 * ref.grad.abs().max().item() + 1e-7, (name, err)
        checked += 1
    assert checked >= 6, checked


@pytest.mark.parametrize("i,o", [(64, 128), (128, 64)])
def test_wide_ferro_autograd_sequence_and_grads(dev, i, o):
    """FerroelectricBasis(K = 10) under autograd — the generic wide forward with wild rows and
    |gs Ec| > 80 parameters, two stateful calls — and the parameter / input gradients of the
    second call vs the oracle's autograd."""
    m = _ferro_with_edges(i, o, 10, seed=7 * i + o)
    names = ("k", "Ec", "Ps", "bias", "coef")
    p0 = [getattr(m, n).detach().clone() for n in names]
    m = m.to(dev)
    st = O.FerroState(i, o, 10)
    B = 300
    x1 = _x(B, i, seed=5, wild_rows=(3, 200))
    x2 = _x(B, i, seed=6) * 0.9
    w = torch.randn(B, o, generator=torch.Generator().manual_seed(8))
    with torch.no_grad():
        m(x1.to(dev))
    O.ferro_forward(x1, O.FerroParams(*p0), st)
    xg = x2.to(dev).requires_grad_(True)
    got = m(xg)
    (got * w.to(dev)).sum().backward()
    pr = [t.clone().requires_grad_(True) for t in p0]
    xr = x2.clone().requires_grad_(True)
    exp = O.ferro_forward(xr, O.FerroParams(*pr), st)
    (exp * w).sum().backward()
    assert row_rel(got.detach(), exp.detach()) <= 1e-5
    gx = (xg.grad.cpu() - xr.grad).abs().max().item()
    assert gx <= 2e-4 * xr.grad.abs().max().item(), gx
    for n, r in zip(names, pr):
        g = getattr(m, n).grad.cpu()
        err = (g - r.grad).abs().max().item()
        assert err <= 2e-4 * r.grad.abs().max().item() + 1e-7, (n, err)


# ---------------------------------------------------------------------------------------------
# the ETT bench batch itself (B = 8192): layer 0 (64 -> 128) launches 1 024 tiles and takes the
# nslice = 1 branch of wide_layer_kernel<10, true, true, 8> (fetode_wide.hip wide_layer_forward);
# layer 1 (128 -> 64) has 512 tiles and takes nslice = 2.  The oracle runs on a subset of rows
# (rows are independent given their own prev_x; a subset of B > 1 rows keeps the first-call rule).
# ---------------------------------------------------------------------------------------------

def test_wide_kanfet_field_b8192_both_slice_branches(dev):
    """KANFET([64, 128, 64], K = 10) at B = 8192, three stateful evaluations, with |gs x| > 80
    rows and |gs Ec| > 80 parameters in both layers: 1e-5 per row against the fp32 oracle on 640
    rows (the wild rows, rows at both ends of every 64-row tile, and a random sample)."""
    torch.manual_seed(81)
    m = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10)
    with torch.no_grad():
        for fer in (m.layers[0].ferro, m.layers[1].ferro):
            fer.Ec[0, :, 0] = 9.5
            fer.Ec[1, :, 1] = -9.0
            fer.Ec[2, 3, :] = -0.3
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    B = 8192
    wild = (5, 63, 64, 4095, 4096, 8191)
    g = torch.Generator().manual_seed(82)
    rows = torch.cat([torch.tensor(wild), torch.arange(0, B, 64), torch.arange(63, B, 64),
                      torch.randperm(B, generator=g)[:256]]).unique()
    ref = O.KANFETRef.from_state_dict(sd, 2)
    for call in range(3):
        x = _x(B, 64, seed=8192 + call, wild_rows=wild if call != 1 else ()) * (1.0 + 0.1 * call)
        with torch.no_grad():
            got = m(x.to(dev))
        exp = ref(x[rows])
        assert torch.isfinite(got).all()
        err = row_rel(got.cpu()[rows], exp)
        assert err <= 1e-5, (call, err)
        assert torch.equal(m.layers[0].ferro.prev_x[:, :, 0, 0].cpu(), x)


def test_wide_kanlinear_noncontiguous_input(dev):
    """A column slice of a wider tensor (non-contiguous 2-D view) into a 64 -> 128 KANLinear under
    no_grad (the MFMA wide-layer path) gives the same rows as the autograd path."""
    torch.manual_seed(3)
    m = F.KANLinear(64, 128).to(dev)
    big = _x(1000, 96, seed=4).to(dev)
    xs = big[:, 16:80]
    assert not xs.is_contiguous()
    with torch.no_grad():
        got = m(xs)
    exp = m(xs.clone().requires_grad_(True)).detach()
    assert row_rel(got, exp) <= 1e-5, row_rel(got, exp)


# ---------------------------------------------------------------------------------------------
# the one-pass Ferro VJP at production widths (fetode_ferro_backward_wide) against the generic
# two-kernel VJP (itself pinned to the oracle's autograd above and in test_gpu_grad.py)
# ---------------------------------------------------------------------------------------------

@pytest.mark.parametrize("i,o,K", [(64, 128, 10), (128, 64, 10), (64, 128, 12), (128, 64, 12)])
@pytest.mark.parametrize("B", [300, 5000])
def test_wide_ferro_backward_one_pass(dev, i, o, K, B):
    """d/dx and the five parameter gradients, stateful (prev_x) and first-call (reinit) forms, plain
    and accumulating, with wild rows (|gs x| > 80) and |gs Ec| > 80 parameters (the direct gate);
    B = 5000 spans several row segments.  Run twice: the fixed-order reductions repeat bitwise."""
    from fet_ode_amd import autograd_ops as A
    m = _ferro_with_edges(i, o, K, seed=3 * i + o + K).to(dev)
    x = _x(B, i, seed=B + K, wild_rows=(1, 150, B - 1)).to(dev)
    prev = (_x(B, i, seed=B + K + 1, wild_rows=(2, 150)) * 0.7).to(dev)
    g = torch.randn(B, o, generator=torch.Generator().manual_seed(B + 3)).to(dev)
    want = (True,) * 5
    for reinit in (False, True):
        gx_w, gp_w = A._ferro_backward_wide(m, x, prev, reinit, g, True, want, None)
        gx_r, gp_r = A._ferro_backward_generic(m, x, prev, reinit, None, g, True, want, None)
        gx_w2, gp_w2 = A._ferro_backward_wide(m, x, prev, reinit, g, True, want, None)
        assert torch.equal(gx_w, gx_w2) and all(torch.equal(a, b) for a, b in zip(gp_w, gp_w2))
        assert torch.isfinite(gx_w).all()
        # saturated (wild) rows carry gradients ~1e-5 of the others, where 1 - th^2 loses most of its
        # digits in either fp32 form: those rows are held to the tensor's scale, the rest per row
        tame = torch.ones(B, dtype=torch.bool)
        tame[[1, 150, B - 1]] = False
        assert row_rel(gx_w[tame], gx_r[tame]) <= 2e-5, (reinit, row_rel(gx_w[tame], gx_r[tame]))
        assert (gx_w - gx_r).abs().max().item() <= 2e-5 * gx_r.abs().max().item()
        for n, a, b in zip(A.FERRO_PARAM_NAMES, gp_w, gp_r):
            err = (a - b).abs().max().item()
            assert err <= 1e-4 * b.abs().max().item() + 1e-7, (reinit, n, err)
    # accumulate: d/dx added into an existing buffer, parameter sums from zero
    base = torch.randn(B, i, generator=torch.Generator().manual_seed(9)).to(dev)
    acc = base.clone()
    gx_a, gp_a = A._ferro_backward_wide(m, x, prev, False, g, True, (False, True, False, False, True), acc)
    assert gx_a is acc
    gx_w, gp_w = A._ferro_backward_wide(m, x, prev, False, g, True, want, None)
    assert torch.equal(acc, base + gx_w)            # the same fixed-order sum, added once
    assert gp_a[0] is None and torch.equal(gp_a[1], gp_w[1]) and torch.equal(gp_a[4], gp_w[4])


# the MFMA KANLinear VJP at production widths (fetode_kanlinear_backward_wide) against the generic
# kernels (pinned to the oracle's autograd in test_gpu_grad.py / above)
@pytest.mark.parametrize("i,o", [(64, 128), (128, 64), (128, 128)])
@pytest.mark.parametrize("B", [37, 1000, 9000])
def test_wide_kanlinear_backward_mfma(dev, i, o, B):
    """d/dx and the seven parameter gradients; x in and out of the knot grid (and on a knot), a
    ragged batch (B % 16 != 0), several row segments; plain, accumulating and parameters-only
    forms; run twice: the fixed-order reductions repeat bitwise."""
    from fet_ode_amd import autograd_ops as A
    torch.manual_seed(i + 2 * o + B)
    m = F.KANLinear(i, o).to(dev)
    with torch.no_grad():
        m.spline_scaler.mul_(torch.rand_like(m.spline_scaler) + 0.5)
        m.logistic_scaler.mul_(torch.rand_like(m.logistic_scaler) + 0.5)
    x = _x(B, i, seed=B + i).to(dev)
    x[0, 0] = m.grid[0, 5]                     # exactly on a knot
    x[min(3, B - 1), :] = 40.0                  # far outside the grid
    g = torch.randn(B, o, generator=torch.Generator().manual_seed(B)).to(dev)
    want = tuple(p is not None for p in A.kan_params(m))
    gx_w, gp_w = A._kan_backward_wide(m, x, g, True, want)
    gx_w2, gp_w2 = A._kan_backward_wide(m, x, g, True, want)
    gx_r, gp_r = A._kan_backward_generic(m, x, g, True, want)
    assert torch.equal(gx_w, gx_w2)
    assert all(a is None or torch.equal(a, b) for a, b in zip(gp_w, gp_w2))
    assert row_rel(gx_w, gx_r) <= 1e-5, row_rel(gx_w, gx_r)
    n = 0
    for name, a, b in zip(A.KAN_PARAM_NAMES, gp_w, gp_r):
        if b is None:
            continue
        err = (a - b).abs().max().item()
        assert err <= 2e-5 * b.abs().max().item() + 1e-7, (name, err, b.abs().max().item())
        n += 1
    assert n == 7
    # accumulate into existing d/dx; parameters-only (no d/dx)
    base = torch.randn(B, i, generator=torch.Generator().manual_seed(2)).to(dev)
    acc = base.clone()
    _, gp_a = A._kan_backward_wide(m, x, g, True, want, acc)
    assert torch.equal(acc, base + gx_w)
    assert all(a is None or torch.equal(a, b) for a, b in zip(gp_a, gp_w))
    gx_n, gp_n = A._kan_backward_wide(m, x, g, False, want)
    assert gx_n is None and all(a is None or torch.equal(a, b) for a, b in zip(gp_n, gp_w))


def test_wide_kanfet_field_autograd_two_calls(dev):
    """KANFET([64, 128, 64]) under autograd (the wide-layer forward + the MFMA / one-pass VJPs,
    _WideLayerFn) against the per-module autograd path: two stateful calls (first-call rule, then
    prev_x), loss through both, every parameter gradient and d/dx."""
    from fet_ode_amd import autograd_ops as A
    torch.manual_seed(21)
    base = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10)
    x1 = _x(700, 64, seed=1).to(dev) * 0.5
    x2 = _x(700, 64, seed=2, wild_rows=(9,)).to(dev) * 0.5
    w = torch.randn(700, 64, generator=torch.Generator().manual_seed(3)).to(dev)
    res = []
    for wide in (True, False):
        A._WIDE_GRAD = wide
        try:
            m = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10)
            m.load_state_dict(base.state_dict())
            m = m.to(dev)
            xa = x1.clone().requires_grad_(True)
            xb = x2.clone().requires_grad_(True)
            y1 = m(xa)
            y2 = m(xb)
            ((y1 * w).sum() + (y2 * y2).mean()).backward()
            res.append((y1.detach(), y2.detach(), xa.grad, xb.grad,
                        {n: p.grad.clone() for n, p in m.named_parameters()}))
        finally:
            A._WIDE_GRAD = True
    (a1, a2, ga, gb, pa), (r1, r2, gra, grb, pr) = res
    assert row_rel(a1, r1) <= 1e-5 and row_rel(a2, r2) <= 1e-5
    for got, exp in ((ga, gra), (gb, grb)):
        assert (got - exp).abs().max().item() <= 1e-4 * exp.abs().max().item()
    assert len(pa) == len(pr) and len(pa) >= 20
    for n in pr:
        err = (pa[n] - pr[n]).abs().max().item()
        assert err <= 1e-4 * pr[n].abs().max().item() + 1e-7, (n, err)


def test_wide_field_flat_parameter_gradients(dev):
    """The wide layers' parameter gradients through one flat tensor per layer (_WideLayerFlatFn)
    against the per-parameter _WideLayerFn: two calls per graph; a second graph after an optimizer
    step (the concatenation is rebuilt); two graphs recorded before either backward; a frozen
    parameter (the per-parameter path)."""
    from fet_ode_amd import autograd_ops as A
    torch.manual_seed(23)
    base = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10)
    xs = [_x(300, 64, seed=s).to(dev) * 0.5 for s in (4, 5, 6, 7)]
    w = torch.randn(300, 64, generator=torch.Generator().manual_seed(8)).to(dev)

    def run(flat, freeze=False):
        A._FLAT_GRAD = flat
        try:
            m = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10)
            m.load_state_dict(base.state_dict())
            m = m.to(dev)
            if freeze:
                A.field_layers(m)[0][0].base_weight.requires_grad_(False)
            opt = torch.optim.SGD([p for p in m.parameters() if p.requires_grad], lr=1e-2)
            out = []
            ((m(xs[0]) * w).sum() + m(xs[1]).square().mean()).backward()
            out.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
            if flat and not freeze:
                kan = A.field_layers(m)[0][0]
                assert not kan.__dict__["_fetode_flat"][3][0]   # the backward reached it
            opt.step()
            opt.zero_grad(set_to_none=True)
            l1 = (m(xs[2]) * w).sum()
            l2 = m(xs[3]).square().mean()
            l1.backward()
            out.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
            l2.backward()
            out.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
            return out
        finally:
            A._FLAT_GRAD = True

    for freeze in (False, True):
        got, exp = run(True, freeze), run(False, freeze)
        for g, e in zip(got, exp):
            assert g.keys() == e.keys() and len(e) >= (19 if freeze else 20)
            for n in e:
                err = (g[n] - e[n]).abs().max().item()
                assert err <= 1e-6 * e[n].abs().max().item() + 1e-9, (freeze, n, err)
