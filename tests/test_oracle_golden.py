"""The CPU oracle reproduces the reference bit for bit on every golden fixture
(fixtures generated from the imported reference modules by tests/golden/make_golden.py)."""
import numpy as np
import torch

from conftest import golden_sd, load_golden
from oracle import torch_ref as O


def test_kanlinear_and_bsplines_bitwise():
    for tag in ("kanlinear_2x10", "kanlinear_10x2"):
        g = load_golden(tag)
        p = O.KANLinearParams.from_state_dict(golden_sd(g))
        x = torch.from_numpy(g["x"])
        assert torch.equal(O.kanlinear_forward(x, p), torch.from_numpy(g["y"])), tag
        assert torch.equal(O.b_splines(x, p.grid, 3), torch.from_numpy(g["bases"])), tag


def test_bsplines_edges():
    """Half-open indicator (efficientkan.py:122): x at the last knot or outside -> zeros;
    +-inf and NaN -> NaN (the (x-g)/d * 0 products), exactly as the reference fixture shows."""
    g = O.make_grid(1)
    x = torch.tensor([[-2.2], [2.2], [-3.0], [3.0], [1e30], [2.1999998]])
    b = O.b_splines(x, g, 3)
    assert b[1:5].abs().sum() == 0
    assert b[0].sum() == 0  # at g0 only the order-0 basis is non-zero -> cubic bases vanish
    assert b[5].sum() > 0
    for tag in ("kanlinear_2x10", "kanlinear_10x2"):
        gg = load_golden(tag)
        p = O.KANLinearParams.from_state_dict(golden_sd(gg))
        bo = O.b_splines(torch.from_numpy(gg["x_odd"]), p.grid, 3)
        exp = torch.from_numpy(gg["bases_odd"])
        assert torch.equal(torch.isnan(bo), torch.isnan(exp))
        assert torch.isnan(exp[:3]).all() and (exp[3] == 0).all()


def test_ferro_sequences_bitwise():
    for tag in ("ferro_2x10x10", "ferro_10x2x10"):
        g = load_golden(tag)
        sd = golden_sd(g)
        p = O.FerroParams.from_state_dict(sd)
        st = O.FerroState(*p.k.shape)
        for n in range(g["xs1"].shape[0]):
            y, basis, _ = O.ferro_forward(torch.from_numpy(g["xs1"][n]), p, st, return_activations=True)
            assert torch.equal(y, torch.from_numpy(g["ys1"][n]))
            assert torch.equal(basis, torch.from_numpy(g["basis1"][n]))
            assert torch.equal(st.prev_x[:, :, 0, 0], torch.from_numpy(g["prev1"][n]))
        p2 = O.FerroParams.from_state_dict(golden_sd(g, "sd2/"))
        st2 = O.FerroState(*p2.k.shape)
        for n in range(g["xs5"].shape[0]):
            y = O.ferro_forward(torch.from_numpy(g["xs5"][n]), p2, st2)
            assert torch.equal(y, torch.from_numpy(g["ys5"][n]))
        st2.reset()
        assert torch.equal(O.ferro_forward(torch.from_numpy(g["x_reset"]), p2, st2),
                           torch.from_numpy(g["y_reset"]))


def test_ferro_first_call_rules():
    """ferro_class.py:373-378: B=1 fresh keeps prev_x=0 (dx=x); B>1 fresh re-inits (dx=0)."""
    torch.manual_seed(0)
    p = O.FerroParams(*(torch.rand(2, 3, 4) + 0.5 for _ in range(5)))
    x1 = torch.tensor([[0.3, -0.7]])
    st = O.FerroState(2, 3, 4)
    O.ferro_forward(x1, p, st)
    assert torch.equal(st.prev_x[0, :, 0, 0], x1[0])
    st5 = O.FerroState(2, 3, 4)
    x5 = torch.randn(5, 2)
    a = O.ferro_forward(x5, p, st5)
    st5b = O.FerroState(2, 3, 4)
    st5b.prev_x = x5[:, :, None, None].expand(5, 2, 3, 4).clone()
    st5b.branch_sign = torch.ones(5, 2, 3, 4)
    b = O.ferro_forward(x5, p, st5b)
    assert torch.equal(a, b)


def test_kanfet_field_bitwise_and_grad_fixture_shapes():
    g = load_golden("kanfet_field")
    ref = O.KANFETRef.from_state_dict(golden_sd(g), 2)
    y0 = torch.from_numpy(g["y0"])
    assert torch.equal(ref(y0), torch.from_numpy(g["f1"]))
    assert torch.equal(ref(y0 * 1.01 + 0.05), torch.from_numpy(g["f2"]))
    assert g["grad/x"].shape == (16, 2)
    assert g["grad/layers.0.ferro.k"].shape == (2, 10, 10)


def test_rk4_trajectories_bitwise():
    for name in ("kan", "kanfet"):
        g = load_golden("traj_" + name)
        sd = golden_sd(g)
        for B in (1, 64):
            for tag in ("t35", "t140"):
                if name == "kan":
                    f = O.KANRef([O.KANLinearParams.from_state_dict(sd, f"layers.{l}.") for l in range(2)])
                else:
                    f = O.KANFETRef.from_state_dict(sd, 2)
                y0 = torch.from_numpy(g[f"y0_B{B}"])
                sol = O.odeint(lambda t, y: f(y), y0, torch.from_numpy(g[tag]), method="rk4")
                assert torch.equal(sol, torch.from_numpy(g[f"sol_B{B}_{tag}"])), (name, B, tag)


def test_dopri5_trace_bitwise():
    g = load_golden("dopri5_kanfet")
    f = O.KANFETRef.from_state_dict(golden_sd(g), 2)
    tr = O.Dopri5Trace()
    sol = O.odeint(lambda t, y: f(y), torch.from_numpy(g["y0"]), torch.from_numpy(g["t"]),
                   method="dopri5", rtol=1e-3, atol=1e-4, trace=tr)
    assert torch.equal(sol, torch.from_numpy(g["sol"]))
    att = np.array([[a[0], a[1], a[2], float(a[3])] for a in tr.attempts])
    np.testing.assert_array_equal(att, g["attempts"])
    assert tr.nfev == int(g["nfev"])
    # 2 evaluations before stepping + 6 per attempt (FSAL)
    assert tr.nfev == 2 + 6 * len(tr.attempts)
