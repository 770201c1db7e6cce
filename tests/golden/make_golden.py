"""Generate the golden fixtures under tests/golden/ from the REFERENCE modules.

Run in the survey/build container (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py

It imports the reference's own ``efficient_kan/efficientkan.py`` (KANLinear, KAN)
and ``ferro_class.py`` (FerroelectricBasis), drives them on seeded inputs, and
stores inputs + parameters + outputs as .npz (no pickles).  The reference ships
no odeint (torchdiffeq is absent), so trajectory fixtures integrate
the *reference modules* with the oracle's restated torchdiffeq solver
(oracle/torch_ref.py).  Before writing, every fixture is cross-checked bit for
bit against the oracle restatement, so the oracle is pinned to the reference.
"""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FETODE_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REF, "efficient_kan"))
sys.path.insert(0, REF)

import efficientkan  # noqa: E402  (reference)
import ferro_class  # noqa: E402  (reference)

from oracle import torch_ref as O  # noqa: E402

torch.set_num_threads(1)


class RefKANFETLayer(nn.Module):
    """SURVEY §8a A9 composition of the two reference modules."""

    def __init__(self, i, o, grid_size=5, K=10):
        super().__init__()
        self.kan = efficientkan.KANLinear(i, o, grid_size=grid_size)
        self.ferro = ferro_class.FerroelectricBasis(i, o, K)

    def forward(self, x):
        return self.kan(x) + self.ferro(x)


class RefKANFET(nn.Module):
    def __init__(self, dims, grid_size=5, K=10):
        super().__init__()
        self.layers = nn.ModuleList(RefKANFETLayer(i, o, grid_size, K) for i, o in zip(dims, dims[1:]))

    def forward(self, x):
        for l in self.layers:
            x = l(x)
        return x


def sd_np(module, prefix="sd/"):
    return {prefix + k: v.detach().cpu().numpy() for k, v in module.state_dict().items()}


def assert_bitwise(a, b, what):
    a = a.detach() if torch.is_tensor(a) else torch.as_tensor(a)
    b = b.detach() if torch.is_tensor(b) else torch.as_tensor(b)
    same_nan = torch.equal(torch.isnan(a), torch.isnan(b))
    if not (same_nan and torch.equal(torch.nan_to_num(a, nan=0.0), torch.nan_to_num(b, nan=0.0))):
        d = (a - b).abs().max().item()
        raise SystemExit(f"oracle != reference for {what}: max|diff|={d}")


def kanlinear_cases():
    out = {}
    torch.manual_seed(1234)
    for (i, o) in ((2, 10), (10, 2)):
        m = efficientkan.KANLinear(i, o, grid_size=5)
        g = torch.Generator().manual_seed(7 + i)
        x_wide = torch.rand(48, i, generator=g) * 6 - 3                  # [-3,3)
        x_lv = torch.rand(48, i, generator=g) * 6.75 + 0.25              # LV range [0.25,7)
        knots = m.grid[0].clone()
        x_knot = knots[torch.arange(16) % knots.numel()].unsqueeze(1).expand(16, i).clone()
        # non-finite / huge inputs: the reference returns NaN bases for +-inf and NaN, zeros for 1e30
        x_odd = torch.tensor([float("inf"), float("-inf"), float("nan"), 1e30]).unsqueeze(1).expand(4, i).clone()
        x = torch.cat([x_wide, x_lv, x_knot]).contiguous()
        with torch.no_grad():
            bases_odd = m.b_splines(x_odd)
        with torch.no_grad():
            y = m(x)
            bases = m.b_splines(x)
        p = O.KANLinearParams.from_state_dict(m.state_dict())
        assert_bitwise(O.kanlinear_forward(x, p), y, f"KANLinear({i},{o}).forward")
        assert_bitwise(O.b_splines(x, p.grid, 3), bases, f"KANLinear({i},{o}).b_splines")
        tag = f"kanlinear_{i}x{o}"
        assert_bitwise(O.b_splines(x_odd, p.grid, 3), bases_odd, "b_splines non-finite")
        out[tag] = dict(x=x.numpy(), y=y.numpy(), bases=bases.numpy(), x_odd=x_odd.numpy(),
                        bases_odd=bases_odd.numpy(), **sd_np(m))
    return out


def ferro_cases():
    out = {}
    torch.manual_seed(4321)
    for (i, o, K) in ((2, 10, 10), (10, 2, 10)):
        # (a) fresh module, B=1 first call (prev_x = zeros, dx = x), then a 4-call sequence
        m = ferro_class.FerroelectricBasis(i, o, K)
        init_sd = sd_np(m)
        p = O.FerroParams.from_state_dict(m.state_dict())
        st = O.FerroState(i, o, K)
        g = torch.Generator().manual_seed(99 + i)
        xs1 = [torch.randn(1, i, generator=g) * 2 for _ in range(4)]
        ys1, prev1, basis1 = [], [], []
        for x in xs1:
            with torch.no_grad():
                y, basis, _ = m(x, return_activations=True)
            yo, bo, _ = O.ferro_forward(x, p, st, return_activations=True)
            assert_bitwise(yo, y, "Ferro B=1 out")
            assert_bitwise(bo, basis, "Ferro B=1 basis")
            assert_bitwise(st.prev_x, m.prev_x, "Ferro B=1 prev_x")
            ys1.append(y.numpy())
            prev1.append(m.prev_x[:, :, 0, 0].numpy().copy())
            basis1.append(basis.numpy())
        # (b) fresh module, B=5 (reinit rule: prev_x := x, dx = 0), 5 consecutive calls
        m2 = ferro_class.FerroelectricBasis(i, o, K)
        init_sd2 = sd_np(m2)
        p2 = O.FerroParams.from_state_dict(m2.state_dict())
        st2 = O.FerroState(i, o, K)
        xs5 = [torch.randn(5, i, generator=g) * 2 for _ in range(5)]
        ys5, prev5 = [], []
        for x in xs5:
            with torch.no_grad():
                y = m2(x)
            assert_bitwise(O.ferro_forward(x, p2, st2), y, "Ferro B=5 out")
            assert_bitwise(st2.prev_x, m2.prev_x, "Ferro B=5 prev_x")
            assert bool((m2.prev_x == m2.prev_x[:, :, :1, :1]).all()), "prev_x not compactible"
            assert bool((m2.branch_sign == 1).all()), "branch_sign changed"
            ys5.append(y.numpy())
            prev5.append(m2.prev_x[:, :, 0, 0].numpy().copy())
        # (c) after reset_state (ferro_class.py:422-424): prev zeros of shape (5,...)
        m2.reset_state()
        st2.reset()
        xr = torch.randn(5, i, generator=g)
        with torch.no_grad():
            yr = m2(xr)
        assert_bitwise(O.ferro_forward(xr, p2, st2), yr, "Ferro after reset")
        tag = f"ferro_{i}x{o}x{K}"
        out[tag] = dict(
            xs1=np.stack([x.numpy() for x in xs1]), ys1=np.stack(ys1), prev1=np.stack(prev1),
            basis1=np.stack(basis1), xs5=np.stack([x.numpy() for x in xs5]), ys5=np.stack(ys5),
            prev5=np.stack(prev5), x_reset=xr.numpy(), y_reset=yr.numpy(),
            **init_sd, **{("sd2/" + k[3:]): v for k, v in init_sd2.items()})
    return out


def kanfet_field_and_grad():
    torch.manual_seed(0)
    m = RefKANFET([2, 10, 2])
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    y0 = O.lv_y0(16, seed=3)
    x = y0.clone().requires_grad_(True)
    # two consecutive calls so that the second sees dx != 0
    f1 = m(x)
    f2 = m(x * 1.01 + 0.05)
    loss = (f1.square().mean() + (f2 * torch.linspace(-1, 1, 2)).sum())
    loss.backward()
    grads = {"grad/" + n: p.grad.numpy().copy() for n, p in m.named_parameters()}
    grads["grad/x"] = x.grad.numpy().copy()
    # oracle cross-check on the forward values (state sequence included)
    ref = O.KANFETRef.from_state_dict(sd0, 2)
    xo = y0.clone()
    assert_bitwise(ref(xo), f1, "KANFET call 1")
    assert_bitwise(ref(xo * 1.01 + 0.05), f2, "KANFET call 2")
    return {"kanfet_field": dict(y0=y0.numpy(), f1=f1.detach().numpy(), f2=f2.detach().numpy(),
                                 **{"sd/" + k: v.numpy() for k, v in sd0.items()}, **grads)}


def trajectories():
    out = {}
    t35 = torch.tensor(np.linspace(0, 3.5, 35))                      # float64, as t_learn (:155)
    t140 = torch.tensor(np.linspace(0, 14, 140), dtype=torch.float32)  # as t (:154)
    for name, ctor in (("kan", lambda: efficientkan.KAN([2, 10, 2], grid_size=5)),
                       ("kanfet", lambda: RefKANFET([2, 10, 2]))):
        torch.manual_seed(0)
        m = ctor()
        sd0 = {k: v.clone() for k, v in m.state_dict().items()}
        rec = {"sd/" + k: v.numpy() for k, v in sd0.items()}
        for B in (1, 64):
            y0 = O.lv_y0(B, seed=11)
            for tag, t in (("t35", t35), ("t140", t140)):
                m.load_state_dict(sd0, strict=False)
                fresh = ctor()
                fresh.load_state_dict(sd0)
                func = lambda tt, yy: fresh(yy)
                with torch.no_grad():
                    sol = O.odeint(func, y0, t, method="rk4")
                # oracle-only restatement of the field must give the same bits
                if name == "kan":
                    oref = O.KANRef([O.KANLinearParams.from_state_dict(sd0, f"layers.{l}.") for l in range(2)])
                else:
                    oref = O.KANFETRef.from_state_dict(sd0, 2)
                with torch.no_grad():
                    sol_o = O.odeint(lambda tt, yy: oref(yy), y0, t, method="rk4")
                assert_bitwise(sol_o, sol, f"{name} rk4 B={B} {tag}")
                rec[f"y0_B{B}"] = y0.numpy()
                rec[f"sol_B{B}_{tag}"] = sol.numpy()
                if name == "kanfet":
                    rec[f"prev0_B{B}_{tag}"] = fresh.layers[0].ferro.prev_x[:, :, 0, 0].numpy().copy()
                    rec[f"prev1_B{B}_{tag}"] = fresh.layers[1].ferro.prev_x[:, :, 0, 0].numpy().copy()
        rec["t35"] = t35.numpy()
        rec["t140"] = t140.numpy()
        out[f"traj_{name}"] = rec
    return out


def dopri5_trace():
    torch.manual_seed(5)
    m = RefKANFET([2, 10, 2])
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    y0 = O.lv_y0(8, seed=21) * 0.5
    t = torch.tensor([0.0, 0.25, 0.5, 1.0])
    tr = O.Dopri5Trace()
    with torch.no_grad():
        sol = O.odeint(lambda tt, yy: m(yy), y0, t, method="dopri5", rtol=1e-3, atol=1e-4, trace=tr)
    oref = O.KANFETRef.from_state_dict(sd0, 2)
    tr2 = O.Dopri5Trace()
    with torch.no_grad():
        sol2 = O.odeint(lambda tt, yy: oref(yy), y0, t, method="dopri5", rtol=1e-3, atol=1e-4, trace=tr2)
    assert_bitwise(sol2, sol, "dopri5 solution")
    assert tr.attempts == tr2.attempts
    att = np.array([[a[0], a[1], a[2], float(a[3])] for a in tr.attempts])
    return {"dopri5_kanfet": dict(y0=y0.numpy(), t=t.numpy(), sol=sol.numpy(), attempts=att,
                                  nfev=np.array(tr.nfev), first_step=np.array(tr.first_step),
                                  **{"sd/" + k: v.numpy() for k, v in sd0.items()})}


def lv_truth():
    t, soln = O.lotka_volterra_truth()
    return {"lv_lsoda": dict(t=t, soln=soln)}


def main():
    allc = {}
    for fn in (kanlinear_cases, ferro_cases, kanfet_field_and_grad, trajectories, dopri5_trace, lv_truth):
        allc.update(fn())
    for name, d in allc.items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **d)
        print(f"wrote {path}  ({os.path.getsize(path)} B, {len(d)} arrays)")


if __name__ == "__main__":
    main()
