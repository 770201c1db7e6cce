"""MI355X parity of the ETT KAN-RNN encoder (train_kan_fet_ett.py:741-818; the encoder of
KAN_FET_LatentODE_DiffusionForecaster, :822-837): fetode_kanrnn_forward / _backward and
fetode_logistic_basis_* against the reference fixtures (tests/golden/ett_kanrnn_*.npz, ett_kancell.npz,
made by the reference's own classes) and, at the production batch, against oracle/ett_ref.py.

Bars: forward 1e-5 per row (norm-relative), NaN patterns equal; gradients within 1e-4 of the
largest reference magnitude per tensor, NaN patterns equal (the reference autograd's NaN from
dropped columns whose exp overflows, and from NaN / inf inputs)."""
import numpy as np
import pytest
import torch

from conftest import golden_sd, load_golden
from oracle import ett_ref as E

pytestmark = pytest.mark.gpu


def row_rel(got, exp):
    got, exp = torch.as_tensor(got).double().cpu(), torch.as_tensor(exp).double().cpu()
    got, exp = got.reshape(got.shape[0], -1), exp.reshape(exp.shape[0], -1)
    fin = torch.isfinite(exp).all(1)
    if not fin.any():
        return 0.0
    g, e = got[fin], exp[fin]
    return ((g - e).norm(dim=1) / e.norm(dim=1).clamp_min(1e-30)).max().item()


def same_nan(got, exp):
    got, exp = torch.as_tensor(got).cpu(), torch.as_tensor(exp).cpu()
    return torch.equal(got.isnan(), exp.isnan())


def grad_close(got, exp, tol=1e-4):
    got, exp = torch.as_tensor(got).double().cpu(), torch.as_tensor(exp).double().cpu()
    assert same_nan(got, exp), (int(got.isnan().sum()), int(exp.isnan().sum()))
    m = ~exp.isnan()
    if not m.any():
        return
    scale = exp[m].abs().max().item()
    err = (got[m] - exp[m]).abs().max().item()
    assert err <= tol * scale + 1e-12, (err, scale)


def _encoder(g, dev):
    from fet_ode_amd import ett
    F_, H, latent, nb = (int(v) for v in g["dims"])
    enc = ett.KANRNNEncoder(F_, H, latent, nb)
    enc.load_state_dict(golden_sd(g))
    return enc.to(dev)


@pytest.mark.parametrize("name", ["ett_kanrnn_prod", "ett_kanrnn_deep", "ett_kanrnn_overflow"])
def test_kanrnn_encoder_forward_and_grads_vs_reference(dev, name):
    g = load_golden(name)
    enc = _encoder(g, dev)
    for T in g["Ts"]:
        x = torch.from_numpy(g[f"T{T}/x"]).to(dev)
        with torch.no_grad():
            z_nograd = enc(x)
        exp = g[f"T{T}/z0"]
        assert same_nan(z_nograd, exp)
        assert row_rel(z_nograd, exp) <= 1e-5, (T, row_rel(z_nograd, exp))
        enc.zero_grad(set_to_none=True)
        xr = x.clone().requires_grad_(True)
        z = enc(xr)
        assert torch.equal(z.detach().isnan(), z_nograd.isnan())
        assert row_rel(z.detach(), exp) <= 1e-5
        (z * torch.from_numpy(g[f"T{T}/w"]).to(dev)).sum().backward()
        for k, p in enc.named_parameters():
            grad_close(p.grad, g[f"T{T}/grad/{k}"])
        grad_close(xr.grad, g[f"T{T}/grad_in/x"])


def test_kanrnn_cone_equals_full_recurrence(dev):
    """fetode_kanrnn_forward with full = 0 (only the steps that reach h_T) and full = 1 give the
    same h_T bit for bit, NaN / inf inputs anywhere in the context included."""
    from fet_ode_amd import _lib, ett
    for (F_, H, nb) in [(7, 64, 10), (2, 16, 1), (1, 130, 1), (3, 200, 2)]:
        torch.manual_seed(F_ + H)
        cell = ett.FullyNonlinearKANCell(F_, H, nb).to(dev)
        x = torch.randn(300, 40, F_, device=dev)
        x[0, 3, 0] = float("nan")
        x[1, 38, 0] = float("inf")
        x[2, 39, F_ - 1] = float("nan")
        keep = []
        d = ett._rnn_desc(cell, None, keep)
        outs = []
        for full in (0, 1):
            h = torch.empty(300, H, device=dev)
            _lib.check(_lib.load().fetode_kanrnn_forward(_lib.ctypes.byref(d), x.data_ptr(), 300, 40, None,
                                                         h.data_ptr(), None, None, full, _lib.stream_handle(dev)))
            outs.append(h.cpu())
        a, b = outs
        assert torch.equal(a.isnan(), b.isnan()) and torch.equal(a.nan_to_num(0.0), b.nan_to_num(0.0)), (F_, H, nb)
        ref = torch.zeros(300, H)
        p = [t.detach().cpu() for t in (cell.input_basis.a, cell.input_basis.b, cell.hidden_basis.a,
                                         cell.hidden_basis.b)]
        for t in range(40):
            ref = E.kan_cell(x[:, t].cpu(), ref, *p)
        assert same_nan(a, ref) and row_rel(a, ref) <= 1e-5, (F_, H, nb, row_rel(a, ref))


def test_kancell_and_logistic_basis_linear_vs_reference(dev):
    """FullyNonlinearKANCell from a given h_prev (T = 1 launch with h0, gradients to x_t and h_prev)
    and LogisticBasisLinear (fetode_logistic_basis_* + library GEMM) against the fixture."""
    from fet_ode_amd import ett
    g = load_golden("ett_kancell")
    cell = ett.FullyNonlinearKANCell(3, 8, 2)
    cell.load_state_dict(golden_sd(g, "cell/"))
    cell = cell.to(dev)
    x = torch.from_numpy(g["cell_x"]).to(dev).requires_grad_(True)
    h = torch.from_numpy(g["cell_h"]).to(dev).requires_grad_(True)
    y = cell(x, h)
    assert row_rel(y.detach(), g["cell_y"]) <= 1e-5
    (y * torch.from_numpy(g["cell_w"]).to(dev)).sum().backward()
    for k, p in cell.named_parameters():
        grad_close(p.grad, g[f"cell_grad/{k}"])
    grad_close(x.grad, g["cell_grad_in/x"])
    grad_close(h.grad, g["cell_grad_in/h"])
    lin = ett.LogisticBasisLinear(5, 4, 3)
    lin.load_state_dict(golden_sd(g, "lin/"))
    lin = lin.to(dev)
    xl = torch.from_numpy(g["lin_x"]).to(dev).requires_grad_(True)
    yl = lin(xl)
    assert row_rel(yl.detach(), g["lin_y"]) <= 1e-5
    (yl * torch.from_numpy(g["lin_w"]).to(dev)).sum().backward()
    for k, p in lin.named_parameters():
        grad_close(p.grad, g[f"lin_grad/{k}"])
    grad_close(xl.grad, g["lin_grad_in/x"])


def test_kanrnn_encoder_production_batch_vs_oracle(dev):
    """The bench workload: KANRNNEncoder(7, 64, 64, 10) on B = 8192 windows of 96 steps (ETT
    context), forward (no_grad: the one-step cone; autograd: the full recurrence with its tape) and
    every gradient against the oracle's autograd; the backward is run-to-run bitwise identical."""
    from fet_ode_amd import ett
    torch.manual_seed(0)
    enc = ett.KANRNNEncoder(7, 64, 64, 10)
    sd = {k: v.clone() for k, v in enc.state_dict().items()}
    enc = enc.to(dev)
    gen = torch.Generator().manual_seed(5)
    x = torch.cumsum(torch.randn(8192, 96, 7, generator=gen), 1) * 0.1
    w = torch.randn(8192, 64, generator=gen)
    with torch.no_grad():
        z_fast = enc(x.to(dev)).cpu()
    ps = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    z_ref = E.KANRNNEncoderRef(ps)(x)
    (z_ref * w).sum().backward()
    assert row_rel(z_fast, z_ref.detach()) <= 1e-5
    grads = []
    for rep in range(2):
        enc.zero_grad(set_to_none=True)
        z = enc(x.to(dev))
        (z * w.to(dev)).sum().backward()
        grads.append({k: p.grad.detach().cpu().clone() for k, p in enc.named_parameters()})
        assert row_rel(z.detach(), z_ref.detach()) <= 1e-5
    for k, p in ps.items():
        grad_close(grads[0][k], p.grad)
        assert torch.equal(grads[0][k], grads[1][k]), k
