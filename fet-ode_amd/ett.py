"""Drop-in ETT forecasting path (BASELINE config "train_kan_fet_ett.py: ETTh1
96 -> 96 forecast, KAN-FET vector field"), train_kan_fet_ett.py:
  * odeint_rk4                 :51-83   classic RK4 with ``n_substeps`` substeps per output interval
  * EnergyWindowDataset        :107-131 sliding (context, future) windows — device resident here,
                                        with a batched gather (``batch(idx)``) for the training loop
  * LatentNeuralODEForecaster  :155-197 MLP encoder -> latent ODE -> MLP decoder per time slice
  * KANFETDynamics             the KAN-FET latent vector field that config 4 names in place of the
                               reference's MLP ODEDynamics (:136-152)

The latent ODE runs on the HIP integrator (``odeint_rk4`` builds the reference's substep grid and
drives the same fixed-grid machinery as ``fet_ode_amd.odeint``: the fused single launch when the
field has a fused kernel, otherwise one HIP field evaluation per stage with HIP combines).  The
encoder / decoder Linear layers are plain library GEMMs (hipBLASLt through torch).  There is no
CPU path: CPU tensors raise.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from ._lib import CacheFreeState
from .efficientkan import KANFET
from .odeint import Schedule, _per_stage_fixed, _try_fused

_SUB_CACHE: Dict[tuple, Schedule] = {}


def _substep_schedule(t: torch.Tensor, n_substeps: int) -> Schedule:
    tp = t.detach().cpu()
    key = (tp.dtype, tuple(tp.tolist()), int(n_substeps))
    s = _SUB_CACHE.get(key)
    if s is None:
        if len(_SUB_CACHE) > 64:
            _SUB_CACHE.clear()
        s = _SUB_CACHE[key] = Schedule.substeps(tp, int(n_substeps))
    return s


def odeint_rk4(f, z0: torch.Tensor, t: torch.Tensor, n_substeps: int = 4) -> torch.Tensor:
    """train_kan_fet_ett.py:51-83 on the GPU: z0 (B, D), t (T,) increasing -> (T, B, D).

    Per interval h = (t1 - t0) / n_substeps (t's dtype), then n_substeps classic-RK4 steps
    (k2, k3 at ti + h/2, k4 at ti + h; z += (h / 6)(k1 + 2 k2 + 2 k3 + k4)); solution[j] is z
    after interval j.  ``f(t, z)``; fields wrapped by ``fet_ode_amd.autonomous`` (or
    KANFETDynamics) integrate in the HIP fused or per-stage path."""
    assert t.ndim == 1
    if n_substeps < 1:
        raise ValueError("n_substeps must be >= 1")
    if not torch.is_floating_point(z0):
        raise TypeError("`z0` must be a floating point Tensor")
    _lib.require_gpu_tensor(z0, "odeint_rk4")
    if t.shape[0] > 1 and not bool((t[1:] > t[:-1]).all()):
        raise AssertionError("t must be strictly increasing")
    sched = _substep_schedule(t, n_substeps)
    out = _try_fused(f, z0, sched, _lib.RK4_CLASSIC)
    if out is not None:
        return out
    return _per_stage_fixed(f, z0, sched, "rk4_classic", t.dtype, False)


class EnergyWindowDataset:
    """train_kan_fet_ett.py:107-131, device resident: X (N, F), y (N,) standardized series.
    ``ds[i]`` -> (x_ctx (c, F), y_fut (p,)) views; ``ds.batch(idx)`` -> ((n, c, F), (n, p)) gathered
    in HBM for a LongTensor of window starts (the DataLoader's collate, without a host round trip)."""

    def __init__(self, X, y, context_len: int, pred_len: int, device=None):
        X = torch.as_tensor(np.asarray(X, dtype=np.float32) if not torch.is_tensor(X) else X, dtype=torch.float32)
        y = torch.as_tensor(np.asarray(y, dtype=np.float32) if not torch.is_tensor(y) else y, dtype=torch.float32)
        self.context_len, self.pred_len = int(context_len), int(pred_len)
        self.N = len(X)
        self.max_start = self.N - (self.context_len + self.pred_len) + 1
        if self.max_start <= 0:
            raise ValueError("Not enough rows for given context_len + pred_len.")
        self.X = X.to(device) if device is not None else X
        self.y = y.to(device) if device is not None else y

    def __len__(self) -> int:
        return self.max_start

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, torch.Tensor]:
        if idx < 0:
            idx += self.max_start
        if not 0 <= idx < self.max_start:
            raise IndexError(idx)
        c, p = self.context_len, self.pred_len
        return self.X[idx:idx + c], self.y[idx + c:idx + c + p]

    def batch(self, idx: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        c, p = self.context_len, self.pred_len
        idx = idx.to(self.X.device)
        xw = self.X.unfold(0, c, 1)[idx].transpose(1, 2)        # (n, c, F)
        yw = self.y.unfold(0, p, 1)[idx + c]                    # (n, p)
        return xw.contiguous(), yw.contiguous()


class KANFETDynamics(CacheFreeState, nn.Module):
    """Latent vector field f(t, z) = KANFET([latent, hidden, latent])(z) (autonomous; t ignored),
    the KAN-FET field of BASELINE config 4 in the place of ODEDynamics (train_kan_fet_ett.py:136-152).
    Tagged so that the integrators take the HIP fused path whenever the shape has one."""

    def __init__(self, latent_dim: int, hidden: int = 128, grid_size: int = 5, num_fet_basis: int = 10):
        super().__init__()
        self.net = KANFET([latent_dim, hidden, latent_dim], grid_size=grid_size, num_fet_basis=num_fet_basis)

    @property
    def _fetode_field(self):
        return self.net

    def forward(self, t, z):
        return self.net(z)


class LatentNeuralODEForecaster(CacheFreeState, nn.Module):
    """train_kan_fet_ett.py:155-197 with the KAN-FET latent field.  Same constructor arguments and
    encoder / decoder state_dict keys (encoder.1, encoder.3, decoder.0, decoder.2); ``solver`` picks
    the latent integrator: 'dopri5' (the reference's forward, :192, torchdiffeq defaults) or 'rk4'
    (its odeint_rk4 alternative with ``rk4_substeps``)."""

    def __init__(self, num_features: int, context_len: int, pred_len: int, latent_dim: int = 64,
                 enc_hidden: int = 128, dec_hidden: int = 128, dyn_hidden: int = 128, solver: str = "dopri5",
                 rtol: float = 1e-7, atol: float = 1e-9, grid_size: int = 5, num_fet_basis: int = 10):
        super().__init__()
        if solver not in ("dopri5", "rk4"):
            raise ValueError(f"solver must be 'dopri5' or 'rk4', got {solver!r}")
        self.context_len, self.pred_len, self.latent_dim = context_len, pred_len, latent_dim
        self.solver, self.rtol, self.atol = solver, rtol, atol
        self.encoder = nn.Sequential(nn.Flatten(), nn.Linear(context_len * num_features, enc_hidden), nn.ReLU(),
                                     nn.Linear(enc_hidden, latent_dim))
        self.dynamics = KANFETDynamics(latent_dim, dyn_hidden, grid_size=grid_size, num_fet_basis=num_fet_basis)
        self.decoder = nn.Sequential(nn.Linear(latent_dim, dec_hidden), nn.ReLU(), nn.Linear(dec_hidden, 1))

    def forward(self, x_ctx: torch.Tensor, t_fut: torch.Tensor, rk4_substeps: int = 4) -> torch.Tensor:
        """x_ctx (B, context_len, F), t_fut (pred_len,) -> y_hat (B, pred_len)."""
        _lib.require_gpu_tensor(x_ctx, "LatentNeuralODEForecaster.forward")
        z0 = self.encoder(x_ctx)
        if self.solver == "rk4":
            zt = odeint_rk4(self.dynamics, z0, t_fut, n_substeps=rk4_substeps)
        else:
            from .odeint import odeint
            zt = odeint(self.dynamics, z0, t_fut, rtol=self.rtol, atol=self.atol, method="dopri5")
        return self.decoder(zt).squeeze(-1).transpose(0, 1)


# ---------------------------------------------------------------------------------------------
# KAN-RNN encoder of KAN_FET_LatentODE_DiffusionForecaster (train_kan_fet_ett.py:741-818, used at
# :832-837): LogisticBasis, LogisticBasisLinear, FullyNonlinearKANCell, KANRNNEncoder.  Same
# constructor arguments, parameter names / shapes and init RNG order as the reference; the
# recurrence runs in ONE HIP launch (fetode_kanrnn_forward, h on chip, to_latent fused) with a HIP
# VJP (fetode_kanrnn_backward); LogisticBasis alone runs fetode_logistic_basis_*.
# ---------------------------------------------------------------------------------------------

def _stream(t):
    return _lib.stream_handle(t.device)


class _LogisticBasisFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, a, b):
        xc = _lib.f32c(x)
        B, n = xc.shape
        nb = a.shape[1]
        ac, bc = _lib.f32c(a), _lib.f32c(b)
        phi = torch.empty(B, n, nb, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().fetode_logistic_basis_forward(xc.data_ptr(), B, n, nb, ac.data_ptr(), bc.data_ptr(),
                                                             phi.data_ptr(), _stream(x)), "LogisticBasis.forward")
        ctx.save_for_backward(xc, ac, bc)
        return phi

    @staticmethod
    def backward(ctx, g):
        xc, ac, bc = ctx.saved_tensors
        B, n = xc.shape
        nb = ac.shape[1]
        lib = _lib.load()
        gx = torch.empty_like(xc) if ctx.needs_input_grad[0] else None
        want_p = ctx.needs_input_grad[1] or ctx.needs_input_grad[2]
        ga = torch.empty_like(ac) if want_p else None
        gb = torch.empty_like(bc) if want_p else None
        ws = None
        if want_p:
            ws = torch.empty(max(1, lib.fetode_logistic_basis_backward_workspace(n, nb, B) // 4), device=xc.device)
        _lib.check(lib.fetode_logistic_basis_backward(xc.data_ptr(), B, n, nb, ac.data_ptr(), bc.data_ptr(),
                                                      _lib.f32c(g).data_ptr(), _lib.ptr(gx), _lib.ptr(ga), _lib.ptr(gb),
                                                      _lib.ptr(ws), _stream(xc)), "LogisticBasis backward")
        return gx, ga, gb


class LogisticBasis(CacheFreeState, nn.Module):
    """train_kan_fet_ett.py:741-749: phi = 2 / (1 + exp(-a (x - b))), x (B, in) -> (B, in, nb)."""

    def __init__(self, in_dim, num_basis):
        super().__init__()
        self.a = nn.Parameter(torch.randn(in_dim, num_basis))
        self.b = nn.Parameter(torch.randn(in_dim, num_basis))

    def forward(self, x):
        _lib.require_gpu_tensor(x, "LogisticBasis.forward")
        if x.dim() != 2 or x.shape[1] != self.a.shape[0]:
            raise ValueError(f"LogisticBasis expects x of shape (B, {self.a.shape[0]}), got {tuple(x.shape)}")
        return _LogisticBasisFn.apply(x, self.a, self.b)


class LogisticBasisLinear(CacheFreeState, nn.Module):
    """train_kan_fet_ett.py:753-776: logistic basis expansion, then phi @ weight + bias (the
    contraction is a plain library GEMM through torch)."""

    def __init__(self, in_dim: int, out_dim: int, num_basis: int, bias: bool = True):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.num_basis = num_basis
        self.basis = LogisticBasis(in_dim, num_basis)
        self.weight = nn.Parameter(torch.randn(in_dim * num_basis, out_dim) * 0.02)
        self.bias = nn.Parameter(torch.zeros(out_dim)) if bias else None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        phi = self.basis(x).reshape(x.shape[0], -1)
        y = phi @ self.weight
        if self.bias is not None:
            y = y + self.bias
        return y


def _rnn_desc(cell, lin, keep):
    ps = [_lib.f32c(p) for p in (cell.input_basis.a, cell.input_basis.b, cell.hidden_basis.a, cell.hidden_basis.b)]
    w = b = None
    latent = 0
    if lin is not None:
        w, b = _lib.f32c(lin.weight), _lib.f32c(lin.bias) if lin.bias is not None else None
        latent = w.shape[0]
        if b is None:
            b = torch.zeros(latent, device=w.device)
    keep += ps + [w, b]
    F_, nb = ps[0].shape
    H = ps[2].shape[0]
    return _lib.KANRNNDesc(F_, H, nb, latent, *(t.data_ptr() for t in ps), _lib.ptr(w), _lib.ptr(b))


def _fused_projection(lin, H) -> bool:
    """to_latent inside the recurrence launch (W^T in LDS, rows padded to latent + 1) when it fits."""
    return lin is not None and lin.weight.shape[0] <= 256 and (lin.weight.shape[0] + 1) * H <= 16384


class _KANRNNFn(torch.autograd.Function):
    """h_T of the recurrence (and z0 = to_latent(h_T) when `lin` is given and fits the launch)."""

    @staticmethod
    def forward(ctx, cell, lin, x, h0, ax, bx, ah, bh, w, bias):
        keep = []
        fuse = _fused_projection(lin, cell.hidden_size)
        d = _rnn_desc(cell, lin if fuse else None, keep)
        xc = _lib.f32c(x)
        B, T, _ = xc.shape
        H = cell.hidden_size
        h0c = _lib.f32c(h0) if h0 is not None else None
        grad = any(ctx.needs_input_grad[2:])
        tape = torch.empty(B, T, H, device=x.device) if grad else None
        hT = torch.empty(B, H, device=x.device) if (grad or not fuse) else None
        z0 = torch.empty(B, d.latent, device=x.device) if fuse else None
        _lib.check(_lib.load().fetode_kanrnn_forward(ctypes_byref(d), xc.data_ptr(), B, T, _lib.ptr(h0c), _lib.ptr(hT),
                                                     _lib.ptr(z0), _lib.ptr(tape), 0, _stream(x)), "KAN-RNN forward")
        ctx.cell, ctx.lin, ctx.fuse = cell, lin, fuse
        ctx.save_for_backward(xc, h0c, tape, hT)
        if lin is not None and not fuse:
            return torch.nn.functional.linear(hT, lin.weight, lin.bias)
        return z0 if fuse else hT

    @staticmethod
    def backward(ctx, g):
        xc, h0c, tape, hT = ctx.saved_tensors
        cell, lin = ctx.cell, ctx.lin
        B, T, _ = xc.shape
        g = _lib.f32c(g)
        gw = gbias = None
        if lin is not None:
            w = lin.weight.detach()
            if ctx.needs_input_grad[8]:
                gw = g.t() @ hT
            if ctx.needs_input_grad[9]:
                gbias = g.sum(0)
            g_h = (g @ w).contiguous()
        else:
            g_h = g
        keep = []
        d = _rnn_desc(cell, None, keep)
        lib = _lib.load()
        gx = torch.empty_like(xc) if ctx.needs_input_grad[2] else None
        gh0 = torch.empty_like(h0c) if (h0c is not None and ctx.needs_input_grad[3]) else None
        want_p = any(ctx.needs_input_grad[4:8])
        gp = [torch.empty_like(p) for p in (cell.input_basis.a, cell.input_basis.b, cell.hidden_basis.a,
                                            cell.hidden_basis.b)] if want_p else [None] * 4
        ws = torch.empty(max(1, lib.fetode_kanrnn_backward_workspace(ctypes_byref(d), B) // 4), device=xc.device)
        _lib.check(lib.fetode_kanrnn_backward(ctypes_byref(d), xc.data_ptr(), B, T, _lib.ptr(h0c), tape.data_ptr(),
                                              g_h.data_ptr(), _lib.ptr(gx), _lib.ptr(gh0), *(_lib.ptr(t) for t in gp),
                                              ws.data_ptr(), _stream(xc)), "KAN-RNN backward")
        return (None, None, gx, gh0, *gp, gw, gbias)


def ctypes_byref(d):
    return _lib.ctypes.byref(d)


def kanrnn_apply(cell, x, h0=None, lin=None):
    """h_T (or to_latent(h_T)) of FullyNonlinearKANCell run over x (B, T, F) from h0 (None = zeros)."""
    _lib.require_gpu_tensor(x, "KAN-RNN")
    params = (cell.input_basis.a, cell.input_basis.b, cell.hidden_basis.a, cell.hidden_basis.b)
    w = lin.weight if lin is not None else None
    bias = lin.bias if lin is not None else None
    return _KANRNNFn.apply(cell, lin, x, h0, *params, w, bias)


class FullyNonlinearKANCell(CacheFreeState, nn.Module):
    """train_kan_fet_ett.py:780-795: h = sigmoid(cat(phi_x(x_t), phi_h(h_prev)))[:, :hidden_size]."""

    def __init__(self, input_size, hidden_size, num_basis):
        super().__init__()
        self.input_basis = LogisticBasis(input_size, num_basis)
        self.hidden_basis = LogisticBasis(hidden_size, num_basis)
        self.activation = nn.Sigmoid()
        self.hidden_size = hidden_size
        self.num_basis = num_basis

    def forward(self, x_t, h_prev):
        if x_t.dim() != 2 or h_prev.dim() != 2 or h_prev.shape[1] != self.hidden_size:
            raise ValueError("FullyNonlinearKANCell expects x_t (B, input_size) and h_prev (B, hidden_size)")
        _lib.require_gpu_tensor(h_prev, "FullyNonlinearKANCell.forward")
        return kanrnn_apply(self, x_t.unsqueeze(1), h_prev)


class KANRNNEncoder(CacheFreeState, nn.Module):
    """train_kan_fet_ett.py:798-818: the cell over the context from h = 0, then to_latent(h_T).
    The whole recurrence + projection is one launch."""

    def __init__(self, num_features: int, hidden_size: int, latent_dim: int, num_basis: int):
        super().__init__()
        self.hidden_size = hidden_size
        self.rnn_cell = FullyNonlinearKANCell(num_features, hidden_size, num_basis)
        self.to_latent = nn.Linear(hidden_size, latent_dim)

    def forward(self, x_ctx: torch.Tensor) -> torch.Tensor:
        B, T, F_ = x_ctx.shape
        if T == 0:
            _lib.require_gpu_tensor(x_ctx, "KANRNNEncoder.forward")
            h = torch.zeros(B, self.hidden_size, device=x_ctx.device, dtype=x_ctx.dtype)
            return self.to_latent(h)
        return kanrnn_apply(self.rnn_cell, x_ctx, None, self.to_latent)
