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


class KANFETDynamics(nn.Module):
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


class LatentNeuralODEForecaster(nn.Module):
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
