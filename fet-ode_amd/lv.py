"""Lotka-Volterra training harness (SURVEY §8c "Python-harness counterpart", §8f rank 4):
train_kanfet_node_predprey.py and train_kanfet_mlp_node_predprey.py on the HIP integrator.

  * lv_problem                 train_kanfet_node_predprey.py:20-52,148-155  X0 (1, 2), t (140,) f32,
                               t_learn (35,) (f64 in the plain script, f32 in the MLP-head script),
                               the scipy LSODA ground truth soln_arr (140, 2)
  * ResidualBottleneckMLPHead  train_kanfet_mlp_node_predprey.py:192-203  y + MLP(y), applied to the
                               predicted trajectory after odeint
  * KANFET_ODE_WithHead        :206-220  KANFET dynamics (``rhs``) + the head; ``rhs`` is tagged so
                               ``odeint(model.rhs, ...)`` is one fused HIP launch (and one reverse-
                               sweep launch under autograd)
  * train_epoch / test_loss    :240-275 (plain: :244-262)  one Adam epoch on the 35-point window,
                               the test MSE on points 35..139

The head is a (T, 1, 2)-sized torch MLP (negligible next to the solve); the solve runs in
libfetode.so.  There is no CPU path for the solve: CPU tensors raise.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from ._lib import CacheFreeState

from .efficientkan import autonomous
from .odeint import fused_field as fused_field_of
from .odeint import odeint


@dataclass
class LVProblem:
    X0: torch.Tensor          # (1, 2) f32
    t: torch.Tensor           # (N_t,) f32, 0 .. tf
    t_learn: torch.Tensor     # (N_t_train,) 0 .. tf_learn
    soln_arr: torch.Tensor    # (N_t, 2) f32 LSODA truth
    n_train: int

    @property
    def soln_train(self) -> torch.Tensor:
        return self.soln_arr[:self.n_train]


def lv_problem(device="cuda", tf=14.0, tf_learn=3.5, n_train=35, x0=1.0, y0=1.0, alpha=1.5, beta=1.0,
               gamma=3.0, delta=1.0, t_learn_dtype=torch.float64) -> LVProblem:
    """train_kanfet_node_predprey.py:20-52 (data) and :148-155 (tensors)."""
    import scipy.integrate

    def deriv(X, t, alpha, beta, delta, gamma):
        x, y = X[0], X[1]
        return [alpha * x - beta * x * y, delta * x * y - gamma * y]

    n_t = int(35 * tf / tf_learn)
    t = np.linspace(0, tf, n_t)
    soln = scipy.integrate.odeint(deriv, np.array([x0, y0]), t, args=(alpha, beta, delta, gamma))
    X0 = torch.unsqueeze(torch.Tensor(np.transpose(np.array([x0, y0]))), 0)
    return LVProblem(X0=X0.to(device), t=torch.Tensor(t).to(device),
                     t_learn=torch.tensor(np.linspace(0, tf_learn, n_train), dtype=t_learn_dtype).to(device),
                     soln_arr=torch.Tensor(soln).to(device), n_train=n_train)


class ResidualBottleneckMLPHead(CacheFreeState, nn.Module):
    """train_kanfet_mlp_node_predprey.py:192-203."""

    def __init__(self, d_out: int, bottleneck: int = 32, dropout: float = 0.0):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(d_out, bottleneck), nn.GELU(), nn.Dropout(dropout),
                                 nn.Linear(bottleneck, d_out), nn.Dropout(dropout))

    def forward(self, y):
        return y + self.net(y)


class KANFET_ODE_WithHead(CacheFreeState, nn.Module):
    """train_kanfet_mlp_node_predprey.py:206-220: dz/dt = kanfet(z); the head maps the predicted
    trajectory afterwards (not inside the ODE)."""

    def __init__(self, kanfet: nn.Module, state_dim: int, head_bottleneck: int = 32, head_dropout: float = 0.0):
        super().__init__()
        self.kanfet = kanfet
        self.head = ResidualBottleneckMLPHead(state_dim, bottleneck=head_bottleneck, dropout=head_dropout)

    @property
    def rhs(self):
        """``rhs(t, z) = kanfet(z)``, tagged for the fused integrator (not a registered submodule)."""
        f = self.__dict__.get("_rhs")
        if f is None or f.field is not self.kanfet:
            f = autonomous(self.kanfet)
            self.__dict__["_rhs"] = f
        return f


def train_epoch(model: nn.Module, prob: LVProblem, optimizer, method: Optional[str] = None,
                head: Optional[nn.Module] = None) -> torch.Tensor:
    """One epoch of train_kanfet_node_predprey.py:248-256 (``model`` = the KANFET field) or of
    train_kanfet_mlp_node_predprey.py:254-268 (``model`` = KANFET_ODE_WithHead): zero_grad, solve on
    t_learn, MSE of pred[:, 0, :] against the 35-point truth, backward, Adam step.  Returns the loss.

    ``method=None`` is what the reference runs: ``torchodeint(calDeriv, X0, t_learn)`` without a
    method, i.e. dopri5 at rtol 1e-7 / atol 1e-9 (:252).  ``method="rk4"`` is BASELINE configs[1]'s
    fixed-step choice (one fused launch + one reverse-sweep launch)."""
    optimizer.zero_grad()
    if isinstance(model, KANFET_ODE_WithHead):
        pred = model.head(odeint(model.rhs, prob.X0, prob.t_learn, method=method))
    else:
        pred = odeint(autonomous(model), prob.X0, prob.t_learn, method=method)
        if head is not None:
            pred = head(pred)
    loss = torch.mean((pred[:, 0, :] - prob.soln_train) ** 2)
    loss.backward()
    optimizer.step()
    return loss.detach()


@torch.no_grad()
def test_loss(model: nn.Module, prob: LVProblem, method: Optional[str] = None) -> torch.Tensor:
    """The test MSE of :259-261 / :271-275 on points n_train.. of the 140-point horizon (default
    method: dopri5, as the reference's :260)."""
    if isinstance(model, KANFET_ODE_WithHead):
        pred = model.head(odeint(model.rhs, prob.X0, prob.t, method=method))
    else:
        pred = odeint(autonomous(model), prob.X0, prob.t, method=method)
    return torch.mean((pred[prob.n_train:, 0, :] - prob.soln_arr[prob.n_train:]) ** 2)
