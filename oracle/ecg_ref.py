"""CPU ORACLE — test infrastructure only (see oracle/torch_ref.py for the rules).

Restatement of the ECG KAN-FET Neural ODE of the reference (BASELINE configs[2], SURVEY §3.3,
§8f rank 1-2), in the reference's own eager-op order so that on CPU it reproduces the reference
bit for bit (pinned by tests/golden/ecg_*.npz, generated from the reference classes themselves
by tests/golden/make_golden_ecg.py):

  * LogisticBasis (hysteretic, hard branch switch)   train_ecg_kan_fet_nn_ode.py:54-133
      - prev_x (1, in, nb) remembers the LAST ROW of the previous call's batch (:131-132), so
        every row's branch depends on that row of the previous call: the batch is coupled;
      - branch_state = (sigmoid(gate_slope * (x - prev_x)) > 0.5), rebound to (B, in, nb) (:119)
  * KANFeatureMixer: act(LogisticBasis(x)) flattened to (B, in*nb)   :408-421
  * No_MLP_KANODEFunc: Linear(KANFeatureMixer(h))                      :483-509
  * KanFet_NODE: encoder Linear -> odeint(dopri5) on [0, 1] -> dropout -> KANFeatureMixer
    -> Linear                                                          :512-572
The product package never imports this module.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from . import torch_ref as O


class HLogisticParams:
    """Parameters + buffers of the hysteretic LogisticBasis (names = reference state_dict keys)."""

    def __init__(self, k, Ec, Ps, bias, coef, prev_x=None, branch_state=None, gate_slope=5.0,
                 branch_breaking_point=0.5):
        self.k, self.Ec, self.Ps, self.bias, self.coef = k, Ec, Ps, bias, coef
        in_dim, nb = k.shape
        self.prev_x = torch.zeros(1, in_dim, nb, dtype=k.dtype) if prev_x is None else prev_x.clone()
        self.branch_state = (torch.ones(1, in_dim, nb, dtype=k.dtype) if branch_state is None
                             else branch_state.clone())
        self.gate_slope = gate_slope
        self.branch_breaking_point = branch_breaking_point

    @classmethod
    def from_state_dict(cls, sd, prefix="", **kw):
        g = lambda n: sd[prefix + n]
        return cls(g("k"), g("Ec"), g("Ps"), g("bias"), g("coef"), sd.get(prefix + "prev_x"),
                   sd.get(prefix + "branch_state"), **kw)

    def to(self, dtype):
        c = HLogisticParams(*(getattr(self, n).detach().to(dtype) for n in ("k", "Ec", "Ps", "bias", "coef")),
                            self.prev_x.to(dtype), self.branch_state.to(dtype), self.gate_slope,
                            self.branch_breaking_point)
        return c


def hlogistic_forward(x: torch.Tensor, p: HLogisticParams) -> torch.Tensor:
    """LogisticBasis.forward, train_ecg_kan_fet_nn_ode.py:102-133 (use_noise=False); mutates the
    buffers exactly as the module does."""
    if x.dim() != 2 or x.size(1) != p.k.shape[0]:
        raise ValueError(f"x must be (B,{p.k.shape[0]}), got {tuple(x.shape)}")
    nb = p.k.shape[1]
    x_exp = x.unsqueeze(-1).expand(-1, -1, nb)
    up = p.Ps * (1 / (1 + torch.exp(-p.k * (x_exp - p.Ec)))) * 2 - p.Ps
    down = p.Ps * (1 / (1 + torch.exp(-p.k * (x_exp + p.Ec)))) * 2 - p.Ps
    dx = x_exp - p.prev_x
    g = torch.sigmoid(p.gate_slope * dx)
    p.branch_state = (g > p.branch_breaking_point).float()
    basis = p.branch_state * up + (1.0 - p.branch_state) * down + p.bias
    with torch.no_grad():
        p.prev_x.copy_(x_exp[-1:, :, :].detach())
    return basis


def feature_mixer(x: torch.Tensor, p: HLogisticParams) -> torch.Tensor:
    """KANFeatureMixer.forward with act = nn.Sigmoid (:417-421)."""
    phi = hlogistic_forward(x, p)
    phi = torch.sigmoid(phi)
    return phi.reshape(x.size(0), -1)


class ECGFieldRef:
    """No_MLP_KANODEFunc (:483-509) as a callable f(t, h)."""

    def __init__(self, basis: HLogisticParams, proj_w: torch.Tensor, proj_b: torch.Tensor):
        self.basis, self.w, self.b = basis, proj_w, proj_b

    def __call__(self, t, h):
        phi = feature_mixer(h, self.basis)
        dh = F.linear(phi, self.w, self.b)
        assert dh.shape == h.shape, (dh.shape, h.shape)
        return dh

    @classmethod
    def from_state_dict(cls, sd, prefix=""):
        return cls(HLogisticParams.from_state_dict(sd, prefix + "feat.basis."), sd[prefix + "proj.weight"],
                   sd[prefix + "proj.bias"])


class ECGNodeRef:
    """KanFet_NODE.forward (:551-572) in eval mode (dropout = identity)."""

    def __init__(self, sd, solver="dopri5", rtol=1e-3, atol=1e-4):
        self.enc_w, self.enc_b = sd["encoder.weight"], sd["encoder.bias"]
        self.field = ECGFieldRef.from_state_dict(sd, "odefunc.")
        self.cls_basis = HLogisticParams.from_state_dict(sd, "cls_feat.basis.")
        self.cls_w, self.cls_b = sd["cls.weight"], sd["cls.bias"]
        self.solver, self.rtol, self.atol = solver, rtol, atol
        self.trace: Optional[O.Dopri5Trace] = None

    def __call__(self, x):
        h0 = F.linear(x, self.enc_w, self.enc_b)
        t_eval = torch.tensor([0.0, 1.0], dtype=x.dtype)
        self.trace = O.Dopri5Trace()
        h_traj = O.odeint(self.field, h0, t_eval, method=self.solver, rtol=self.rtol, atol=self.atol,
                          trace=self.trace)
        hT = h_traj[-1]
        feat = feature_mixer(hT, self.cls_basis)
        return F.linear(feat, self.cls_w, self.cls_b)


def _ferro_from_sd(sd, prefix):
    p = O.FerroParams.from_state_dict(sd, prefix)
    st = O.FerroState(*p.k.shape, dtype=p.k.dtype)
    if prefix + "prev_x" in sd:
        st.prev_x = sd[prefix + "prev_x"].clone()
    if prefix + "branch_sign" in sd:
        st.branch_sign = sd[prefix + "branch_sign"].clone()
    return p, st


class FerroNetFieldRef:
    """KANFetODEFunc (train_ecg.py:986-1013; the same class at compare_noise_ecg.py:1561-1588):
    h_bound * tanh(h / h_bound) -> FerroelectricBasis(latent -> hidden) -> tanh ->
    FerroelectricBasis(hidden -> latent) -> nan_to_num(0, 1e3, -1e3) -> clamp(-50, 50)."""

    def __init__(self, p1, st1, p2, st2, h_bound=1.0):
        self.p1, self.st1, self.p2, self.st2, self.h_bound = p1, st1, p2, st2, h_bound

    @classmethod
    def from_state_dict(cls, sd, prefix="", h_bound=1.0):
        p1, st1 = _ferro_from_sd(sd, prefix + "fc1.")
        p2, st2 = _ferro_from_sd(sd, prefix + "fc2.")
        return cls(p1, st1, p2, st2, h_bound)

    def __call__(self, t, h):
        if h.dim() == 1:
            h = h.unsqueeze(0)
        h = self.h_bound * torch.tanh(h / self.h_bound)
        z = O.ferro_forward(h, self.p1, self.st1)
        z = torch.tanh(z)
        dh = O.ferro_forward(z, self.p2, self.st2)
        dh = torch.nan_to_num(dh, nan=0.0, posinf=1e3, neginf=-1e3)
        return torch.clamp(dh, -50.0, 50.0)


class FerroNetNodeRef:
    """KanFet_MLP_NODE.forward (train_ecg.py:1043-1059) in eval mode: the reference solves each row
    on its own (batch 1, so the Ferro state carries from row to row) and returns the classifier
    of the LAST row's h(1) only, shape (1, num_classes)."""

    def __init__(self, sd, solver="dopri5", rtol=1e-3, atol=1e-4, h_bound=1.0):
        self.enc_w, self.enc_b = sd["encoder.weight"], sd["encoder.bias"]
        self.field = FerroNetFieldRef.from_state_dict(sd, "odefunc.", h_bound)
        self.cls_w, self.cls_b = sd["cls.weight"], sd["cls.bias"]
        self.solver, self.rtol, self.atol = solver, rtol, atol

    def __call__(self, x):
        h0 = F.linear(x, self.enc_w, self.enc_b)   # :1044, unused like the reference's
        t = torch.tensor([0.0, 1.0], dtype=x.dtype)
        for b in range(x.size(0)):
            h0 = F.linear(x[b:b + 1], self.enc_w, self.enc_b)
            hT = O.odeint(self.field, h0, t, method=self.solver, rtol=self.rtol, atol=self.atol)[-1]
        return F.linear(hT, self.cls_w, self.cls_b)


def ecg_x(batch: int, T: int = 96, seed: int = 0, dtype=torch.float32) -> torch.Tensor:
    """Synthetic ECG200-shaped series (the dataset is not in the image): a seeded sum of two
    sinusoids + noise per row, z-normalised like the UCR files (T = 96)."""
    g = torch.Generator().manual_seed(seed)
    tt = torch.linspace(0, 1, T, dtype=torch.float64)
    f = 1.0 + 3.0 * torch.rand(batch, 1, generator=g, dtype=torch.float64)
    ph = 6.283185307179586 * torch.rand(batch, 1, generator=g, dtype=torch.float64)
    x = torch.sin(6.283185307179586 * f * tt + ph) + 0.3 * torch.sin(18.84955592153876 * f * tt)
    x = x + 0.1 * torch.randn(batch, T, generator=g, dtype=torch.float64)
    x = (x - x.mean(dim=1, keepdim=True)) / x.std(dim=1, keepdim=True)
    return x.to(dtype)
