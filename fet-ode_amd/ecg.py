"""Drop-in ECG KAN-FET Neural ODE modules (BASELINE configs[2]).

Reference: train_ecg_kan_fet_nn_ode.py
  * LogisticBasis          :54-133  hysteretic logistic basis with a HARD branch switch:
                                    branch_state = sigmoid(gate_slope (x - prev_x)) > 0.5 picks
                                    the up (centred at +Ec) or down (-Ec) logistic; prev_x
                                    remembers the LAST ROW of the previous call's batch
  * KANFeatureMixer        :408-421  act(LogisticBasis(x)) flattened to (B, dim*num_basis)
  * No_MLP_KANODEFunc      :483-509  dh/dt = Linear(KANFeatureMixer(h))   (the dopri5 field)
  * KanFet_NODE            :512-572  encoder Linear -> odeint(dopri5, [0, 1]) -> dropout ->
                                    KANFeatureMixer -> Linear
Reference: train_ecg.py (the FerroElectricNet field)
  * KANFetODEFunc          :986-1013  h_bound tanh(h / h_bound) -> FerroelectricBasis(latent ->
                                    hidden, K) -> tanh -> FerroelectricBasis(hidden -> latent, K)
                                    -> nan_to_num -> clamp(-50, 50)
  * KanFet_MLP_NODE        :1017-1059 per-row batch-1 solves, classifier of the last row

Same constructor arguments, parameter names / shapes / init RNG order, buffers (prev_x (1, in,
nb); branch_state, rebound to (B, in, nb) by every call like the reference) and error types.
The mixer (+ Linear head) is one HIP launch per call (fetode_hlogistic_mixer_forward) with a HIP
VJP; the encoder / classifier Linear layers are plain library GEMMs (torch).  There is no CPU
path.  Not provided: use_noise=True (random).  Backprop through dopri5 works like torchdiffeq's
direct backprop (dopri5._Dopri5Grad: every stage, error ratio and step size, with the mixer's HIP
VJP per evaluation); the device-resident solve serves inference only.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import _lib
from ._lib import CacheFreeState
from .ferro_class import FerroelectricBasis
from .odeint import odeint

_PARAMS = ("k", "Ec", "Ps", "bias")


def _stream(x):
    return _lib.stream_handle(x.device)


class _HMixerFn(torch.autograd.Function):
    """basis -> [sigmoid] -> [Linear head] in one launch; prev_x / branch_state updated in place
    exactly once per call (train_ecg_kan_fet_nn_ode.py:119, :131-132)."""

    @staticmethod
    def forward(ctx, mod, x, act_sigmoid, training, w, b, *params):
        lib = _lib.load()
        keep = []
        d = mod.desc(keep)
        xc = _lib.f32c(x)
        B = xc.shape[0]
        F = mod.in_dim * mod.num_basis
        dev = x.device
        prev = mod._prev_for(dev)
        prev_read = prev.clone() if training else prev
        head = w is not None
        need_phi = training or not head
        phi = torch.empty(B, F, device=dev, dtype=torch.float32) if need_phi else None
        out = torch.empty(B, w.shape[0], device=dev, dtype=torch.float32) if head else None
        branch = torch.empty(B, mod.in_dim, mod.num_basis, device=dev, dtype=torch.float32)
        wc = _lib.f32c(w) if head else None
        bc = _lib.f32c(b) if b is not None else None
        _lib.check(lib.fetode_hlogistic_mixer_forward(
            _lib.ctypes.byref(d), xc.data_ptr(), B, prev.data_ptr(), int(act_sigmoid), _lib.ptr(wc), _lib.ptr(bc),
            int(w.shape[0]) if head else 0, _lib.ptr(phi), _lib.ptr(out), branch.data_ptr(), prev.data_ptr(),
            _stream(x)), "KANFeatureMixer.forward")
        mod.branch_state = branch
        ctx.mod, ctx.act_sigmoid, ctx.head = mod, act_sigmoid, head
        if training:
            ctx.save_for_backward(xc, prev_read, phi, wc)
        if head:
            return out
        return phi

    @staticmethod
    def backward(ctx, g):
        lib = _lib.load()
        xc, prev, phi, wc = ctx.saved_tensors
        mod = ctx.mod
        keep = []
        d = mod.desc(keep)
        B = xc.shape[0]
        gc = _lib.f32c(g)
        want = ctx.needs_input_grad
        gx = torch.empty_like(xc) if want[1] else None
        gw = torch.empty_like(wc) if (ctx.head and want[4]) else None
        gbh = torch.empty(wc.shape[0], device=xc.device) if (ctx.head and want[5]) else None
        gp = [torch.empty(mod.in_dim, mod.num_basis, device=xc.device) if want[6 + i] else None
              for i in range(len(_PARAMS))]
        ws = None
        if ctx.head:
            nb = lib.fetode_hlogistic_mixer_backward_workspace(_lib.ctypes.byref(d), B)
            ws = torch.empty(max(1, nb // 4), device=xc.device, dtype=torch.float32)
        _lib.check(lib.fetode_hlogistic_mixer_backward(
            _lib.ctypes.byref(d), xc.data_ptr(), B, prev.data_ptr(), int(ctx.act_sigmoid), phi.data_ptr(),
            _lib.ptr(wc), int(wc.shape[0]) if ctx.head else 0, gc.data_ptr(), _lib.ptr(gx), _lib.ptr(gw),
            _lib.ptr(gbh), *[_lib.ptr(t) for t in gp], _lib.ptr(ws), _stream(xc)), "KANFeatureMixer backward")
        return (None, gx, None, None, gw, gbh, *gp)


def _mixer_apply(basis: "LogisticBasis", x, act_sigmoid: bool, w=None, b=None):
    params = [getattr(basis, n) for n in _PARAMS]
    training = torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in [x, w, b, *params])
    return _HMixerFn.apply(basis, x, act_sigmoid, training, w, b, *params)


class LogisticBasis(CacheFreeState, nn.Module):
    """Hysteretic logistic basis, train_ecg_kan_fet_nn_ode.py:54-133."""

    # per-batch state (rebound to (B, in, nb) every call): never broadcast across ranks
    _rank_local_buffers = ("prev_x", "branch_state")

    def __init__(self, in_dim: int, num_basis: int, gate_slope: float = 5.0, init_prev: float = 0.0,
                 eps: float = 1e-6, branch_breaking_point=0.5, use_noise=False, noise_std=0.05):
        super().__init__()
        self.in_dim = in_dim
        self.num_basis = num_basis
        self.gate_slope = gate_slope
        self.eps = eps
        self.use_noise = use_noise
        self.noise_std = noise_std
        self.branch_breaking_point = branch_breaking_point
        # same init distributions and RNG order as :84-88
        self.k = nn.Parameter(torch.rand(in_dim, num_basis) * 2 + 0.5)
        self.Ec = nn.Parameter(torch.rand(in_dim, num_basis) * 2 + 0.5)
        self.Ps = nn.Parameter(torch.rand(in_dim, num_basis) * 1.5 + 0.5)
        self.bias = nn.Parameter(torch.randn(in_dim, num_basis) * 0.1)
        self.coef = nn.Parameter(torch.randn(in_dim, num_basis))
        self.register_buffer("prev_x", torch.zeros(1, in_dim, num_basis))
        self.register_buffer("branch_state", torch.ones(1, in_dim, num_basis))

    def reset_state(self, value: float = 0.0):
        """:96-99 (``value`` is ignored there too)."""
        self.prev_x.zero_()
        self.branch_state.fill_(1.0)

    def desc(self, keep: list) -> _lib.HLogisticDesc:
        def p(t):
            t = _lib.f32c(t)
            keep.append(t)
            return t.data_ptr()
        return _lib.HLogisticDesc(self.in_dim, self.num_basis, p(self.k), p(self.Ec), p(self.Ps), p(self.bias),
                                  float(self.gate_slope), float(self.branch_breaking_point))

    def _prev_for(self, dev) -> torch.Tensor:
        """prev_x as the contiguous fp32 (1, in, nb) tensor the kernel reads and rewrites."""
        p = self.prev_x
        if p.device != dev or p.dtype != torch.float32 or not p.is_contiguous() or p.shape[0] != 1:
            self.prev_x = p.to(device=dev, dtype=torch.float32).contiguous()[-1:]
        return self.prev_x

    def _check(self, x):
        if x.dim() != 2 or x.size(1) != self.in_dim:
            raise ValueError(f"x must be (B,{self.in_dim}), got {tuple(x.shape)}")
        if self.use_noise:
            raise NotImplementedError("use_noise=True (random basis noise) is not on the hot path")
        _lib.require_gpu_tensor(x, "LogisticBasis.forward")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """(B, in) -> basis (B, in, num_basis)."""
        self._check(x)
        return _mixer_apply(self, x, False).view(x.shape[0], self.in_dim, self.num_basis)


class KANFeatureMixer(CacheFreeState, nn.Module):
    """:408-421 — act(LogisticBasis(x)) as (B, dim*num_basis); act = Sigmoid runs in the kernel."""

    def __init__(self, dim, num_basis, act=nn.Sigmoid()):
        super().__init__()
        self.basis = LogisticBasis(dim, num_basis)
        self.act = act

    def forward(self, x):
        self.basis._check(x)
        if isinstance(self.act, nn.Sigmoid):
            return _mixer_apply(self.basis, x, True)
        phi = self.act(self.basis(x))
        return phi.reshape(x.size(0), -1)


class No_MLP_KANODEFunc(CacheFreeState, nn.Module):
    """:483-509 — dh/dt = Linear(KANFeatureMixer(h)); mixer + head in one launch."""

    def __init__(self, latent_dim=64, num_basis=10, hidden=128):
        super().__init__()
        self.latent_dim = latent_dim
        self.num_basis = num_basis
        self.feat = KANFeatureMixer(latent_dim, num_basis, act=nn.Sigmoid())
        self.proj = nn.Linear(latent_dim * num_basis, latent_dim)
        nn.init.zeros_(self.proj.bias)
        nn.init.normal_(self.proj.weight, mean=0.0, std=0.01)

    def forward(self, t, h):
        self.feat.basis._check(h)
        if isinstance(self.feat.act, nn.Sigmoid):
            dh = _mixer_apply(self.feat.basis, h, True, self.proj.weight, self.proj.bias)
        else:
            dh = self.proj(self.feat(h))
        assert dh.shape == h.shape, (dh.shape, h.shape)
        return dh


class KanFet_NODE(CacheFreeState, nn.Module):
    """:512-572 — encode (B, T) to h0, integrate on [0, 1] with dopri5, decode h(1) -> logits."""

    def __init__(self, T: int, num_classes: int, latent_dim: int = 64, num_basis: int = 10,
                 ode_hidden: int = 128, dropout: float = 0.1, solver: str = "dopri5", rtol: float = 1e-3,
                 atol: float = 1e-4):
        super().__init__()
        self.T = T
        self.num_classes = num_classes
        self.latent_dim = latent_dim
        self.solver = solver
        self.rtol = rtol
        self.atol = atol
        self.encoder = nn.Linear(T, latent_dim)
        self.odefunc = No_MLP_KANODEFunc(latent_dim=latent_dim, num_basis=num_basis, hidden=ode_hidden)
        self.dropout = nn.Dropout(dropout)
        self.cls_feat = KANFeatureMixer(latent_dim, num_basis, act=nn.Sigmoid())
        self.cls = nn.Linear(latent_dim * num_basis, num_classes)
        self.last_solve: Optional[object] = None

    def forward(self, x):
        _lib.require_gpu_tensor(x, "KanFet_NODE.forward")
        from .dopri5 import deferred_status, dopri5_solve
        # the solve's status is read once, after the classifier is launched too (deferred_status):
        # a failed solve still raises from this forward, but the host issues the whole forward
        # without waiting for the solve in between
        with deferred_status():
            h0 = self.encoder(x)
            # the reference builds t on x's device; odeint reads the grid on the host, so it is
            # built there (same values and dtype, no device round trip), once per dtype
            t_eval = self.__dict__.get("_t_eval")
            if t_eval is None or t_eval.dtype != x.dtype:
                t_eval = torch.tensor([0.0, 1.0], dtype=x.dtype)
                self.__dict__["_t_eval"] = t_eval
            h_traj = odeint(self.odefunc, h0, t_eval, method=self.solver, rtol=self.rtol, atol=self.atol)
            if self.solver == "dopri5":
                self.last_solve = getattr(dopri5_solve, "last", None)
            hT = h_traj[-1]
            hT = self.dropout(hT)
            feat = self.cls_feat(hT)
            return self.cls(feat)


# ---------------------------------------------------------------------------------------------
# The FerroElectricNet field of train_ecg.py: FerroelectricBasis layers (HIP, fetode_ferro_*)
# joined by HIP elementwise stages (fetode_ferronet.hip) with HIP VJPs
# ---------------------------------------------------------------------------------------------

class _TanhBoundFn(torch.autograd.Function):
    """h_bound * tanh(h / h_bound) (train_ecg.py:1002)."""

    @staticmethod
    def forward(ctx, x, hb, training):
        lib = _lib.load()
        xc = _lib.f32c(x)
        out = torch.empty_like(xc)
        t = torch.empty_like(xc) if training else None
        _lib.check(lib.fetode_tanh_bound(xc.numel(), float(hb), xc.data_ptr(), out.data_ptr(), _lib.ptr(t),
                                         _stream(xc)), "KANFetODEFunc h_bound")
        if training:
            ctx.save_for_backward(t)
            ctx.hb = hb
        return out

    @staticmethod
    def backward(ctx, g):
        (t,) = ctx.saved_tensors
        gc = _lib.f32c(g)
        gx = torch.empty_like(gc)
        _lib.check(_lib.load().fetode_tanh_bound_backward(gc.numel(), float(ctx.hb), gc.data_ptr(), t.data_ptr(),
                                                          gx.data_ptr(), _stream(gc)), "KANFetODEFunc h_bound backward")
        return gx, None, None


class _TanhFn(torch.autograd.Function):
    """nn.Tanh between the Ferro layers (:1004)."""

    @staticmethod
    def forward(ctx, x, training):
        xc = _lib.f32c(x)
        out = torch.empty_like(xc)
        _lib.check(_lib.load().fetode_tanh(xc.numel(), xc.data_ptr(), out.data_ptr(), _stream(xc)), "tanh")
        if training:
            ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        gc = _lib.f32c(g)
        gx = torch.empty_like(gc)
        _lib.check(_lib.load().fetode_tanh_backward(gc.numel(), gc.data_ptr(), y.data_ptr(), gx.data_ptr(),
                                                    _stream(gc)), "tanh backward")
        return gx, None


_NAN_CLAMP = (0.0, 1e3, -1e3, -50.0, 50.0)   # nan_to_num(nan, posinf, neginf), clamp(lo, hi): :1008-1011


class _NanClampFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, training):
        xc = _lib.f32c(x)
        out = torch.empty_like(xc)
        _lib.check(_lib.load().fetode_nan_clamp(xc.numel(), *_NAN_CLAMP, xc.data_ptr(), out.data_ptr(), _stream(xc)),
                   "nan_to_num / clamp")
        if training:
            ctx.save_for_backward(xc)
        return out

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        gc = _lib.f32c(g)
        gx = torch.empty_like(gc)
        _lib.check(_lib.load().fetode_nan_clamp_backward(gc.numel(), *_NAN_CLAMP, gc.data_ptr(), x.data_ptr(),
                                                         gx.data_ptr(), _stream(gc)), "nan_to_num / clamp backward")
        return gx, None


def _grad_on(x):
    return torch.is_grad_enabled() and x.requires_grad


class KANFetODEFunc(CacheFreeState, nn.Module):
    """train_ecg.py:986-1013 (compare_noise_ecg.py:1561-1588): the FerroElectricNet ODE field.
    fc1 / fc2 are the drop-in FerroelectricBasis (same RNG order, buffers and state rules)."""

    def __init__(self, latent_dim: int, hidden_dim: int, num_basis: int, h_bound: float = 1.0):
        super().__init__()
        self.h_bound = h_bound
        self.fc1 = FerroelectricBasis(latent_dim, hidden_dim, num_basis)
        self.act = nn.Tanh()
        self.fc2 = FerroelectricBasis(hidden_dim, latent_dim, num_basis)

    def forward(self, t, h):
        if h.dim() == 1:
            h = h.unsqueeze(0)
        _lib.require_gpu_tensor(h, "KANFetODEFunc.forward")
        h = _TanhBoundFn.apply(h, float(self.h_bound), _grad_on(h))
        z = self.fc1(h)
        z = _TanhFn.apply(z, _grad_on(z)) if isinstance(self.act, nn.Tanh) else self.act(z)
        dh = self.fc2(z)
        return _NanClampFn.apply(dh, _grad_on(dh))


class KanFet_MLP_NODE(CacheFreeState, nn.Module):
    """train_ecg.py:1017-1059, as the reference runs it: every row is solved on its own with batch
    1 (the Ferro state carries from row to row) and the classifier of the LAST row's h(1) is
    returned, shape (1, num_classes)."""

    def __init__(self, T: int, num_classes: int, latent_dim: int = 64, num_basis: int = 10,
                 ode_hidden: int = 128, dropout: float = 0.1, solver: str = "dopri5", rtol: float = 1e-3,
                 atol: float = 1e-4):
        super().__init__()
        self.T = T
        self.num_classes = num_classes
        self.latent_dim = latent_dim
        self.solver = solver
        self.rtol = rtol
        self.atol = atol
        self.encoder = nn.Linear(T, latent_dim)
        self.odefunc = KANFetODEFunc(latent_dim=latent_dim, hidden_dim=ode_hidden, num_basis=num_basis)
        self.dropout = nn.Dropout(dropout)
        self.cls = nn.Linear(latent_dim, num_classes)

    def forward(self, x):
        _lib.require_gpu_tensor(x, "KanFet_MLP_NODE.forward")
        h0 = self.encoder(x)
        t = torch.tensor([0.0, 1.0], dtype=x.dtype)   # host grid: same values as the reference's
        for b in range(x.size(0)):
            xb = x[b:b + 1]
            h0 = self.encoder(xb)
            hT = odeint(self.odefunc, h0, t, method=self.solver, rtol=self.rtol, atol=self.atol)[-1]
            hT = self.dropout(hT)
        return self.cls(hT)
