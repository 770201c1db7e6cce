"""Dispatch from the drop-in modules to libfetode, with autograd wrappers.

Everything here runs HIP kernels through the C ABI; there is no CPU or torch-eager
fallback for the forward maths.  Hysteresis state updates happen exactly once per
forward call, in call order (ferro_class.py:409), whether or not autograd records.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib


def _stream(x):
    return _lib.stream_handle(x.device)


# ---------------------------------------------------------------------------------------------
# plans (pre-transformed parameters, one small kernel per call)
# ---------------------------------------------------------------------------------------------

def build_plan(owner, handle: _lib.FieldHandle, device) -> torch.Tensor:
    lib = _lib.load()
    nbytes = lib.fetode_plan_bytes(handle.ref)
    if nbytes < 0:
        _lib.check(_lib.FETODE_EINVAL, "fetode_plan_bytes")
    n = max(1, nbytes // 4)
    plan = getattr(owner, "_fetode_plan", None)
    if plan is None or plan.numel() < n or plan.device != device:
        plan = torch.empty(n, dtype=torch.float32, device=device)
        owner._fetode_plan = plan
    _lib.check(lib.fetode_plan_build(handle.ref, plan.data_ptr(), _lib.stream_handle(device)),
               "fetode_plan_build")
    return plan


# ---------------------------------------------------------------------------------------------
# KANLinear
# ---------------------------------------------------------------------------------------------

class _KANLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, *params):
        keep = []
        d = mod.desc(keep)
        xc = _lib.f32c(x)
        out = torch.empty(x.shape[0], mod.out_features, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().fetode_kanlinear_forward(_lib.ctypes.byref(d), xc.data_ptr(), x.shape[0],
                                                        out.data_ptr(), _stream(x)), "KANLinear.forward")
        return out

    @staticmethod
    def backward(ctx, grad):
        raise NotImplementedError("KANLinear backward: use the fused odeint path")


def kanlinear_apply(mod, x2d):
    params = [p for p in mod.parameters()]
    return _KANLinearFn.apply(mod, x2d, *params)


# ---------------------------------------------------------------------------------------------
# FerroelectricBasis
# ---------------------------------------------------------------------------------------------

class _FerroFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, reinit, bsign, want_basis, accumulate_into, *params):
        keep = []
        d = mod.desc(keep, bsign)
        xc = _lib.f32c(x)
        B = x.shape[0]
        if accumulate_into is not None:
            out = accumulate_into.clone()
        else:
            out = torch.empty(B, mod.out_dim, device=x.device, dtype=torch.float32)
        basis = (torch.empty(B, mod.in_dim, mod.out_dim, mod.num_basis, device=x.device, dtype=torch.float32)
                 if want_basis else None)
        prev = None if reinit else mod._prev
        _lib.check(_lib.load().fetode_ferro_forward(
            _lib.ctypes.byref(d), xc.data_ptr(), B, _lib.ptr(prev), int(reinit),
            int(accumulate_into is not None), out.data_ptr(), _lib.ptr(basis), None, _stream(x)),
            "FerroelectricBasis.forward")
        if basis is not None:
            ctx.mark_non_differentiable(basis)
        return out, basis

    @staticmethod
    def backward(ctx, grad, gbasis):
        raise NotImplementedError("FerroelectricBasis backward: use the fused odeint path")


def ferro_apply(mod, x, reinit: bool, bsign, want_basis: bool, accumulate_into=None):
    params = [mod.k, mod.Ec, mod.Ps, mod.bias, mod.coef]
    out, basis = _FerroFn.apply(mod, x, reinit, bsign, want_basis, accumulate_into, *params)
    return out, basis


# ---------------------------------------------------------------------------------------------
# whole field (KAN / KANFET) — one stateful evaluation
# ---------------------------------------------------------------------------------------------

def field_layers(model):
    """[(KANLinear, FerroelectricBasis|None)] for KAN and KANFET stacks."""
    out = []
    for l in model.layers:
        if hasattr(l, "kan"):
            out.append((l.kan, l.ferro))
        else:
            out.append((l, None))
    return out


def make_handle(model, B: int, device) -> tuple:
    """Descriptor of the field + the per-layer explicit branch_sign tensors (None = ones)."""
    keep = []
    layers = field_layers(model)
    kan = [k.desc(keep) for k, _ in layers]
    ferro = None
    if layers[0][1] is not None:
        ferro = []
        for _, f in layers:
            b = f._bsign
            if b is not None and (b.shape[0] != B or b.device != device):
                b = None
            ferro.append(f.desc(keep, b))
    return _lib.FieldHandle(kan, ferro, keep)


def pack_state(model, B: int, device):
    """Concatenate the compact prev_x of every Ferro layer into (B, W); init-mask bits for the
    layers whose stored state does not match the batch (ferro_class.py:373-375 rule)."""
    layers = field_layers(model)
    if layers[0][1] is None:
        return None, 0
    cols, mask = [], 0
    for l, (_, f) in enumerate(layers):
        p = f._prev
        if p.shape[0] != B or p.device != device or p.dtype != torch.float32:
            mask |= 1 << l
            cols.append(torch.zeros(B, f.in_dim, device=device, dtype=torch.float32))
        else:
            cols.append(p)
    return torch.cat(cols, dim=1).contiguous(), mask


def unpack_state(model, state: torch.Tensor):
    off = 0
    for _, f in field_layers(model):
        f._prev = state[:, off:off + f.in_dim].contiguous()
        off += f.in_dim
        if f._bsign is not None and f._bsign.shape[0] != state.shape[0]:
            f._bsign = None


class _FieldEvalFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, handle, x, state, mask, *params):
        plan = build_plan(model, handle, x.device)
        out = torch.empty(x.shape[0], field_layers(model)[-1][0].out_features, device=x.device,
                          dtype=torch.float32)
        _lib.check(_lib.load().fetode_field_forward(handle.ref, plan.data_ptr(), x.data_ptr(), x.shape[0],
                                                    _lib.ptr(state), mask, out.data_ptr(), _stream(x)),
                   "field forward")
        return out

    @staticmethod
    def backward(ctx, grad):
        raise NotImplementedError("field backward: use the fused odeint path")


def field_apply(model, x: torch.Tensor) -> torch.Tensor:
    """KAN.forward / KANFET.forward: one evaluation, fused single-launch when the shape has a
    fused kernel, otherwise one HIP kernel per KANLinear / Ferro layer."""
    in0 = field_layers(model)[0][0].in_features
    lead = x.shape[:-1]
    x2 = x.reshape(-1, in0) if model.has_ferro is False else x
    if model.has_ferro and x.dim() != 2:
        raise ValueError("KANFET expects x of shape (B, in_features)")
    _lib.require_gpu_tensor(x2, type(model).__name__ + ".forward")
    x2 = x2.contiguous()
    B = x2.shape[0]
    handle = make_handle(model, B, x2.device)
    lib = _lib.load()
    if lib.fetode_fused_supported(handle.ref):
        state, mask = pack_state(model, B, x2.device)
        params = [p for p in model.parameters()]
        out = _FieldEvalFn.apply(model, handle, x2, state, mask, *params)
        if state is not None:
            unpack_state(model, state)
    else:
        h = x2
        for kan, fer in field_layers(model):
            y = kanlinear_apply(kan, h)
            if fer is not None:
                reinit = fer._needs_reinit(h)
                bsign = fer._branch_sign_for(h)
                y, _ = ferro_apply(fer, h, reinit, bsign, False, accumulate_into=y)
                fer._commit_state(h, reinit)
            h = y
        out = h
    if not model.has_ferro:
        out = out.reshape(*lead, out.shape[-1])
    return out
