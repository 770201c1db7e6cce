"""Dispatch from the drop-in modules to libfetode, with autograd wrappers.

Everything here runs HIP kernels through the C ABI; there is no CPU or torch-eager
fallback for the forward or backward maths.  Hysteresis state updates happen exactly once
per forward call, in call order (ferro_class.py:409), whether or not autograd records; the
state is a detached snapshot in the reference (:381-382), so it carries no gradient.
"""
from __future__ import annotations

import os

from typing import List, Optional

import torch

from . import _lib


def _stream(x):
    return _lib.stream_handle(x.device)


def axpby(a: float, x: torch.Tensor, b: float = 0.0, y: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a*x + b*y on the GPU (HIP)."""
    x = x.contiguous()
    out = torch.empty_like(x)
    _lib.check(_lib.load().fetode_axpby(x.numel(), float(a), x.data_ptr(), float(b), _lib.ptr(
        None if y is None else y.contiguous()), out.data_ptr(), _stream(x)), "fetode_axpby")
    return out


def grad_enabled_for(*tensors) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


# ---------------------------------------------------------------------------------------------
# plans (pre-transformed parameters, one small kernel per call)
# ---------------------------------------------------------------------------------------------

_PLAN_CACHE = os.environ.get("FETODE_NO_PLAN_CACHE", "0") != "1"


def build_plan(owner, handle: _lib.FieldHandle, device) -> torch.Tensor:
    """The pre-transformed parameters of the field (fetode_plan_build).  Rebuilt whenever the
    parameter values may have changed (handle.vkey: version counters + optimizer-step generation),
    i.e. after optimizer steps (fused ones included), load_state_dict and in-place updates.  Writes through `.data`
    bypass version counters; call `owner._fetode_handle = None` after those (or set
    FETODE_NO_PLAN_CACHE=1 to rebuild on every solve)."""
    plan = getattr(owner, "_fetode_plan", None)
    pfor = getattr(owner, "_fetode_plan_for", None)
    vkey = getattr(handle, "vkey", None)
    if _PLAN_CACHE and plan is not None and vkey is not None and pfor is not None and pfor[0] is handle \
            and pfor[1] == vkey:
        return plan
    lib = _lib.load()
    nbytes = lib.fetode_plan_bytes(handle.ref)
    if nbytes < 0:
        _lib.check(_lib.FETODE_EINVAL, "fetode_plan_bytes")
    n = max(1, nbytes // 4)
    plan = getattr(owner, "_fetode_plan", None)
    # a plan a pending backward still reads (pin_plan) is never rebuilt in place: the rebuild gets a
    # fresh buffer and the pinned one lives on in that backward's context
    if plan is None or plan.numel() < n or plan.device != device or owner.__dict__.get("_fetode_plan_pin") is plan:
        plan = torch.empty(n, dtype=torch.float32, device=device)
        owner._fetode_plan = plan
    _lib.check(lib.fetode_plan_build(handle.ref, plan.data_ptr(), _lib.stream_handle(device)),
               "fetode_plan_build")
    owner._fetode_plan_for = (handle, vkey)
    return plan


def pin_plan(owner, plan: torch.Tensor) -> torch.Tensor:
    """Keep `plan` unchanged for a backward that runs after later solves (build_plan then
    rebuilds into a new buffer instead of this one): no per-iteration copy of the plan."""
    owner.__dict__["_fetode_plan_pin"] = plan
    return plan


# ---------------------------------------------------------------------------------------------
# KANLinear
# ---------------------------------------------------------------------------------------------

KAN_PARAM_NAMES = ("base_weight", "spline_weight", "spline_scaler", "logistic_a", "logistic_b",
                   "logistic_weight", "logistic_scaler")


def kan_params(mod) -> List[Optional[torch.Tensor]]:
    lg = mod.enable_logistic_basis
    return [mod.base_weight, mod.spline_weight,
            mod.spline_scaler if mod.enable_standalone_scale_spline else None,
            mod.logistic_basis.a if lg else None, mod.logistic_basis.b if lg else None,
            mod.logistic_weight if lg else None,
            mod.logistic_scaler if lg and mod.enable_standalone_scale_logistic else None]


class _KANLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, *params):
        keep = []
        d = mod.desc(keep)
        xc = _lib.f32c(x)
        out = torch.empty(x.shape[0], mod.out_features, device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().fetode_kanlinear_forward(_lib.ctypes.byref(d), xc.data_ptr(), x.shape[0],
                                                        out.data_ptr(), _stream(x)), "KANLinear.forward")
        ctx.mod = mod
        ctx.save_for_backward(xc)
        return out

    @staticmethod
    def backward(ctx, grad):
        (xc,) = ctx.saved_tensors
        mod = ctx.mod
        gx, grads = kan_backward(mod, xc, grad, ctx.needs_input_grad[1], ctx.needs_input_grad[2:])
        return (None, gx, *grads)


def kan_backward(mod, xc, grad, want_x, want_params, gx_accum=None, out=None, entry=None):
    """HIP VJP of KANLinear: returns (gx, [grad per KAN_PARAM_NAMES or None]).  At the wide-layer
    widths with 64 / 128 outputs (ETT / ECG fields) the MFMA VJP (fetode_kanlinear_backward_wide);
    otherwise the generic kernels.  `out`: zero-filled tensors (per KAN_PARAM_NAMES) the parameter
    gradients are written into instead of fresh ones."""
    if mod.out_features in (64, 128) and mod.in_features >= 16 and (want_x or any(want_params)):
        r = _kan_backward_wide(mod, xc, grad, want_x, want_params, gx_accum, out, entry)
        if r is not None:
            return r
    return _kan_backward_generic(mod, xc, grad, want_x, want_params, gx_accum, out)


def _grad_bufs(params, want, alloc, out):
    """Per-parameter gradient buffers: out[k] (zero-filled, given by the caller) or alloc(p)."""
    return [None if (p is None or not w) else (alloc(p) if out is None else out[k])
            for k, (p, w) in enumerate(zip(params, want))]


def _kan_backward_wide(mod, xc, grad, want_x, want_params, gx_accum=None, out=None, entry=None):
    if entry is None:
        entry = wide_plan(mod, None, xc.device)
    if entry is None:
        return None
    plan, kd, _, _ = entry
    lib = _lib.load()
    B = xc.shape[0]
    g = _lib.f32c(grad)
    if g.data_ptr() % 16:
        g = g.clone()
    gx = None
    if want_x:
        gx = torch.empty_like(xc) if gx_accum is None else gx_accum
    alloc = torch.empty_like if gx_accum is None else torch.zeros_like
    grads = _grad_bufs(kan_params(mod), want_params, alloc, out)
    any_param = any(t is not None for t in grads)
    gstruct = _lib.KANLinearGrad(*[_lib.ptr(t) for t in grads]) if any_param else None
    nb = lib.fetode_kanlinear_backward_wide_workspace(_lib.ctypes.byref(kd), None, B)
    if nb < 0:
        return None
    ws = torch.empty(max(1, nb // 4), device=xc.device, dtype=torch.float32)
    _lib.check(lib.fetode_kanlinear_backward_wide(
        _lib.ctypes.byref(kd), None, plan.data_ptr(), xc.data_ptr(), B, g.data_ptr(), _lib.ptr(gx),
        _lib.ctypes.byref(gstruct) if any_param else None, int(gx_accum is not None), ws.data_ptr(), _stream(xc)),
        "KANLinear backward (wide)")
    return gx, grads


def _kan_backward_generic(mod, xc, grad, want_x, want_params, gx_accum=None, out=None):
    lib = _lib.load()
    keep = []
    d = mod.desc(keep)
    g = _lib.f32c(grad)
    B = xc.shape[0]
    gx = None
    if want_x:
        gx = torch.empty_like(xc) if gx_accum is None else gx_accum
    params = kan_params(mod)
    grads = _grad_bufs(params, want_params, torch.zeros_like, out)
    any_param = any(t is not None for t in grads)
    gstruct = _lib.KANLinearGrad(*[_lib.ptr(t) for t in grads]) if any_param else None
    ws = None
    if any_param:
        nb = lib.fetode_kanlinear_backward_workspace(_lib.ctypes.byref(d))
        ws = torch.empty(max(1, nb // 4), device=xc.device, dtype=torch.float32)
    _lib.check(lib.fetode_kanlinear_backward(
        _lib.ctypes.byref(d), xc.data_ptr(), B, g.data_ptr(), _lib.ptr(gx),
        _lib.ctypes.byref(gstruct) if any_param else None, _lib.ptr(ws),
        int(gx_accum is not None), _stream(xc)), "KANLinear backward")
    return gx, grads


def kanlinear_apply(mod, x2d):
    if not grad_enabled_for(x2d, *[p for p in kan_params(mod) if p is not None]):
        out = wide_apply(mod, None, _lib.f32c(x2d))   # production widths: the MFMA wide-layer kernel
        if out is not None:
            return out
    return _KANLinearFn.apply(mod, x2d, *kan_params(mod))


# ---------------------------------------------------------------------------------------------
# FerroelectricBasis
# ---------------------------------------------------------------------------------------------

FERRO_PARAM_NAMES = ("k", "Ec", "Ps", "bias", "coef")


class _FerroFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, reinit, bsign, want_basis, accumulate_into, *params):
        keep = []
        d = mod.desc(keep, bsign)
        xc = _lib.f32c(x)
        B = x.shape[0]
        if accumulate_into is not None:
            out = accumulate_into.detach().clone()
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
        ctx.mod, ctx.reinit, ctx.bsign = mod, reinit, bsign
        # the module's prev_x is overwritten right after this call: keep the snapshot
        ctx.save_for_backward(xc, None if prev is None else prev.detach().clone())
        return out, basis

    @staticmethod
    def backward(ctx, grad, gbasis):
        xc, prev = ctx.saved_tensors
        gx, grads = ferro_backward(ctx.mod, xc, prev, ctx.reinit, ctx.bsign, grad, ctx.needs_input_grad[1],
                                   ctx.needs_input_grad[6:])
        gacc = grad if ctx.needs_input_grad[5] else None
        return (None, gx, None, None, None, gacc, *grads)


def ferro_backward(mod, xc, prev, reinit, bsign, grad, want_x, want_params, gx_accum=None, out=None, entry=None):
    """HIP VJP of FerroelectricBasis: returns (gx, [grad per FERRO_PARAM_NAMES or None]).  At the
    wide-layer widths (ETT / ECG fields) with the constant branch sign, one pass over the element
    evaluations gives both (fetode_ferro_backward_wide); otherwise the generic two-kernel VJP."""
    if bsign is None and mod.in_dim >= 16 and mod.out_dim >= 16 and (want_x or any(want_params)):
        r = _ferro_backward_wide(mod, xc, prev, reinit, grad, want_x, want_params, gx_accum, out, entry)
        if r is not None:
            return r
    return _ferro_backward_generic(mod, xc, prev, reinit, bsign, grad, want_x, want_params, gx_accum, out)


def _ferro_backward_generic(mod, xc, prev, reinit, bsign, grad, want_x, want_params, gx_accum=None, out=None):
    lib = _lib.load()
    keep = []
    d = mod.desc(keep, bsign)
    g = _lib.f32c(grad)
    gx = None
    if want_x:
        gx = torch.empty_like(xc) if gx_accum is None else gx_accum
    params = [getattr(mod, n) for n in FERRO_PARAM_NAMES]
    grads = _grad_bufs(params, want_params, torch.zeros_like, out)
    any_param = any(t is not None for t in grads)
    gstruct = _lib.FerroGrad(*[_lib.ptr(t) for t in grads]) if any_param else None
    _lib.check(lib.fetode_ferro_backward(
        _lib.ctypes.byref(d), xc.data_ptr(), xc.shape[0], _lib.ptr(prev), int(reinit), g.data_ptr(),
        _lib.ptr(gx), _lib.ctypes.byref(gstruct) if any_param else None, int(gx_accum is not None),
        _stream(xc)), "FerroelectricBasis backward")
    return gx, grads


def _ferro_backward_wide(mod, xc, prev, reinit, grad, want_x, want_params, gx_accum, out=None, entry=None):
    if entry is None:
        entry = wide_plan(None, mod, xc.device)
    if entry is None:
        return None
    plan, _, fd, _ = entry
    lib = _lib.load()
    B = xc.shape[0]
    g = _lib.f32c(grad)
    gx = None
    if want_x:
        gx = torch.empty_like(xc) if gx_accum is None else gx_accum
    params = [getattr(mod, n) for n in FERRO_PARAM_NAMES]
    # accumulate applies to d/dx and the parameter sums alike: accumulating parameter sums start at 0
    alloc = torch.empty_like if gx_accum is None else torch.zeros_like
    grads = _grad_bufs(params, want_params, alloc, out)
    any_param = any(t is not None for t in grads)
    gstruct = _lib.FerroGrad(*[_lib.ptr(t) for t in grads]) if any_param else None
    nb = lib.fetode_ferro_backward_wide_workspace(_lib.ctypes.byref(fd), B)
    ws = torch.empty(max(1, nb // 4), device=xc.device, dtype=torch.float32)
    _lib.check(lib.fetode_ferro_backward_wide(
        _lib.ctypes.byref(fd), plan.data_ptr(), xc.data_ptr(), B, _lib.ptr(None if reinit else prev), int(reinit),
        g.data_ptr(), _lib.ptr(gx), _lib.ctypes.byref(gstruct) if any_param else None,
        int(gx_accum is not None), ws.data_ptr(), _stream(xc)), "FerroelectricBasis backward (wide)")
    return gx, grads


def ferro_apply(mod, x, reinit: bool, bsign, want_basis: bool, accumulate_into=None):
    params = [getattr(mod, n) for n in FERRO_PARAM_NAMES]
    if (bsign is None and not want_basis and accumulate_into is None
            and not grad_enabled_for(x, *params)):
        out = wide_apply(None, mod, _lib.f32c(x), reinit=reinit)   # production widths: wide-layer kernel
        if out is not None:
            return out, None
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


def _field_tensors(model):
    """Every tensor a field descriptor points at, read straight from the modules' parameter /
    buffer dicts (nn.Module.__getattr__ costs ~0.3 us per access; this runs on every solve)."""
    ts = []
    for l in model.layers.__dict__["_modules"].values():
        md = l.__dict__["_modules"]
        k, f = (md["kan"], md["ferro"]) if "kan" in md else (l, None)
        kp, kb = k.__dict__["_parameters"], k.__dict__["_buffers"]
        ts.append(kb["grid"])
        ts += [t for t in kp.values() if t is not None]
        lb = k.__dict__["_modules"].get("logistic_basis")
        if lb is not None:
            ts += [t for t in lb.__dict__["_parameters"].values() if t is not None]
        if f is not None:
            ts += [t for t in f.__dict__["_parameters"].values() if t is not None]
            b = f.__dict__["_buffers"].get("_bsign")
            if b is not None:
                ts.append(b)
    return ts


def _handle_key(model, B, device):
    """(descriptor key, value key) of the field, or None when a tensor would be converted
    (non-fp32 / non-contiguous: the converted copy could go stale silently).  The descriptor holds
    only pointers and shapes, so it is reused while every tensor keeps its storage; the plan holds
    the parameter VALUES and is rebuilt when a version counter or the optimizer-step generation
    (_lib.param_generation: fused optimizers do not bump version counters) changes."""
    ts = _field_tensors(model)
    key = [B, device]
    vkey = [_lib.param_generation()]
    kapp, vapp = key.append, vkey.append
    for t in ts:
        kapp(t.data_ptr())
        kapp(t.shape[0])
        kapp(t.dtype)
        kapp(t.stride())
        vapp(t._version)
    key = tuple(key)
    # dtype / layout are in the key (cheap attribute reads), so a restride (t_(), as_strided_) or a
    # set_() onto another dtype at the same address makes a new key, which is checked here once
    cached = model.__dict__.get("_fetode_keyok")
    if cached is None or cached[0] != key:
        ok = all(t.dtype == torch.float32 and t.is_contiguous() for t in ts)
        model.__dict__["_fetode_keyok"] = (key, ok)
    elif not cached[1]:
        ok = False
    else:
        ok = True
    return (key, tuple(vkey)) if ok else None


def make_handle(model, B: int, device) -> _lib.FieldHandle:
    """Descriptor of the field (+ explicit branch_sign tensors; None = ones), cached on the model
    while every tensor keeps its storage; handle.vkey identifies the parameter values it was
    asked for (build_plan rebuilds the plan when it changes)."""
    keys = _handle_key(model, B, device)
    cached = model.__dict__.get("_fetode_handle")
    if keys is not None and cached is not None and cached[0] == keys[0]:
        h = cached[1]
        h.vkey = keys[1]
        return h
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
    h = _lib.FieldHandle(kan, ferro, keep)
    h.vkey = None if keys is None else keys[1]   # None: never reuse a plan built for it
    model._fetode_handle = (None if keys is None else keys[0], h)
    return h


def _state_views(buf, model, B):
    """The per-layer (B, in_l) views of the state buffer, made once per buffer (slicing and
    view() cost a few us each on every solve otherwise)."""
    cached = model.__dict__.get("_fetode_views")
    if cached is not None and cached[0] is buf and cached[1] == B:
        return cached[2]
    views, off = [], 0
    for _, f in field_layers(model):
        views.append(buf[B * off:B * (off + f.in_dim)].view(B, f.in_dim))
        off += f.in_dim
    model.__dict__["_fetode_views"] = (buf, B, views)
    return views


def _ferro_modules(model):
    return [l.__dict__["_modules"]["ferro"] for l in model.layers.__dict__["_modules"].values()]


def pack_state(model, B: int, device):
    """The fused kernels read/write the hysteresis state of all Ferro layers in one buffer laid
    out as contiguous (B, in_l) blocks (include/fetode.h).  Each layer's compact prev_x IS a view
    of that buffer between calls, so packing costs nothing in steady state.  Returns the buffer
    and the init-mask bits of the layers whose stored state does not match the batch
    (ferro_class.py:373-375 re-initialisation rule)."""
    if not model.has_ferro:
        return None, 0
    fs = _ferro_modules(model)
    W = sum(f.in_dim for f in fs)
    buf = model.__dict__.get("_fetode_state")
    if buf is None or buf.numel() != B * W or buf.device != device:
        buf = torch.zeros(B * W, device=device, dtype=torch.float32)
        model._fetode_state = buf
    mask = 0
    for l, (f, v) in enumerate(zip(fs, _state_views(buf, model, B))):
        bufs = f.__dict__["_buffers"]
        p = bufs["_prev"]
        if p is v:   # steady state: the layer's prev_x already is this view
            continue
        if p.shape[0] != B or p.device != device or p.dtype != torch.float32:
            mask |= 1 << l
        elif p.data_ptr() != v.data_ptr():
            v.copy_(p)
        bufs["_prev"] = v   # what Module.__setattr__ does for a registered buffer
    return buf, mask


def unpack_state(model, state: torch.Tensor):
    fs = _ferro_modules(model)
    B = state.numel() // sum(f.in_dim for f in fs)
    for f, v in zip(fs, _state_views(state, model, B)):
        bufs = f.__dict__["_buffers"]
        if bufs["_prev"] is not v:
            bufs["_prev"] = v
        b = bufs.get("_bsign")
        if b is not None and b.shape[0] != B:
            bufs["_bsign"] = None


def _fused_eval(model, handle, x):
    B = x.shape[0]
    plan = build_plan(model, handle, x.device)
    state, mask = pack_state(model, B, x.device)
    io = model.__dict__.get("_fetode_io")
    n_out = io[1] if io is not None else field_layers(model)[-1][0].out_features
    out = torch.empty(B, n_out, device=x.device, dtype=torch.float32)
    _lib.check(_lib.load().fetode_field_forward(handle.ref, plan.data_ptr(), x.data_ptr(), B, _lib.ptr(state),
                                                mask, out.data_ptr(), _stream(x)), "field forward")
    if state is not None:
        unpack_state(model, state)
    return out


def field_apply(model, x: torch.Tensor) -> torch.Tensor:
    """KAN.forward / KANFET.forward: one evaluation.  Inference on a shape with a fused kernel
    is one launch; otherwise (other widths, or autograd recording) one HIP kernel per
    KANLinear / Ferro layer, each with its HIP backward."""
    io = model.__dict__.get("_fetode_io")   # (in, out) of the stack (module attribute reads are slow)
    if io is None:
        ls = field_layers(model)
        io = model.__dict__["_fetode_io"] = (ls[0][0].in_features, ls[-1][0].out_features)
    in0 = io[0]
    lead = x.shape[:-1]
    if model.has_ferro and x.dim() != 2:
        raise ValueError("KANFET expects x of shape (B, in_features)")
    x2 = x.reshape(-1, in0)
    _lib.require_gpu_tensor(x2, type(model).__name__ + ".forward")
    B = x2.shape[0]
    # the stack's own tensors (module dict reads): model.parameters() walks the module tree, ~40 us
    # per call — a dopri5 training solve evaluates the field ~200 times
    grad = torch.is_grad_enabled() and (x2.requires_grad or any(t.requires_grad for t in _field_tensors(model)))
    if not grad:
        x2 = x2.contiguous()
        handle = make_handle(model, B, x2.device)
        if handle.supported(_lib.load()):
            out = _fused_eval(model, handle, x2)
            return out.reshape(*lead, out.shape[-1]) if not model.has_ferro else out
    h = x2
    for kan, fer in field_layers(model):
        if not grad:
            # production widths (ETT KANFET[64,128,64], ...): the whole layer KANLinear + Ferro in one launch
            reinit = fer._needs_reinit(h) if fer is not None else False
            if fer is None or fer._branch_sign_for(h) is None:
                y = wide_apply(kan, fer, h.contiguous(), reinit=reinit)
                if y is not None:
                    if fer is not None:
                        fer._commit_state(h, reinit)
                    h = y
                    continue
        if grad and _WIDE_GRAD and kan.out_features in (64, 128):
            # production widths under autograd: the forward in the wide-layer kernel, the VJPs in
            # the wide MFMA / one-pass kernels (_WideLayerFn)
            reinit = fer._needs_reinit(h) if fer is not None else False
            if fer is None or fer._branch_sign_for(h) is None:
                y = wide_layer_grad(kan, fer, h, reinit)
                if y is not None:
                    if fer is not None:
                        fer._commit_state(h, reinit)
                    h = y
                    continue
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


# ---------------------------------------------------------------------------------------------
# wide layers (fetode_wide_layer_*): KANLinear + Ferro of one layer in one launch, Ferro on VALU,
# the KAN contraction on MFMA (production widths: ETT 64/128, ECG FerroElectricNet 64/128)
# ---------------------------------------------------------------------------------------------

def _wide_tensors(kan, fer):
    ts = []
    if kan is not None:
        ts += [kan.grid, *[p for p in kan_params(kan) if p is not None]]
    if fer is not None:
        ts += [getattr(fer, n) for n in FERRO_PARAM_NAMES]
    return ts


def _tkey(ts):
    """Per-tensor (storage address, version counter, contiguity, dtype): a device change moves the
    storage, set_() / restriding at the same address changes dtype or contiguity; the full check
    (fp32, contiguous, on the device) runs when a plan is (re)built."""
    return tuple([(t.data_ptr(), t._version, t.is_contiguous(), t.dtype) for t in ts])


def _wide_key(kan, fer, device, parts=None):
    """The cache key of a wide-layer plan; `parts` = (KAN key, Ferro key) already computed by
    wide_plans (one pass over the layer's tensors for its three plans)."""
    if parts is None:
        parts = (_tkey(_wide_tensors(kan, None)) if kan is not None else (),
                 _tkey(_wide_tensors(None, fer)) if fer is not None else ())
    return (str(device), _lib.param_generation(), parts[0] if kan is not None else (),
            parts[1] if fer is not None else ())


def _plan_tensors_ok(kan, fer, device):
    return all(t.dtype == torch.float32 and t.is_contiguous() and t.device == device
               for t in _wide_tensors(kan, fer))


def wide_plans(kan, fer, device):
    """(KANLinear + Ferro plan, KANLinear plan, Ferro plan) of a layer (wide_plan entries or None;
    the Ferro one None when fer is None): the forward and the two VJPs' plans from one key pass."""
    parts = (_tkey(_wide_tensors(kan, None)), _tkey(_wide_tensors(None, fer)) if fer is not None else ())
    kf = wide_plan(kan, fer, device, parts)
    if fer is None:
        return kf, kf, None
    return kf, wide_plan(kan, None, device, parts), wide_plan(None, fer, device, parts)


def wide_plan(kan, fer, device, parts=None):
    """(plan, kan descriptor, ferro descriptor) of a wide layer, or None when the layer has no
    wide kernel.  Packed once per parameter version (the tensors' version counters, like the
    fused plan), cached on the KANLinear (or the Ferro module when alone)."""
    owner = kan if kan is not None else fer
    attr = "_fetode_wide_kf" if (kan is not None and fer is not None) else "_fetode_wide"
    key = _wide_key(kan, fer, device, parts)
    cached = owner.__dict__.get(attr)
    if cached is not None and cached[0] == key:
        return cached[1]
    if not _plan_tensors_ok(kan, fer, device):
        key = None   # never matched: rebuilt on every call
    lib = _lib.load()
    keep = []
    kd = kan.desc(keep) if kan is not None else None
    fd = fer.desc(keep, None) if fer is not None else None
    kp = _lib.ctypes.byref(kd) if kd is not None else None
    fp = _lib.ctypes.byref(fd) if fd is not None else None
    if not lib.fetode_wide_layer_supported(kp, fp):
        owner.__dict__[attr] = (key, None)
        return None
    n = lib.fetode_wide_layer_plan_bytes(kp, fp)
    plan = torch.empty(max(1, n // 4), device=device, dtype=torch.float32)
    _lib.check(lib.fetode_wide_layer_plan_build(kp, fp, plan.data_ptr(), _lib.stream_handle(device)),
               "fetode_wide_layer_plan_build")
    entry = (plan, kd, fd, keep)
    owner.__dict__[attr] = (key, entry)
    return entry


_WIDE_GRAD = True   # tests flip it to compare with the per-module autograd path
_FLAT_GRAD = True   # tests flip it to compare with the per-parameter _WideLayerFn


class _WideLayerFn(torch.autograd.Function):
    """One KAN-FET (or KANLinear) layer at production widths under autograd: the forward is the
    wide-layer launch (fetode_wide_layer_forward, as under no_grad), the backward the MFMA KANLinear
    VJP then the one-pass Ferro VJP accumulating into the same d/dx.  params = the KANLinear's
    non-None parameters (KAN_PARAM_NAMES order), then the Ferro module's (FERRO_PARAM_NAMES)."""

    @staticmethod
    def forward(ctx, kan, fer, reinit, ents, nk, x, *params):
        xc = _lib.f32c(x)
        out = wide_apply(kan, fer, xc, reinit=reinit, entry=ents[0])
        prev = None if (fer is None or reinit) else fer._prev.detach().clone()   # overwritten after this call
        ctx.kan, ctx.fer, ctx.reinit, ctx.nk, ctx.ents = kan, fer, reinit, nk, ents
        ctx.save_for_backward(xc, prev)
        return out

    @staticmethod
    def backward(ctx, g):
        xc, prev = ctx.saved_tensors
        kan, fer, nk = ctx.kan, ctx.fer, ctx.nk
        want_x = ctx.needs_input_grad[5]
        pn = ctx.needs_input_grad[6:]
        kp = kan_params(kan)
        it = iter(pn[:nk])
        want_k = [next(it) if p is not None else False for p in kp]
        gx, gk = kan_backward(kan, xc, g, want_x, want_k, entry=ctx.ents[1])
        gf = []
        if fer is not None:
            want_f = list(pn[nk:])
            if want_x or any(want_f):
                gxf, gf = ferro_backward(fer, xc, prev, ctx.reinit, None, g, want_x, want_f,
                                         gx_accum=gx if want_x else None, entry=ctx.ents[2])
                if want_x and gx is None:
                    gx = gxf
            else:
                gf = [None] * len(want_f)
        grads_k = [t for t, p in zip(gk, kp) if p is not None]
        return (None, None, None, None, None, gx, *grads_k, *gf)


_FLAT_ALIGN = 64   # floats: every parameter's slice of the flat gradient starts 256-byte aligned


class _WideLayerFlatFn(torch.autograd.Function):
    """_WideLayerFn with the layer's parameters as ONE differentiable input, `flat` (_flat_params:
    their values concatenated, built once per graph and shared by every call of the layer).  The
    backward writes all parameter gradients into one zero-filled buffer laid out like `flat`, so
    autograd adds one tensor per call where it added 24 (the ETT forecaster's dopri5 backward runs
    416 layer VJPs per iteration); the concatenation's own backward hands each parameter its slice
    once per graph."""

    @staticmethod
    def forward(ctx, kan, fer, reinit, ents, layout, x, flat):
        xc = _lib.f32c(x)
        out = wide_apply(kan, fer, xc, reinit=reinit, entry=ents[0])
        prev = None if (fer is None or reinit) else fer._prev.detach().clone()   # overwritten after this call
        ctx.kan, ctx.fer, ctx.reinit, ctx.layout, ctx.ents = kan, fer, reinit, layout, ents
        ctx.save_for_backward(xc, prev)
        return out

    @staticmethod
    def backward(ctx, g):
        xc, prev = ctx.saved_tensors
        kan, fer, (offs, total) = ctx.kan, ctx.fer, ctx.layout
        want_x = ctx.needs_input_grad[5]
        want_p = ctx.needs_input_grad[6]
        kp = kan_params(kan)
        fp = [getattr(fer, n) for n in FERRO_PARAM_NAMES] if fer is not None else []
        gflat = torch.zeros(total, device=xc.device, dtype=torch.float32) if want_p else None
        views = ([gflat.narrow(0, o, p.numel()).view(p.shape) for o, p in zip(offs, [p for p in kp if p is not None] + fp)]
                 if want_p else None)
        it = iter(views or [])
        kout = [None if p is None else next(it) for p in kp] if want_p else None
        fout = list(it) if want_p else None
        gx, _ = kan_backward(kan, xc, g, want_x, [want_p and p is not None for p in kp], out=kout,
                             entry=ctx.ents[1])
        if fer is not None and (want_x or want_p):
            gxf, _ = ferro_backward(fer, xc, prev, ctx.reinit, None, g, want_x, [want_p] * len(fp),
                                    gx_accum=gx if want_x else None, out=fout, entry=ctx.ents[2])
            if want_x and gx is None:
                gx = gxf
        return (None, None, None, None, None, gx, gflat)


def _flat_params(kan, fer, ps):
    """(flat, layout) for _WideLayerFlatFn: the parameters' values concatenated (each slice padded
    to _FLAT_ALIGN floats), cached on the KANLinear and reused by every call of this graph.  A new
    one is made when a parameter changed (version counter, identity, storage) or once the graph's backward
    has reached it (its tensor hook), so a graph built after a backward never shares the old one.
    (A graph discarded unused leaves it cached; a later graph then routes through the same
    concatenation node, which saves no tensors and hands the same values to the parameters.)"""
    key = tuple([(id(p), p._version, p.data_ptr()) for p in ps])   # data_ptr: `.data` swaps (module.to)
    c = kan.__dict__.get("_fetode_flat")
    if c is not None and c[1] == key and c[3][0]:
        return c[0], c[2]
    parts, offs, o = [], [], 0
    for p in ps:
        n = p.numel()
        offs.append(o)
        parts.append(p.reshape(-1))
        pad = -n % _FLAT_ALIGN
        if pad:
            parts.append(p.new_zeros(pad))
        o += n + pad
    flat = torch.cat(parts)
    live = [True]

    def _reached(_g, live=live):
        live[0] = False

    flat.register_hook(_reached)
    layout = (offs, o)
    kan.__dict__["_fetode_flat"] = (flat, key, layout, live)
    return flat, layout


def wide_layer_grad(kan, fer, x, reinit: bool):
    """KANLinear(x) (+ Ferro(x)) with autograd through _WideLayerFlatFn (every parameter requires
    grad: the usual training case) or _WideLayerFn (some frozen), or None if the layer has no wide
    kernels (the caller then runs the per-module path)."""
    # the forward's plan and the two VJPs' (kept for the backward: the gradient at these parameters)
    ents = wide_plans(kan, fer, x.device)
    if ents[0] is None or ents[1] is None or (fer is not None and ents[2] is None):
        return None
    kp = [p for p in kan_params(kan) if p is not None]
    fp = [getattr(fer, n) for n in FERRO_PARAM_NAMES] if fer is not None else []
    if _FLAT_GRAD and all(p.requires_grad for p in kp + fp):
        flat, layout = _flat_params(kan, fer, kp + fp)
        return _WideLayerFlatFn.apply(kan, fer, reinit, ents, layout, x, flat)
    return _WideLayerFn.apply(kan, fer, reinit, ents, len(kp), x, *kp, *fp)


def wide_apply(kan, fer, x, reinit: bool = False, entry=None):
    """out = KANLinear(x) + Ferro(x) (either may be None) through fetode_wide_layer_forward, or None
    if the layer has no wide kernel.  Reads the Ferro module's prev_x; the caller commits the new
    state (ferro_class.py:409).  The ABI takes a raw row-major pointer: x is made contiguous here
    whatever the caller passed (a column slice or an expanded view would be read as wrong rows)."""
    x = _lib.f32c(x)
    B = x.shape[0]
    dev = x.device
    if fer is not None:
        width = fer.in_dim
        outf = fer.out_dim
    else:
        width, outf = kan.in_features, kan.out_features
    if width < 16 or outf < 16:
        return None
    if entry is None:
        entry = wide_plan(kan, fer, dev)
    if entry is None:
        return None
    plan, kd, fd, _ = entry
    prev = None
    if fer is not None and not reinit:
        prev = fer._prev
        if prev.shape != (B, width) or not prev.is_contiguous():
            prev = prev.contiguous()
    out = torch.empty(B, outf, device=dev, dtype=torch.float32)
    lib = _lib.load()
    _lib.check(lib.fetode_wide_layer_forward(
        _lib.ctypes.byref(kd) if kd is not None else None, _lib.ctypes.byref(fd) if fd is not None else None,
        plan.data_ptr(), x.data_ptr(), B, _lib.ptr(prev), int(reinit), out.data_ptr(), _stream(x)),
        "fetode_wide_layer_forward")
    return out
