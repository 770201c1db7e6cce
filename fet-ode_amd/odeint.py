"""torchdiffeq-compatible ``odeint`` on the MI355X (drop-in for ``from torchdiffeq import odeint``).

Reference call sites: train_kanfet_node_predprey.py:252,260 (default method => dopri5),
predator_prey.py:142,149, train_ecg_kan_fet_nn_ode.py:558-565 (dopri5, rtol/atol).
torchdiffeq itself is not vendored in the reference; the semantics follow its
published algorithm (FixedGridODESolver.integrate, rk_common.rk4_alt_step_func,
RKAdaptiveStepsizeODESolver + Dopri5Solver), including the call order of ``func`` — which
matters because the hysteresis basis is stateful (ferro_class.py:409).

Two execution paths, both HIP:
  * fused: ``func`` is ``fet_ode_amd.autonomous(field)`` (or ``field.as_ode_func()``), or the
    reference's unchanged ``calDeriv`` closure ``return kan_fet_model(X)`` (recognised, see
    ``closure_field``), for a KAN / KANFET shape with a fused kernel and a fixed-grid method ->
    the whole solve is one kernel launch (``fetode_integrate_fixed``).
  * per-stage: any other callable -> ``func`` is called stage by stage exactly like
    torchdiffeq, and the stage combines run as HIP kernels (``fetode_rk_combine``).
"""
from __future__ import annotations

import atexit
import math
import os
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .autograd_ops import (FERRO_PARAM_NAMES, axpby, build_plan, field_layers, grad_enabled_for, kan_params,
                           make_handle, pack_state, pin_plan, unpack_state)

FIXED_METHODS = {"euler": _lib.EULER, "midpoint": _lib.MIDPOINT, "rk4": _lib.RK4,
                 "rk4_classic": _lib.RK4_CLASSIC}
SOLVERS = tuple(FIXED_METHODS) + ("dopri5",)


# ---------------------------------------------------------------------------------------------
# input checks (torchdiffeq misc._check_inputs)
# ---------------------------------------------------------------------------------------------

def _check_inputs(y0, t, method):
    if not isinstance(y0, torch.Tensor):
        raise NotImplementedError("tupled y0 is not on the hot path; pass a single tensor")
    if not torch.is_floating_point(y0):
        raise TypeError("`y0` must be a floating point Tensor but is a {}".format(y0.type()))
    if method is None:
        method = "dopri5"
    if method not in SOLVERS:
        raise ValueError('Invalid method "{}". Must be one of {}'.format(
            method, '{"' + '", "'.join(SOLVERS) + '"}.'))
    t = torch.as_tensor(t)
    assert t.dim() == 1, "t must be one dimensional"
    assert not t.requires_grad, "gradients w.r.t. t are not supported"
    tc = t.detach().cpu()
    if not torch.is_floating_point(tc):
        tc = tc.to(torch.get_default_dtype())
    reversed_ = len(tc) > 1 and bool(tc[0] > tc[1])
    tp = -tc if reversed_ else tc
    assert bool((tp[1:] > tp[:-1]).all()), "t must be strictly increasing or decreasing"
    return method, tc, tp, reversed_


# ---------------------------------------------------------------------------------------------
# fixed-grid schedule (FixedGridODESolver.integrate), computed on the host in t's dtype
# ---------------------------------------------------------------------------------------------

class Schedule:
    __slots__ = ("step_coef", "out_step", "out_mode", "out_slope", "n_steps", "T", "grid", "dev", "h")

    def __init__(self, tp: torch.Tensor, step_size, reversed_: bool):
        if step_size is None:
            grid = tp
        else:
            niters = torch.ceil((tp[-1] - tp[0]) / step_size + 1).item()
            grid = torch.arange(0, niters, dtype=tp.dtype) * step_size + tp[0]
            grid[-1] = tp[-1]
        assert grid[0] == tp[0] and grid[-1] == tp[-1]
        g = grid.numpy()
        n = len(g) - 1
        sign = -1.0 if reversed_ else 1.0
        dt = (g[1:] - g[:-1])                     # time dtype arithmetic
        coef = np.zeros((n, 4), dtype=np.float32)
        coef[:, 0] = (sign * dt).astype(np.float32)
        coef[:, 1] = (sign * (0.5 * dt)).astype(np.float32)
        coef[:, 2] = (sign * (dt / 6.0)).astype(np.float32)
        T = len(tp)
        tt = tp.numpy()
        out_step = np.zeros(T, dtype=np.int32)
        out_mode = np.zeros(T, dtype=np.int32)
        out_slope = np.zeros(T, dtype=np.float32)
        j = 1
        for s in range(n):
            t0, t1 = g[s], g[s + 1]
            while j < T and t1 >= tt[j]:
                out_step[j] = s
                if tt[j] == t0:
                    out_mode[j] = 0
                elif tt[j] == t1:
                    out_mode[j] = 1
                else:
                    out_mode[j] = 2
                    out_slope[j] = np.float32((tt[j] - t0) / (t1 - t0))
                j += 1
        self.step_coef, self.out_step, self.out_mode, self.out_slope = coef, out_step, out_mode, out_slope
        self.n_steps, self.T, self.grid, self.h = n, T, g, None
        self.dev: Dict[torch.device, Tuple[torch.Tensor, ...]] = {}

    @classmethod
    def substeps(cls, tp: torch.Tensor, n_sub: int) -> "Schedule":
        """The grid of ``odeint_rk4(f, z0, t, n_substeps)`` (train_kan_fet_ett.py:51-83): per output
        interval h = (t1 - t0) / n_substeps in t's dtype, substep times ti = ti + h accumulated from
        t0, and every substep advanced with that same h; solution[j] = z after interval j."""
        s = object.__new__(cls)
        tt = tp.numpy()
        T = len(tt)
        grid, hs = [tt[0]], []
        for i in range(T - 1):
            t0, t1 = tt[i], tt[i + 1]
            h = (t1 - t0) / tt.dtype.type(n_sub)
            ti = t0
            for k in range(n_sub):
                hs.append(h)
                ti = ti + h
                grid.append(ti)
        hs = np.asarray(hs, dtype=tt.dtype)
        n = len(hs)
        coef = np.zeros((n, 4), dtype=np.float32)
        coef[:, 0] = hs.astype(np.float32)
        coef[:, 1] = (0.5 * hs).astype(np.float32)
        coef[:, 2] = (hs / 6.0).astype(np.float32)
        out_step = np.zeros(T, dtype=np.int32)
        out_mode = np.zeros(T, dtype=np.int32)
        out_step[1:] = np.arange(1, T, dtype=np.int32) * n_sub - 1
        out_mode[1:] = 1
        s.step_coef, s.out_step, s.out_mode, s.out_slope = coef, out_step, out_mode, np.zeros(T, np.float32)
        s.n_steps, s.T, s.grid, s.h = n, T, np.asarray(grid, dtype=tt.dtype), hs
        s.dev = {}
        return s

    def device_arrays(self, device):
        """One async H2D upload per device, cached."""
        if device not in self.dev:
            n, T = self.n_steps, self.T
            buf = torch.empty(4 * n + 3 * T, dtype=torch.float32, pin_memory=True)
            buf[:4 * n] = torch.from_numpy(self.step_coef.reshape(-1))
            buf[4 * n:4 * n + T] = torch.from_numpy(self.out_step.view(np.float32))
            buf[4 * n + T:4 * n + 2 * T] = torch.from_numpy(self.out_mode.view(np.float32))
            buf[4 * n + 2 * T:] = torch.from_numpy(self.out_slope)
            d = buf.to(device, non_blocking=True)
            self.dev[device] = (d, d[:4 * n], d[4 * n:4 * n + T], d[4 * n + T:4 * n + 2 * T], d[4 * n + 2 * T:])
        return self.dev[device]


_SCHED_CACHE: Dict[tuple, Schedule] = {}


_LAST_SCHED = [None, None, None, None]   # tp object, step_size, reversed_, schedule


def get_schedule(tp, step_size, reversed_) -> Schedule:
    # the cached input check hands back the same tp object while t is unchanged: skip the key
    if _LAST_SCHED[0] is tp and _LAST_SCHED[1] == step_size and _LAST_SCHED[2] == reversed_:
        return _LAST_SCHED[3]
    s = _get_schedule(tp, step_size, reversed_)
    _LAST_SCHED[:] = [tp, step_size, reversed_, s]
    return s


def _get_schedule(tp, step_size, reversed_) -> Schedule:
    key = (tp.dtype, tuple(tp.tolist()), step_size, reversed_)
    s = _SCHED_CACHE.get(key)
    if s is None:
        if len(_SCHED_CACHE) > 64:
            _SCHED_CACHE.clear()
        s = _SCHED_CACHE[key] = Schedule(tp, step_size, reversed_)
    return s


# ---------------------------------------------------------------------------------------------
# fused path
# ---------------------------------------------------------------------------------------------

_STAGES = {_lib.EULER: 1, _lib.MIDPOINT: 2, _lib.RK4: 4, _lib.RK4_CLASSIC: 4}


class _FusedFixedFn(torch.autograd.Function):
    """One-launch fixed-grid solve; under autograd the launch also records the layer inputs of
    every evaluation (the tape) and backward is one reverse-sweep launch
    (fetode_integrate_fixed_backward) instead of autograd through every stage."""

    @staticmethod
    def forward(ctx, field, handle, method, y0, sched, training, *params):
        dev = y0.device
        B, D = y0.shape
        lib = _lib.load()
        plan = build_plan(field, handle, dev)
        state, mask = pack_state(field, B, dev)
        _, coef, ostep, omode, oslope = sched.device_arrays(dev)
        sol = torch.empty(sched.T, B, D, device=dev, dtype=torch.float32)
        tape = None  # the caller's flag: needs_input_grad follows requires_grad even under no_grad
        if training:
            H = field_layers(field)[0][0].out_features
            tape = torch.empty(sched.n_steps * _STAGES[method], B, D + H, device=dev, dtype=torch.float32)
            # the backward needs the plan and the state of THIS solve: later solves overwrite the
            # state in place (a copy), and rebuild the plan into a new buffer once it is pinned
            ctx.plan = pin_plan(field, plan)
            ctx.mask, ctx.handle, ctx.method, ctx.sched, ctx.field = mask, handle, method, sched, field
            ctx.B = B
            # freed by autograd after a non-retained backward (kept for retain_graph=True)
            ctx.save_for_backward(tape, None if state is None else state.clone())
        _lib.check(lib.fetode_integrate_fixed(
            handle.ref, plan.data_ptr(), method, y0.data_ptr(), B, coef.data_ptr(), sched.n_steps,
            ostep.data_ptr(), omode.data_ptr(), oslope.data_ptr(), sched.T, sol.data_ptr(),
            _lib.ptr(state), mask, _lib.ptr(tape), _lib.stream_handle(dev)), "fetode_integrate_fixed")
        if state is not None:
            unpack_state(field, state)
        return sol

    @staticmethod
    def backward(ctx, grad):
        lib = _lib.load()
        field, handle, sched, B = ctx.field, ctx.handle, ctx.sched, ctx.B
        tape, state0 = ctx.saved_tensors
        dev = grad.device
        g = _lib.f32c(grad)
        _, coef, ostep, omode, oslope = sched.device_arrays(dev)
        layers = field_layers(field)
        gy0 = torch.empty(B, g.shape[-1], device=dev, dtype=torch.float32) if ctx.needs_input_grad[3] else None
        want = ctx.needs_input_grad[6:]
        params = list(field.parameters())
        # every wanted gradient is a view of ONE flat buffer, in parameter order; where autograd
        # keeps the views as .grad, dist.allreduce_gradients reduces the buffer in place, else
        # (grads accumulated into existing .grad tensors) it flattens them once (12 KB)
        wp = [p for p, w in zip(params, want) if w]
        flat = torch.empty(sum(p.numel() for p in wp), device=dev, dtype=torch.float32)
        grads, off = {}, 0
        for p in wp:
            grads[id(p)] = flat[off:off + p.numel()].view(p.shape)
            off += p.numel()

        def gbuf(p):
            return None if p is None else grads.get(id(p))

        kg = (_lib.KANLinearGrad * len(layers))()
        fg = (_lib.FerroGrad * len(layers))() if layers[0][1] is not None else None
        for l, (kan, fer) in enumerate(layers):
            kg[l] = _lib.KANLinearGrad(*[_lib.ptr(gbuf(p)) for p in kan_params(kan)])
            if fg is not None:
                fg[l] = _lib.FerroGrad(*[_lib.ptr(gbuf(getattr(fer, n))) for n in FERRO_PARAM_NAMES])
        nbytes = lib.fetode_integrate_fixed_backward_workspace(handle.ref, ctx.method, sched.n_steps, B)
        if nbytes < 0:
            _lib.check(_lib.FETODE_EUNSUPPORTED, "fetode_integrate_fixed_backward_workspace")
        ws = torch.empty(max(1, nbytes // 4), device=dev, dtype=torch.float32)
        _lib.check(lib.fetode_integrate_fixed_backward(
            handle.ref, ctx.plan.data_ptr(), ctx.method, B, coef.data_ptr(), sched.n_steps, ostep.data_ptr(),
            omode.data_ptr(), oslope.data_ptr(), sched.T, g.data_ptr(), tape.data_ptr(),
            _lib.ptr(state0), ctx.mask, _lib.ptr(gy0), kg, fg, ws.data_ptr(), _lib.stream_handle(dev)),
            "fetode_integrate_fixed_backward")
        pgrads = [grads.get(id(p)) if w else None for p, w in zip(params, want)]
        return (None, None, None, gy0, None, None, *pgrads)


def fused_field(func):
    """The KAN/KANFET module behind ``func``: tagged by ``autonomous``, or a plain closure that
    only returns the module's call on the state (the reference's unchanged ``calDeriv``)."""
    field = getattr(func, "_fetode_field", None)
    if field is None and _CLOSURE_FUSION:
        field = closure_field(func)
    return field


# ---------------------------------------------------------------------------------------------
# the reference's calDeriv, recognised
# ---------------------------------------------------------------------------------------------
# train_kanfet_node_predprey.py:159-161 (and predator_prey.py:113-115) integrate
#     def calDeriv(t, X):
#         dXdt = kan_fet_model(X)
#         return dXdt
# which calls the module once per stage and does nothing else, so integrating it IS integrating
# autonomous(kan_fet_model): same evaluations, same order, same hysteresis updates.  The function's
# bytecode is checked for exactly that shape (load the module by name, call it on the second
# argument, return the result — nothing else), the name is resolved at every solve (globals or
# closure cell), and only an exact KAN / KANFET instance without hooks qualifies (a subclass may
# override forward; a hook would not run on the fused path).  Anything else takes the per-stage
# path, which calls the closure stage by stage like torchdiffeq.

_CLOSURE_FUSION = os.environ.get("FETODE_CLOSURE_FUSION", "1") != "0"
_IGNORED_OPS = {"NOP", "RESUME", "PUSH_NULL", "PRECALL", "CACHE", "EXTENDED_ARG", "COPY_FREE_VARS"}
_CLOSURE_SHAPES: Dict[object, Optional[Tuple[str, str]]] = {}


def set_closure_fusion(enabled: bool) -> bool:
    """Recognise ``return model(X)`` closures as the module (default on; env
    FETODE_CLOSURE_FUSION=0 turns it off).  Returns the previous value."""
    global _CLOSURE_FUSION
    prev, _CLOSURE_FUSION = _CLOSURE_FUSION, bool(enabled)
    return prev


class closure_fusion:
    """Context manager: ``with closure_fusion(False): ...`` integrates closures stage by stage."""

    def __init__(self, enabled: bool):
        self.enabled = enabled

    def __enter__(self):
        self.prev = set_closure_fusion(self.enabled)
        return self

    def __exit__(self, *exc):
        set_closure_fusion(self.prev)
        return False


def _closure_shape(code) -> Optional[Tuple[str, str]]:
    """('global' | 'deref', name) if `code` is `return M(a1)` or `v = M(a1); return v` over its
    second positional argument a1 (two positional parameters, no *args / **kwargs / keyword-only)."""
    import dis
    if code.co_argcount != 2 or code.co_kwonlyargcount or code.co_flags & 0x0C:
        return None
    arg = code.co_varnames[1]
    ins = [(i.opname, i.argval) for i in dis.get_instructions(code) if i.opname not in _IGNORED_OPS]
    if len(ins) < 4 or ins[0][0] not in ("LOAD_GLOBAL", "LOAD_DEREF") or ins[1] != ("LOAD_FAST", arg):
        return None
    if ins[2][0] not in ("CALL_FUNCTION", "CALL") or ins[2][1] != 1:
        return None
    tail = ins[3:]
    if tail != [("RETURN_VALUE", None)]:
        if len(tail) != 3 or tail[0][0] != "STORE_FAST" or tail[1] != ("LOAD_FAST", tail[0][1]) \
                or tail[2] != ("RETURN_VALUE", None) or tail[0][1] == arg:
            return None
    return ("global" if ins[0][0] == "LOAD_GLOBAL" else "deref", ins[0][1])


def _plain_field(obj) -> bool:
    from .efficientkan import KAN, KANFET
    if type(obj) not in (KAN, KANFET):
        return False
    from torch.nn.modules import module as M
    hooks = (obj._forward_hooks, obj._forward_pre_hooks, obj._backward_hooks,
             getattr(obj, "_backward_pre_hooks", {}), M._global_forward_hooks, M._global_forward_pre_hooks,
             M._global_backward_hooks, getattr(M, "_global_backward_pre_hooks", {}))
    return not any(hooks)


_WARNED_CODES = set()


def _reachable_fields(func):
    """KAN / KANFET modules the function's code can name (globals it loads, closure cells)."""
    from .efficientkan import KAN, KANFET
    code = func.__code__
    objs = [func.__globals__.get(n) for n in code.co_names]
    for cell in func.__closure__ or ():
        try:
            objs.append(cell.cell_contents)
        except ValueError:
            pass
    return [o for o in objs if isinstance(o, (KAN, KANFET))]


def _warn_unfused(func, why):
    code = func.__code__
    if code in _WARNED_CODES or not _reachable_fields(func):
        return
    _WARNED_CODES.add(code)
    import warnings
    warnings.warn(f"fet_ode_amd.odeint: {func.__qualname__} ({code.co_filename}:{code.co_firstlineno}) uses a "
                  f"KAN/KANFET module but {why}, so it is integrated stage by stage (one field launch + one "
                  "combine per stage, ~25x slower than the fused solve).  Write it as `return model(X)` or pass "
                  "fet_ode_amd.autonomous(model).", RuntimeWarning, stacklevel=4)


def closure_field(func):
    """The module a ``calDeriv``-shaped plain function calls, or None (see above).  A function that
    can reach a KAN / KANFET module but does not have that shape warns once (it runs per stage)."""
    import types
    if not isinstance(func, types.FunctionType):
        return None
    code = func.__code__
    shape = _CLOSURE_SHAPES.get(code, False)
    if shape is False:
        shape = _CLOSURE_SHAPES[code] = _closure_shape(code)
    if shape is None:
        _warn_unfused(func, "does more than `return model(X)`")
        return None
    kind, name = shape
    if kind == "global":
        obj = func.__globals__.get(name)
    else:
        try:
            obj = func.__closure__[code.co_freevars.index(name)].cell_contents
        except (ValueError, IndexError, TypeError):   # not a free variable, or an empty cell
            return None
    if _plain_field(obj):
        return obj
    _warn_unfused(func, "the module has hooks or is a subclass")
    return None


_FUSED_TRAINING = os.environ.get("FETODE_FUSED_TRAINING", "1") != "0"


def set_fused_training(enabled: bool) -> bool:
    """Route training solves of fused shapes through the tape + reverse-sweep kernels (default)
    or through the per-stage path (autograd through every stage).  Returns the previous value."""
    global _FUSED_TRAINING
    prev, _FUSED_TRAINING = _FUSED_TRAINING, bool(enabled)
    return prev


def _fused_infer(field, handle, method, y0, sched):
    """_FusedFixedFn.forward without autograd (no tape): the inference solve's host side is
    ~100 us of Python per call otherwise — as long as the whole B = 512 kernel of an 8-way
    strong-scaled shard."""
    dev = y0.device
    B, D = y0.shape
    plan = build_plan(field, handle, dev)
    state, mask = pack_state(field, B, dev)
    _, coef, ostep, omode, oslope = sched.device_arrays(dev)
    sol = torch.empty(sched.T, B, D, device=dev, dtype=torch.float32)
    _lib.check(_lib.load().fetode_integrate_fixed(
        handle.ref, plan.data_ptr(), method, y0.data_ptr(), B, coef.data_ptr(), sched.n_steps,
        ostep.data_ptr(), omode.data_ptr(), oslope.data_ptr(), sched.T, sol.data_ptr(),
        _lib.ptr(state), mask, None, _lib.stream_handle(dev)), "fetode_integrate_fixed")
    if state is not None:
        unpack_state(field, state)
    return sol


def _try_fused(func, y0, sched, method_code):
    field = fused_field(func)
    if field is None or y0.dim() != 2:
        return None
    B = y0.shape[0]
    handle = make_handle(field, B, y0.device)
    lib = _lib.load()
    if not handle.supported(lib):
        return None
    if not torch.is_grad_enabled():
        return _fused_infer(field, handle, method_code, y0.contiguous(), sched)
    params = [p for p in field.parameters()]
    training = grad_enabled_for(y0, *params)
    if training:
        # training: one forward launch that records a tape + one reverse-sweep launch; shapes
        # without a fused backward take the per-stage path (every stage through HIP VJPs)
        if not (_FUSED_TRAINING and lib.fetode_fused_backward_supported(handle.ref)):
            return None
    return _FusedFixedFn.apply(field, handle, method_code, y0.contiguous(), sched, training, *params)


# ---------------------------------------------------------------------------------------------
# per-stage path (any func)
# ---------------------------------------------------------------------------------------------

_THIRD = float(np.float32(1.0) / np.float32(3.0))


def _combine_coefs(method, stage, dt):
    """d out / d (k1..k4) of each stage combine (d out / d y = 1)."""
    if method == _lib.RK4:
        if stage == 1:
            return [dt * _THIRD]
        if stage == 2:
            return [-dt * _THIRD, dt]
        if stage == 3:
            return [dt, -dt, dt]
        return [dt * 0.125, 3 * dt * 0.125, 3 * dt * 0.125, dt * 0.125]
    if method == _lib.RK4_CLASSIC and stage == 4:
        return [dt, 2 * dt, 2 * dt, dt]
    return [dt]


class _CombineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, method, stage, dt, y, k1, k2, k3, k4):
        out = torch.empty_like(y)
        _lib.check(_lib.load().fetode_rk_combine(method, stage, y.data_ptr(), k1.data_ptr(), _lib.ptr(k2),
                                                 _lib.ptr(k3), _lib.ptr(k4), dt, out.data_ptr(), y.numel(),
                                                 _lib.stream_handle(y.device)), "fetode_rk_combine")
        ctx.method, ctx.stage, ctx.dt = method, stage, dt
        return out

    @staticmethod
    def backward(ctx, grad):
        cs = _combine_coefs(ctx.method, ctx.stage, ctx.dt)
        gks = [axpby(c, grad) if ctx.needs_input_grad[4 + i] else None for i, c in enumerate(cs)]
        gks += [None] * (4 - len(gks))
        return (None, None, None, grad if ctx.needs_input_grad[3] else None, *gks)


def _c(v):
    return None if v is None else v.contiguous()


def _combine(method, stage, dt, y, k1, k2=None, k3=None, k4=None):
    if not torch.is_grad_enabled():   # inference: the kernel without the autograd.Function layer
        y, k1, k2, k3, k4 = _c(y), _c(k1), _c(k2), _c(k3), _c(k4)
        out = torch.empty_like(y)
        _lib.check(_lib.load().fetode_rk_combine(method, stage, y.data_ptr(), k1.data_ptr(), _lib.ptr(k2),
                                                 _lib.ptr(k3), _lib.ptr(k4), float(dt), out.data_ptr(), y.numel(),
                                                 _lib.stream_handle(y.device)), "fetode_rk_combine")
        return out
    return _CombineFn.apply(method, stage, float(dt), _c(y), _c(k1), _c(k2), _c(k3), _c(k4))


def _per_stage_fixed(func, y0, sched: Schedule, method: str, tc_dtype, reversed_):
    sol = torch.empty(sched.T, *y0.shape, dtype=y0.dtype, device=y0.device)
    sol[0] = y0
    y = y0
    g = sched.grid
    sign = -1.0 if reversed_ else 1.0

    # stage times on y0's device, like torchdiffeq's t (fields may torch.cat it with the state):
    # every distinct time of the solve uploaded once, then 0-dim views (a tensor per stage would
    # cost a host tensor + a copy launch each)
    times = {}

    def tt(v):
        r = times.get(v)
        if r is None:
            r = times[v] = torch.tensor(sign * v, dtype=y0.dtype).to(y0.device, non_blocking=True)
        return r

    j = 1
    for s in range(sched.n_steps):
        dt, hh, h6 = (float(v) for v in sched.step_coef[s, :3])
        t0, t1 = g[s], g[s + 1]
        hs = sched.h[s] if sched.h is not None else t1 - t0   # odeint_rk4: stage times ti + h / 2, ti + h
        if method == "rk4":
            k1 = func(tt(t0), y)
            k2 = func(tt(t0 + (t1 - t0) / 3), _combine(_lib.RK4, 1, dt, y, k1))
            k3 = func(tt(t0 + 2 * (t1 - t0) / 3), _combine(_lib.RK4, 2, dt, y, k1, k2))
            k4 = func(tt(t1), _combine(_lib.RK4, 3, dt, y, k1, k2, k3))
            y1 = _combine(_lib.RK4, 4, dt, y, k1, k2, k3, k4)
        elif method == "euler":
            y1 = _combine(_lib.EULER, 4, dt, y, func(tt(t0), y))
        elif method == "midpoint":
            k1 = func(tt(t0), y)
            k2 = func(tt(t0 + 0.5 * (t1 - t0)), _combine(_lib.EULER, 4, hh, y, k1))
            y1 = _combine(_lib.EULER, 4, dt, y, k2)
        else:  # rk4_classic
            k1 = func(tt(t0), y)
            k2 = func(tt(t0 + 0.5 * hs), _combine(_lib.EULER, 4, hh, y, k1))
            k3 = func(tt(t0 + 0.5 * hs), _combine(_lib.EULER, 4, hh, y, k2))
            k4 = func(tt(t0 + hs), _combine(_lib.EULER, 4, dt, y, k3))
            y1 = _combine(_lib.RK4_CLASSIC, 4, h6, y, k1, k2, k3, k4)
        while j < sched.T and sched.out_step[j] == s:
            m = sched.out_mode[j]
            if m == 0:
                sol[j] = y
            elif m == 1:
                sol[j] = y1
            else:
                sol[j] = y + float(sched.out_slope[j]) * (y1 - y)
            j += 1
        y = y1
    return sol


# ---------------------------------------------------------------------------------------------
# public entry
# ---------------------------------------------------------------------------------------------

_LAST_T = [None, None, None, None]   # the last t tensor, its version, method, checked inputs


def _clear_last_t():
    _LAST_T[:] = [None] * 4
    _LAST_SCHED[:] = [None] * 4


atexit.register(_clear_last_t)   # before the runtime's teardown


def _check_inputs_cached(y0, t, method):
    """_check_inputs, reusing the result while the same t tensor comes back unmodified (a
    training / bench loop passes one t object: the checks are several small CPU tensor ops)."""
    if (isinstance(t, torch.Tensor) and _LAST_T[0] is t and _LAST_T[1] == t._version and _LAST_T[2] == method
            and isinstance(y0, torch.Tensor) and torch.is_floating_point(y0)):
        return _LAST_T[3]
    r = _check_inputs(y0, t, method)
    if isinstance(t, torch.Tensor):
        _LAST_T[:] = [t, t._version, method, r]
    return r


def odeint(func, y0, t, *, rtol=1e-7, atol=1e-9, method=None, options=None, event_fn=None):
    """torchdiffeq.odeint(func, y0, t, *, rtol, atol, method, options, event_fn) on the GPU.

    Returns a tensor of shape (len(t), *y0.shape).  ``method`` defaults to 'dopri5' like
    torchdiffeq.  Supported: euler, midpoint, rk4 (3/8 rule), rk4_classic, dopri5.
    """
    if event_fn is not None:
        raise NotImplementedError("event_fn is not on the hot path")
    method, tc, tp, reversed_ = _check_inputs_cached(y0, t, method)
    _lib.require_gpu_tensor(y0, "odeint")
    options = dict(options or {})
    if method == "dopri5":
        from .dopri5 import dopri5_solve
        return dopri5_solve(func, y0, tc, tp, reversed_, rtol, atol, options)
    sched = get_schedule(tp, options.pop("step_size", None), reversed_)
    code = FIXED_METHODS[method]
    out = _try_fused(func, y0, sched, code)
    if out is not None:
        return out
    return _per_stage_fixed(func, y0, sched, method, tc.dtype, reversed_)
