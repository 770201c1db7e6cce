"""Dormand–Prince 5(4) — torchdiffeq's default ``odeint`` method — on the GPU.

Reference call sites: every ``odeint`` without ``method`` (train_kanfet_node_predprey.py:252,260;
predator_prey.py:142,149) and the ECG NODEs (train_ecg_kan_fet_nn_ode.py:558-565, :1034-1041,
rtol/atol 1e-2/1e-3 at :1196-1197).  The control flow restates torchdiffeq's
RKAdaptiveStepsizeODESolver + Dopri5Solver: f0 = func(t0, y0); one more call in
_select_initial_step; 6 calls per attempt (FSAL), rejected attempts included — the call order
matters for the stateful hysteresis basis (SURVEY §7.3 hard part 2).  Error ratio = RMS norm of
err / (atol + rtol*max(|y0|,|y1|)) over the whole batch; accept if <= 1; step factor
min(10, max(0.9*ratio^-1/5, 0.2 on reject / 1 on accept)); quartic dense output.

All vector arithmetic runs in HIP kernels (fetode_lincomb, fetode_scaled_rms,
fetode_interp_fit/eval); the accept/reject decision reads one fp32 scalar per attempt back
to the host, as torchdiffeq does (`if accept_step:` on a 0-dim tensor).
"""
from __future__ import annotations

import atexit
import math
import os

import numpy as np
import torch

from . import _lib
from .autograd_ops import axpby

# torchdiffeq _impl/dopri5.py tableau (float64), rounded to the state dtype like
# RKAdaptiveStepsizeODESolver.__init__ does (tableau.to(dtype=y0.dtype))
_A = [1 / 5, 3 / 10, 4 / 5, 8 / 9, 1., 1.]
_BETA = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
_C_ERR = [35 / 384 - 1951 / 21600, 0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
          -2187 / 6784 - -12231 / 42400, 11 / 84 - 649 / 6300, -1. / 60.]
_C_MID = [6025192743 / 30085553152 / 2, 0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
          187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2]

A32 = np.array(_A, dtype=np.float64).astype(np.float32)
BETA32 = [np.array(b, dtype=np.float64).astype(np.float32) for b in _BETA]
CERR32 = np.array(_C_ERR, dtype=np.float64).astype(np.float32)
CMID32 = np.array(_C_MID, dtype=np.float64).astype(np.float32)
ORDER = 5


def _cfloat(arr):
    a = np.ascontiguousarray(arr, dtype=np.float32)
    return a, a.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_float))


_RMS_WS = {}
atexit.register(_RMS_WS.clear)


def _rms_workspace(dev, stream):
    """The norms' multi-workgroup workspace (zeroed once; the kernel leaves it zero): its partials
    and last-arriver counter are reused by every launch, so one per (device, stream) — two solves
    on different streams of one device must not interleave on the same counter."""
    key = (dev, int(stream or 0))
    ws = _RMS_WS.get(key)
    if ws is None:
        n = _lib.load().fetode_scaled_rms_workspace(0)
        ws = _RMS_WS[key] = torch.zeros(max(1, n // 8), device=dev, dtype=torch.float64)
    return ws


class _Dopri5:
    def __init__(self, func, y0, rtol, atol, options, reversed_):
        unsupported = [k for k in ("step_t", "jump_t", "norm", "perturb") if options.get(k) is not None]
        if unsupported:
            raise NotImplementedError(f"dopri5 options not supported: {unsupported}")
        self.lib = _lib.load()
        # trajectory-sharded solve (dist.odeint_sharded): every error norm is the RMS over the
        # global batch, so all ranks take the same steps as one device would
        self.group = options.get("norm_group")
        self.func_user = func
        self.sign = -1.0 if reversed_ else 1.0
        self.y0 = y0.contiguous()
        self.n = self.y0.numel()
        self.dev = y0.device
        self.stream = _lib.stream_handle(self.dev)
        self.rtol, self.atol = float(rtol), float(atol)
        self.first_step = options.get("first_step")
        self.safety = float(options.get("safety", 0.9))
        self.ifactor = float(options.get("ifactor", 10.0))
        self.dfactor = float(options.get("dfactor", 0.2))
        self.min_step = float(options.get("min_step", 0.0))
        self.max_step = float(options.get("max_step", math.inf))
        self.max_num_steps = int(options.get("max_num_steps", 2 ** 31 - 1))
        self.k = torch.empty(7, self.n, device=self.dev, dtype=torch.float32)
        self.scal = torch.empty(2, device=self.dev, dtype=torch.float32)
        self.rms_ws = _rms_workspace(self.dev, self.stream)
        self.n_global = self.n
        if self.group is not None:
            import torch.distributed as dist
            self.group = None if self.group == "world" else self.group
            self.dist = dist
            self.scal64 = torch.empty(2, device=self.dev, dtype=torch.float64)
            self.cpu_reduce = dist.get_backend(self.group) != "nccl"
            cnt = torch.tensor([float(self.n)], dtype=torch.float64,
                               device="cpu" if self.cpu_reduce else self.dev)
            dist.all_reduce(cnt, group=self.group)
            self.n_global = int(cnt.item())
            self.distributed = True
        else:
            self.distributed = False
        self.nfev = 0
        self.attempts = []   # (t0, dt, error_ratio, accepted) like the oracle's Dopri5Trace

    @property
    def n_attempts(self) -> int:
        return len(self.attempts)

    # func with torchdiffeq's _PerturbFunc (t cast to the state dtype) and _ReverseFunc
    def f(self, t: float, y: torch.Tensor) -> torch.Tensor:
        self.nfev += 1
        tt = torch.tensor(self.sign * t, dtype=torch.float64).to(y.dtype)
        out = self.func_user(tt, y.view_as(self.y0))
        if torch.is_grad_enabled() and out.requires_grad:
            raise RuntimeError("the field's output requires grad but the solve was started without "
                               "autograd (a module without trainable parameters closing over trainable "
                               "tensors?); run it with torch.enable_grad()")
        _lib.require_gpu_tensor(out, "odeint func output")
        out = out.reshape(-1)
        if self.sign < 0:
            out = axpby(-1.0, out)
        return out.contiguous()

    def lincomb(self, y0, coefs, out=None):
        c, cp = _cfloat(coefs)
        out = torch.empty(self.n, device=self.dev, dtype=torch.float32) if out is None else out
        _lib.check(self.lib.fetode_lincomb(_lib.ptr(y0), self.k.data_ptr(), self.n, cp, len(c), out.data_ptr(),
                                           self.n, self.stream), "fetode_lincomb")
        return out

    def rms(self, a, sub, y0, y1, check_finite=False) -> float:
        if self.distributed:
            # local sum of squares -> all-reduce (sum, non-finite count) -> global RMS, rounded
            # like the single-device kernel: sqrtf((float)(sum / n))
            _lib.check(self.lib.fetode_scaled_sumsq(a.data_ptr(), _lib.ptr(sub), y0.data_ptr(), _lib.ptr(y1),
                                                    self.rtol, self.atol, self.n, self.scal64.data_ptr(),
                                                    self.rms_ws.data_ptr(), self.stream), "fetode_scaled_sumsq")
            t = self.scal64.cpu() if self.cpu_reduce else self.scal64
            self.dist.all_reduce(t, group=self.group)
            ssum, bad = t.tolist()
            r = np.sqrt(np.float32(ssum / self.n_global))
        else:
            _lib.check(self.lib.fetode_scaled_rms(a.data_ptr(), _lib.ptr(sub), y0.data_ptr(), _lib.ptr(y1),
                                                  self.rtol, self.atol, self.n, self.scal.data_ptr(),
                                                  self.rms_ws.data_ptr(), self.stream), "fetode_scaled_rms")
            r, bad = self.scal.tolist()           # one device->host read per call
        if check_finite and bad:
            raise AssertionError("non-finite values in state `y`")
        return np.float32(r)

    def select_initial_step(self, t0: float, y0, f0) -> float:
        """misc._select_initial_step in fp32 (the state dtype), returned as float64."""
        f32 = np.float32
        d0 = abs(self.rms(y0, None, y0, None))
        d1 = abs(self.rms(f0, None, y0, None))
        if d0 < 1e-5 or d1 < 1e-5:
            h0 = f32(1e-6)
        else:
            h0 = f32(f32(0.01) * d0) / d1
        h0 = abs(f32(h0))
        self.k[0].copy_(f0)
        y1 = self.lincomb(y0, [h0])
        f1 = self.f(t0 + float(h0), y1)
        d2 = abs(f32(self.rms(f1, f0, y0, None)) / h0)
        if d1 <= 1e-15 and d2 <= 1e-15:
            h1 = max(f32(1e-6), f32(h0 * f32(1e-3)))
        else:
            # fp32 power as fp64 pow rounded once (libm powf and the device's differ in the last ulp)
            h1 = f32(np.power(np.float64(f32(0.01) / max(d1, d2)), np.float64(f32(1.0 / float(ORDER - 1 + 1)))))
        return float(min(f32(100 * h0), abs(h1)))

    def integrate(self, tp: torch.Tensor) -> torch.Tensor:
        t = tp.to(torch.float64).tolist()
        T = len(t)
        sol = torch.empty(T, *self.y0.shape, device=self.dev, dtype=torch.float32)
        sol[0] = self.y0
        y = self.y0.reshape(-1).clone()
        f0 = self.f(t[0], y)
        dt = float(self.first_step) if self.first_step is not None else self.select_initial_step(t[0], y, f0)
        t0_state, t1_state = t[0], t[0]
        coeffs = None
        for i in range(1, T):
            next_t = t[i]
            n_steps = 0
            while next_t > t1_state:
                assert n_steps < self.max_num_steps, "max_num_steps exceeded"
                t0 = t1_state
                assert t0 + dt > t0, "underflow in dt {}".format(dt)
                dt32 = np.float32(dt)
                t1 = t0 + dt
                # _runge_kutta_step
                self.k[0].copy_(f0)
                yi = None
                for s in range(6):
                    ti = t1 if A32[s] == 1.0 else float(np.float32(t0) + A32[s] * dt32)
                    yi = self.lincomb(y, BETA32[s] * dt32)
                    self.k[s + 1].copy_(self.f(ti, yi))
                y1 = yi
                err = self.lincomb(None, CERR32 * dt32)
                ratio = self.rms(err, None, y, y1, check_finite=True)
                accept = bool(ratio <= 1)
                self.attempts.append((t0, dt, float(ratio), accept))
                if accept:
                    coeffs = torch.empty(5, self.n, device=self.dev, dtype=torch.float32)
                    _, mp = _cfloat(CMID32 * dt32)
                    _lib.check(self.lib.fetode_interp_fit(y.data_ptr(), y1.data_ptr(), self.k.data_ptr(), self.n,
                                                          mp, dt32, coeffs.data_ptr(), self.n, self.stream),
                               "fetode_interp_fit")
                    y = y1
                    f0 = self.k[6].clone()
                    t0_state, t1_state = t0, t1
                else:
                    t0_state = t0
                dt = self.optimal_step(dt, ratio)
                n_steps += 1
            x = np.float32((next_t - t0_state) / (t1_state - t0_state))
            out = sol[i].view(-1)
            _lib.check(self.lib.fetode_interp_eval(coeffs.data_ptr(), x, out.data_ptr(), self.n, self.stream),
                       "fetode_interp_eval")
        return sol

    def optimal_step(self, dt: float, ratio) -> float:
        """rk_common._optimal_step_size in float64."""
        r = float(ratio)
        if r == 0:
            nxt = dt * self.ifactor
        else:
            dfac = 1.0 if r < 1 else self.dfactor
            if math.isnan(r):
                factor = math.nan
            else:
                factor = min(self.ifactor, max(self.safety / r ** (1.0 / ORDER), dfac))
            nxt = dt * factor
        return min(max(nxt, self.min_step), self.max_step) if not math.isnan(nxt) else nxt


_TABLEAU = np.concatenate([np.concatenate([b, np.zeros(6 - len(b), np.float32)]) for b in BETA32]
                          + [CERR32, CMID32]).astype(np.float32)
_RESIDENT_OPTS = {"first_step", "safety", "ifactor", "dfactor", "min_step", "max_step", "max_num_steps"}


def _raise_status(status: int, timeout_msg: str, restore=None):
    """torchdiffeq's assertions from a resident solver's status word.  Status 4 (a grid barrier
    timed out: the workgroups were not co-resident) runs ``restore`` first, which puts the
    hysteresis memory back to its pre-solve value, so the caller can retry on the host loop."""
    if status == 4 and restore is not None:
        restore()
    if status == 1:
        raise AssertionError("non-finite values in state `y`")
    if status == 2:
        raise AssertionError("underflow in dt")
    if status == 3:
        raise AssertionError("max_num_steps exceeded")
    if status == 4:
        raise RuntimeError(timeout_msg)


_DEFERRED: list = []   # (stats, message) of resident solves whose status a caller checks later
_DEFER = [0]


class deferred_status:
    """Inside this context the resident solvers do not read their status word back at once (one
    device->host read = a full synchronisation per solve); `check_deferred()` — which the context
    calls on exit — raises torchdiffeq's assertion of the first failed solve.  Used by model
    forwards that launch more work after the solve (KanFet_NODE: the classifier), so the host
    does not wait for the solve before issuing it; the exception still comes out of the same
    forward call."""

    def __enter__(self):
        _DEFER[0] += 1
        return self

    def __exit__(self, exc_type, exc, tb):
        _DEFER[0] -= 1
        if _DEFER[0] == 0:
            if exc_type is None:
                check_deferred()
            else:
                _DEFERRED.clear()
        return False


def check_deferred():
    pending = list(_DEFERRED)
    _DEFERRED.clear()
    for stats, msg, restore in pending:
        _raise_status(int(stats[2].item()), msg, restore)


def _status_check(stats, timeout_msg, restore=None):
    """torchdiffeq's assertions from the kernel's status word (one read per solve), or queued
    for `check_deferred` inside `deferred_status`."""
    if _DEFER[0]:
        _DEFERRED.append((stats, timeout_msg, restore))
        return
    _raise_status(int(stats[2].item()), timeout_msg, restore)


def _restorer(pairs):
    """restore() for _raise_status: copies pre-solve snapshots back into the live state tensors
    (and rebinds module attributes) — [(target, snapshot)] or callables."""
    def restore():
        with torch.no_grad():
            for item in pairs:
                if callable(item):
                    item()
                else:
                    item[0].copy_(item[1])
    return restore
_MAX_TRACE = 16384   # attempts logged per resident solve (the count itself is exact beyond it)


class ResidentSolve:
    """nfev / attempts of a device-resident solve, read back from the device lazily."""

    def __init__(self, stats, attempts):
        self._stats, self._att = stats, attempts
        self._host = None

    def _load(self):
        if self._host is None:
            st = self._stats.tolist()
            n = min(st[1], _MAX_TRACE)
            att = [(a[0], a[1], a[2], bool(a[3])) for a in self._att[:n].tolist()]
            self._host = (st[0], att, st[2])
        return self._host

    @property
    def nfev(self):
        return self._load()[0]

    @property
    def attempts(self):
        """(t0, dt, error ratio, accepted) of the first _MAX_TRACE attempts."""
        return self._load()[1]

    @property
    def n_attempts(self):
        return int(self._stats.tolist()[1])


_T_DEV = {}   # (device, time grid) -> the grid as a device fp64 tensor
# dropped at interpreter exit, before module teardown: device memory freed after the runtime's
# (or a profiler's) own exit handlers have run crashes the process
atexit.register(_T_DEV.clear)


def _drop_last_solve():
    dopri5_solve.last = None   # the last solve's device buffers (resident stats / attempt log, k)


atexit.register(_drop_last_solve)


def _try_ecg_resident(func, y0, tp, reversed_, rtol, atol, options):
    """The whole solve in one launch when `func` is the ECG field (No_MLP_KANODEFunc with the
    sigmoid mixer), nothing needs gradients, and the options are the scalar ones."""
    from .ecg import No_MLP_KANODEFunc
    import torch.nn as nn
    if not isinstance(func, No_MLP_KANODEFunc) or reversed_ or y0.dim() != 2:
        return None
    if not isinstance(func.feat.act, nn.Sigmoid) or set(options) - _RESIDENT_OPTS:
        return None
    if not (isinstance(rtol, (int, float)) and isinstance(atol, (int, float))):
        return None
    basis = func.feat.basis
    B, D = y0.shape
    if D != basis.in_dim or D > 64 or B > 3072 or func.proj.out_features != D or basis.use_noise:
        return None
    if torch.is_grad_enabled() and (y0.requires_grad or any(p.requires_grad for p in func.parameters())):
        return None
    lib = _lib.load()
    dev = y0.device
    keep = []
    d = basis.desc(keep)
    w = func.proj.weight
    key = (w.data_ptr(), w._version, _lib.param_generation())
    cached = getattr(func, "_fetode_wT", None)
    if cached is None or cached[0] != key:
        cached = (key, w.detach().t().contiguous().float())
        func._fetode_wT = cached
    wT = cached[1]
    bias = _lib.f32c(func.proj.bias) if func.proj.bias is not None else None
    prev = basis._prev_for(dev)
    prev0 = prev.clone()   # the timeout path restores it (the kernel rewrites prev_x in place)
    yc = _lib.f32c(y0)
    tkey = (dev, tuple(tp.tolist()))   # tp is the host copy odeint made; uploads once per grid
    t_dev = _T_DEV.get(tkey)
    if t_dev is None:
        if len(_T_DEV) > 64:
            _T_DEV.clear()
        t_dev = _T_DEV[tkey] = tp.to(torch.float64).to(dev)
    T = t_dev.numel()
    sol = torch.empty(T, B, D, device=dev, dtype=torch.float32)
    branch = torch.empty(B, basis.in_dim, basis.num_basis, device=dev, dtype=torch.float32)
    ws = torch.empty(max(1, lib.fetode_ecg_dopri5_workspace(B) // 4), device=dev, dtype=torch.float32)
    stats = torch.empty(3, device=dev, dtype=torch.int32)   # the kernel writes all three
    att = torch.empty(_MAX_TRACE, 4, device=dev, dtype=torch.float64)
    fs = options.get("first_step")
    opts = np.array([float(fs) if fs is not None else 0.0, float(options.get("safety", 0.9)),
                     float(options.get("ifactor", 10.0)), float(options.get("dfactor", 0.2)),
                     float(options.get("min_step", 0.0)), float(options.get("max_step", math.inf)),
                     float(options.get("max_num_steps", 2 ** 31 - 1))], dtype=np.float64)
    rc = lib.fetode_ecg_dopri5(
        _lib.ctypes.byref(d), wT.data_ptr(), _lib.ptr(bias), D, prev.data_ptr(), yc.data_ptr(), B, t_dev.data_ptr(),
        T, float(rtol), float(atol), opts.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_double)),
        _TABLEAU.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_float)), sol.data_ptr(), prev.data_ptr(),
        branch.data_ptr(), ws.data_ptr(), stats.data_ptr(), att.data_ptr(), _MAX_TRACE,
        _lib.stream_handle(dev))
    if rc == _lib.FETODE_EUNSUPPORTED:   # no resident grid for this batch / width: host-driven loop
        return None
    _lib.check(rc, "fetode_ecg_dopri5")   # prev_x was rewritten in place (read before, written after)
    old_branch = basis.branch_state
    basis.branch_state = branch
    dopri5_solve.last = ResidentSolve(stats, att)

    def back():
        basis.branch_state = old_branch
    _status_check(stats, "fetode_ecg_dopri5: a grid barrier timed out (workgroups not co-resident); "
                         "the solution is invalid", _restorer([(prev, prev0), back]))
    return sol


def _try_field_resident(func, y0, tp, reversed_, rtol, atol, options):
    """The whole solve in one launch when `func` is a tagged KAN / KAN-FET field with a fused
    kernel (fet_ode_amd.autonomous(model): the LV [2,10,2] fields), nothing needs gradients and
    the options are the scalar ones (fetode_integrate_dopri5)."""
    from .autograd_ops import build_plan, make_handle, pack_state, unpack_state
    from .odeint import fused_field
    field = fused_field(func)
    options = dict(options)
    group = options.pop("norm_group", None)
    if field is None or reversed_ or y0.dim() != 2 or set(options) - _RESIDENT_OPTS:
        return None
    if not (isinstance(rtol, (int, float)) and isinstance(atol, (int, float))):
        return None
    if torch.is_grad_enabled() and (y0.requires_grad or any(p.requires_grad for p in field.parameters())):
        return None
    lib = _lib.load()
    dev = y0.device
    B = y0.shape[0]
    handle = make_handle(field, B, dev)
    xr = None
    if group is not None:
        # trajectory-sharded: every rank must take the resident path, or none (their kernels exchange)
        from . import dist as D
        grp = None if group == "world" else group
        ok = (D._RESIDENT_SHARDED[0] and bool(lib.fetode_fused_supported(handle.ref))
              and 0 < B <= lib.fetode_integrate_dopri5_max_batch(handle.ref, 1))
        agreed = D.resident_agreement(grp, dev, B, ok)
        if agreed is None:
            return None
        B_total, b_off = agreed
        xr = D.XRank.get(grp, dev)
        if not xr.ok:   # agreed over the group: every rank takes the host loop
            return None
    elif B > lib.fetode_integrate_dopri5_max_batch(handle.ref, 0):
        # no resident solver for this shape / batch: decide BEFORE pack_state, which rebinds the
        # layers' prev_x to the fused state buffer (a declined launch would leave them there and
        # skip the first-call re-initialisation of the host loop's first evaluation)
        return None
    plan = build_plan(field, handle, dev)
    state, mask = pack_state(field, B, dev)
    state0 = None if state is None else state.clone()   # for the timeout path
    yc = _lib.f32c(y0)
    tkey = (dev, tuple(tp.tolist()))
    t_dev = _T_DEV.get(tkey)
    if t_dev is None:
        if len(_T_DEV) > 64:
            _T_DEV.clear()
        t_dev = _T_DEV[tkey] = tp.to(torch.float64).to(dev)
    T = t_dev.numel()
    sol = torch.empty(T, B, y0.shape[1], device=dev, dtype=torch.float32)
    ws = torch.empty(max(1, lib.fetode_integrate_dopri5_workspace(B) // 4), device=dev, dtype=torch.float32)
    stats = torch.empty(3, device=dev, dtype=torch.int32)
    att = torch.empty(_MAX_TRACE, 4, device=dev, dtype=torch.float64)
    fs = options.get("first_step")
    opts = np.array([float(fs) if fs is not None else 0.0, float(options.get("safety", 0.9)),
                     float(options.get("ifactor", 10.0)), float(options.get("dfactor", 0.2)),
                     float(options.get("min_step", 0.0)), float(options.get("max_step", math.inf)),
                     float(options.get("max_num_steps", 2 ** 31 - 1))], dtype=np.float64)
    optp = opts.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_double))
    tabp = _TABLEAU.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_float))
    if xr is not None:
        xd = xr.desc(b_off)
        rc = lib.fetode_integrate_dopri5_xrank(
            handle.ref, plan.data_ptr(), yc.data_ptr(), B, B_total, t_dev.data_ptr(), T, float(rtol), float(atol),
            optp, tabp, sol.data_ptr(), _lib.ptr(state), mask, ws.data_ptr(), stats.data_ptr(), att.data_ptr(),
            _MAX_TRACE, _lib.ctypes.byref(xd), _lib.stream_handle(dev))
    else:
        rc = lib.fetode_integrate_dopri5(
            handle.ref, plan.data_ptr(), yc.data_ptr(), B, t_dev.data_ptr(), T, float(rtol), float(atol),
            optp, tabp, sol.data_ptr(), _lib.ptr(state), mask, ws.data_ptr(), stats.data_ptr(), att.data_ptr(),
            _MAX_TRACE, _lib.stream_handle(dev))
    if rc == _lib.FETODE_EUNSUPPORTED:   # the grid does not fit one resident launch: host-driven loop
        return None
    _lib.check(rc, "fetode_integrate_dopri5")
    if state is not None:
        unpack_state(field, state)
    dopri5_solve.last = ResidentSolve(stats, att)
    _status_check(stats, "fetode_integrate_dopri5: a grid reduction timed out (workgroups not co-resident); "
                         "the solution is invalid", None if state is None else _restorer([(state, state0)]))
    return sol


def _opts_array(options):
    fs = options.get("first_step")
    return np.array([float(fs) if fs is not None else 0.0, float(options.get("safety", 0.9)),
                     float(options.get("ifactor", 10.0)), float(options.get("dfactor", 0.2)),
                     float(options.get("min_step", 0.0)), float(options.get("max_step", math.inf)),
                     float(options.get("max_num_steps", 2 ** 31 - 1))], dtype=np.float64)


def _t_device(tp, dev):
    tkey = (dev, tuple(tp.tolist()))
    t_dev = _T_DEV.get(tkey)
    if t_dev is None:
        if len(_T_DEV) > 64:
            _T_DEV.clear()
        t_dev = _T_DEV[tkey] = tp.to(torch.float64).to(dev)
    return t_dev


_TAPE_BYTES0 = 1 << 30    # first-call tape budget; later calls size the tape from the last solve
_TAPE_GUESS_MAX = 16 << 30  # a size learnt at another batch is capped here (a longer solve re-runs)


class _FusedDopri5Fn(torch.autograd.Function):
    """Training through the device-resident dopri5 solve of a fused-shape field (the reference's
    own training call, odeint(calDeriv, X0, t_learn) at rtol 1e-7 / atol 1e-9 followed by
    loss.backward(), train_kanfet_node_predprey.py:252-257).  Forward: ONE launch
    (fetode_integrate_dopri5_tape) that also records the layer inputs and the output of every
    evaluation, the attempt log and the initial-step scalars; the tape is sized from the previous
    solve of the field, and a longer solve is re-run from the same hysteresis state with a larger
    one.  Backward: ONE resident launch (fetode_integrate_dopri5_backward) — reverse-mode through
    every evaluation of every attempt, the stage sums, the interpolant, the error norm and the
    step-size control, like autograd through torchdiffeq (which detaches none of them)."""

    @staticmethod
    def forward(ctx, field, handle, y0, t_dev, rtol, atol, opts, *params):
        from .autograd_ops import build_plan, field_layers, pack_state, pin_plan, unpack_state
        lib = _lib.load()
        dev = y0.device
        B, D = y0.shape
        T = t_dev.numel()
        H = field_layers(field)[0][0].out_features
        plan = build_plan(field, handle, dev)
        state, mask = pack_state(field, B, dev)
        state0 = None if state is None else state.clone()
        per_ev = B * (2 * D + H) * 4
        cap, max_att = getattr(field, "_fetode_d5tape", (max(64, min(1 << 20, _TAPE_BYTES0 // per_ev)), 4096))
        cap = max(64, min(cap, _TAPE_GUESS_MAX // per_ev))
        sol = torch.empty(T, B, D, device=dev, dtype=torch.float32)
        ws = torch.empty(max(1, lib.fetode_integrate_dopri5_workspace(B) // 4), device=dev, dtype=torch.float32)
        stats = torch.empty(3, device=dev, dtype=torch.int32)
        init_rec = torch.zeros(5, device=dev, dtype=torch.float64)
        optp = opts.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_double))
        tabp = _TABLEAU.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_float))
        while True:
            tape = torch.empty(cap, B, 2 * D + H, device=dev, dtype=torch.float32)   # x, h, k per evaluation
            att = torch.empty(max_att, 4, device=dev, dtype=torch.float64)
            _lib.check(lib.fetode_integrate_dopri5_tape(
                handle.ref, plan.data_ptr(), y0.data_ptr(), B, t_dev.data_ptr(), T, rtol, atol, optp, tabp,
                sol.data_ptr(), _lib.ptr(state), mask, ws.data_ptr(), stats.data_ptr(), att.data_ptr(), max_att,
                tape.data_ptr(), cap, init_rec.data_ptr(), _lib.stream_handle(dev)),
                "fetode_integrate_dopri5_tape")
            nfev, n_att, status = stats.tolist()
            if status == 4 and state is not None:
                # a grid timeout leaves the pre-solve memory (the caller may rerun on the host loop);
                # torchdiffeq's own assertions (1-3) keep the last evaluation's, as the reference's
                # prev_x does when they fire — the same rule as _raise_status on the inference paths
                state.copy_(state0)
            if status != 0 and state is not None:
                unpack_state(field, state)
            _raise_status(status, "fetode_integrate_dopri5_tape: a grid reduction timed out (workgroups not "
                                  "co-resident); the solution is invalid")
            if nfev <= cap and n_att <= max_att:
                break
            if state is not None:   # the tape ran out: the same solve again with room for all of it
                state.copy_(state0)
            cap, max_att = nfev + 64, n_att + 16
        field._fetode_d5tape = (nfev + max(64, nfev // 8), n_att + max(16, n_att // 8))
        if state is not None:
            unpack_state(field, state)
        dopri5_solve.last = ResidentSolve(stats, att)
        ctx.field, ctx.handle, ctx.B, ctx.mask = field, handle, B, mask
        ctx.plan = pin_plan(field, plan)
        ctx.t_dev, ctx.rtol, ctx.atol, ctx.opts = t_dev, rtol, atol, opts
        # through save_for_backward (not ctx attributes): autograd frees the tape — GBs at large B
        # and tight rtol — after a non-retained backward, before the next iteration's forward
        # allocates its own, and keeps it for retain_graph=True
        ctx.save_for_backward(tape, att, init_rec, state0)
        ctx.n_ev, ctx.n_att = nfev, n_att
        return sol

    @staticmethod
    def backward(ctx, grad):
        from .autograd_ops import FERRO_PARAM_NAMES, field_layers, kan_params
        lib = _lib.load()
        field, B = ctx.field, ctx.B
        tape, att, init_rec, state0 = ctx.saved_tensors
        dev = grad.device
        g = _lib.f32c(grad)
        layers = field_layers(field)
        gy0 = torch.empty(B, g.shape[-1], device=dev, dtype=torch.float32) if ctx.needs_input_grad[2] else None
        want = ctx.needs_input_grad[7:]
        params = list(field.parameters())
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
        nbytes = lib.fetode_integrate_dopri5_backward_workspace_ev(ctx.handle.ref, B, ctx.n_ev)
        if nbytes < 0:
            _lib.check(_lib.FETODE_EUNSUPPORTED, "fetode_integrate_dopri5_backward_workspace_ev")
        ws = torch.empty(max(1, nbytes // 4), device=dev, dtype=torch.float32)
        status = torch.empty(1, device=dev, dtype=torch.int32)
        _lib.check(lib.fetode_integrate_dopri5_backward(
            ctx.handle.ref, ctx.plan.data_ptr(), B, ctx.t_dev.data_ptr(), ctx.t_dev.numel(), ctx.rtol, ctx.atol,
            ctx.opts.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_double)),
            _TABLEAU.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_float)), g.data_ptr(), tape.data_ptr(),
            ctx.n_ev, att.data_ptr(), ctx.n_att, init_rec.data_ptr(),
            _lib.ptr(state0), ctx.mask, _lib.ptr(gy0), kg, fg, ws.data_ptr(), status.data_ptr(),
            _lib.stream_handle(dev)), "fetode_integrate_dopri5_backward")
        _raise_status(int(status.item()), "fetode_integrate_dopri5_backward: a grid sum timed out (workgroups "
                                          "not co-resident); the gradients are invalid")
        pgrads = [grads.get(id(p)) if w else None for p, w in zip(params, want)]
        return (None, None, gy0, None, None, None, None, *pgrads)


_RESIDENT_TRAIN = os.environ.get("FETODE_DOPRI5_TAPE", "1") != "0"


def set_resident_dopri5_training(enabled: bool) -> bool:
    """Route dopri5 training solves of the fused fields through the taped resident solve + reverse
    sweep (default) or through _Dopri5Grad (host-driven autograd).  Returns the previous value."""
    global _RESIDENT_TRAIN
    prev, _RESIDENT_TRAIN = _RESIDENT_TRAIN, bool(enabled)
    return prev


def _try_field_resident_train(func, y0, tp, reversed_, rtol, atol, options):
    """The taped resident solve + reverse sweep when `func` is a fused-shape field (the LV [2,10,2]
    KAN / KAN-FET, or another depth-2 width on fieldn's driver and sweep), something needs
    gradients, the solve is single-device and forward in time, and the options are the scalar ones."""
    from .autograd_ops import make_handle
    from .odeint import fused_field
    field = fused_field(func)
    if field is None or reversed_ or y0.dim() != 2 or set(options) - _RESIDENT_OPTS:
        return None
    if not (isinstance(rtol, (int, float)) and isinstance(atol, (int, float))):
        return None
    lib = _lib.load()
    dev = y0.device
    B = y0.shape[0]
    handle = make_handle(field, B, dev)
    if not (lib.fetode_fused_supported(handle.ref) and lib.fetode_fused_backward_supported(handle.ref)):
        return None
    if B > min(lib.fetode_integrate_dopri5_max_batch(handle.ref, 0),
               lib.fetode_integrate_dopri5_backward_max_batch(handle.ref)):
        return None
    params = list(field.parameters())
    return _FusedDopri5Fn.apply(field, handle, y0.to(torch.float32).contiguous(), _t_device(tp, dev), float(rtol), float(atol),
                                _opts_array(options), *params)


def _try_wide_resident(func, y0, tp, reversed_, rtol, atol, options):
    """The whole solve in one launch (fetode_wide_dopri5) when `func` is a tagged two-layer wide
    KAN-FET field — the ETT forecaster's KANFETDynamics, KANFET([latent, hidden, latent]),
    train_kan_fet_ett.py:192 — nothing needs gradients and the options are the scalar ones.
    Trajectory-sharded (options["norm_group"], dist.odeint_sharded): one launch per rank whose
    norms are exchanged between the ranks' kernels (fetode_wide_dopri5_xrank) — every rank takes the
    resident path or none."""
    from .autograd_ops import field_layers, wide_plan
    from .odeint import fused_field
    field = fused_field(func)
    options = dict(options)
    group = options.pop("norm_group", None)
    if field is None or reversed_ or y0.dim() != 2 or set(options) - _RESIDENT_OPTS:
        return None
    if not getattr(field, "has_ferro", False):
        return None
    if not (isinstance(rtol, (int, float)) and isinstance(atol, (int, float))):
        return None
    layers = field_layers(field)
    if len(layers) != 2 or any(f is None or f._bsign is not None or f.use_noise for _, f in layers):
        return None
    (k0, f0), (k1, f1) = layers
    B, D = y0.shape
    H = k0.out_features
    dev = y0.device
    ok = True
    if group is None and _WIDE_RESIDENT_GAP[0] < B < _WIDE_RESIDENT_GAP[1]:
        # measured crossover: between these batches the per-layer launches beat the
        # persistent grid's tiles plus its three grid barriers per evaluation
        return None
    if D != k0.in_features or k1.in_features != H or k1.out_features != D or f0.num_basis != f1.num_basis:
        ok = False
    if B <= 0:   # an empty shard votes no: every rank then falls back to the host loop together
        ok = False
    if torch.is_grad_enabled() and (y0.requires_grad or any(p.requires_grad for p in field.parameters())):
        ok = False
    e0 = e1 = None
    if ok:
        e0, e1 = wide_plan(k0, f0, dev), wide_plan(k1, f1, dev)
        ok = e0 is not None and e1 is not None
    lib = _lib.load()
    xr = None
    if group is not None:
        # trajectory-sharded: all ranks take the resident path or none (their kernels exchange norms)
        from . import dist as Dd
        grp = None if group == "world" else group
        agreed = Dd.resident_agreement(grp, dev, B, ok and Dd._RESIDENT_SHARDED[0])
        if agreed is None:
            return None
        B_total, b_off = agreed
        xr = Dd.XRank.get(grp, dev)
        if not xr.ok:   # agreed over the group: every rank takes the host loop
            return None
        ws_bytes = lib.fetode_wide_dopri5_xrank_workspace(B, B_total, b_off, D, H)
    elif not ok:
        return None
    else:
        ws_bytes = lib.fetode_wide_dopri5_workspace(B, D, H)
    if ws_bytes < 0:
        if xr is not None:
            raise RuntimeError("sharded wide dopri5: no workspace for this shard after every rank agreed")
        return None
    yc = _lib.f32c(y0)

    def mem(f, width):
        # the first-call rule of FerroelectricBasis._needs_reinit (ferro_class.py:373-378): batch,
        # device, dtype; a matching but non-contiguous memory is the same state, made contiguous
        p = f._prev
        fresh = p.shape != (B, width) or p.device != dev or p.dtype != torch.float32
        if not fresh and not p.is_contiguous():
            p = f._prev = p.contiguous()
        return fresh, p

    re0, p0 = mem(f0, D)
    re1, p1 = mem(f1, H)
    snap = [(p, p.clone()) for re, p in ((re0, p0), (re1, p1)) if not re]   # for the timeout path
    st0 = torch.empty(B, D, device=dev, dtype=torch.float32) if re0 else p0   # prev_x after the solve
    st1 = torch.empty(B, H, device=dev, dtype=torch.float32) if re1 else p1
    tkey = (dev, tuple(tp.tolist()))
    t_dev = _T_DEV.get(tkey)
    if t_dev is None:
        if len(_T_DEV) > 64:
            _T_DEV.clear()
        t_dev = _T_DEV[tkey] = tp.to(torch.float64).to(dev)
    T = t_dev.numel()
    sol = torch.empty(T, B, D, device=dev, dtype=torch.float32)
    ws = torch.empty(max(1, ws_bytes // 4), device=dev, dtype=torch.float32)
    stats = torch.empty(3, device=dev, dtype=torch.int32)
    att = torch.empty(_MAX_TRACE, 4, device=dev, dtype=torch.float64)
    fs = options.get("first_step")
    opts = np.array([float(fs) if fs is not None else 0.0, float(options.get("safety", 0.9)),
                     float(options.get("ifactor", 10.0)), float(options.get("dfactor", 0.2)),
                     float(options.get("min_step", 0.0)), float(options.get("max_step", math.inf)),
                     float(options.get("max_num_steps", 2 ** 31 - 1))], dtype=np.float64)
    by = _lib.ctypes.byref
    optp = opts.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_double))
    tabp = _TABLEAU.ctypes.data_as(_lib.ctypes.POINTER(_lib.ctypes.c_float))
    mask = (1 if re0 else 0) | (2 if re1 else 0)
    if xr is not None:
        xd = xr.desc(b_off)
        rc = lib.fetode_wide_dopri5_xrank(
            by(e0[1]), by(e0[2]), e0[0].data_ptr(), by(e1[1]), by(e1[2]), e1[0].data_ptr(), yc.data_ptr(), B, B_total,
            None if re0 else p0.data_ptr(), None if re1 else p1.data_ptr(), mask, t_dev.data_ptr(), T, float(rtol),
            float(atol), optp, tabp, sol.data_ptr(), st0.data_ptr(), st1.data_ptr(), ws.data_ptr(), stats.data_ptr(),
            att.data_ptr(), _MAX_TRACE, by(xd), _lib.stream_handle(dev))
    else:
        rc = lib.fetode_wide_dopri5(
            by(e0[1]), by(e0[2]), e0[0].data_ptr(), by(e1[1]), by(e1[2]), e1[0].data_ptr(), yc.data_ptr(), B,
            None if re0 else p0.data_ptr(), None if re1 else p1.data_ptr(), mask, t_dev.data_ptr(), T, float(rtol),
            float(atol), optp, tabp, sol.data_ptr(), st0.data_ptr(), st1.data_ptr(), ws.data_ptr(), stats.data_ptr(),
            att.data_ptr(), _MAX_TRACE, _lib.stream_handle(dev))
    if rc == _lib.FETODE_EUNSUPPORTED:
        if xr is not None:   # the peers' kernels are waiting for this rank's norms
            raise RuntimeError("sharded wide dopri5: this rank's launch was refused after every rank agreed: "
                               + _lib.load().fetode_last_error().decode(errors="replace"))
        return None
    _lib.check(rc, "fetode_wide_dopri5")
    old = (f0._prev, f1._prev)   # the memory before the solve (rebound back on a timeout)

    def back():
        f0._prev, f1._prev = old
    if re0:
        f0._prev = st0
    if re1:
        f1._prev = st1
    dopri5_solve.last = ResidentSolve(stats, att)
    _status_check(stats, "fetode_wide_dopri5: a grid barrier timed out (workgroups not co-resident); "
                         "the solution is invalid", _restorer(snap + [back]))
    return sol


_RESIDENT = True
_WIDE_RESIDENT = os.environ.get("FETODE_WIDE_RESIDENT", "1") != "0"
# batches strictly inside (lo, hi) take the host loop: resident / host measured at the ETT widths
# (rtol 1e-3, 96 outputs): B = 256 1.49x, 512 1.14x, 1024 0.84x, 2048 0.88x, 4096 0.94x, 8192 1.02x
_WIDE_RESIDENT_GAP = [512, 8192]


def set_wide_resident_dopri5(enabled: bool, gap=None) -> bool:
    """Device-resident dopri5 for the wide KAN-FET fields (default) or the host-driven loop;
    ``gap = (lo, hi)`` sets the batch range (exclusive) that takes the host loop anyway ((0, 0): none)."""
    global _WIDE_RESIDENT
    prev, _WIDE_RESIDENT = _WIDE_RESIDENT, bool(enabled)
    if gap is not None:
        _WIDE_RESIDENT_GAP[:] = [int(gap[0]), int(gap[1])]
    return prev


def set_resident_dopri5(enabled: bool) -> bool:
    """Device-resident dopri5 for fields that have one (default) or the host-driven loop."""
    global _RESIDENT
    prev, _RESIDENT = _RESIDENT, bool(enabled)
    return prev


class _NormAllReduce(torch.autograd.Function):
    """Sum of a small fp64 vector over the ranks of a trajectory-sharded solve, differentiable:
    forward all-reduces the values, backward all-reduces their adjoints.  The error ratio of every
    attempt (and the initial-step norms) is a function of the WHOLE batch, so d loss / d theta
    through the step-size control has cross-rank terms: rank r's loss depends on dt, dt on every
    rank's sum of squares.  All-reducing the adjoint of the global sum hands every rank the full
    d loss_total / d S, and rank r then backpropagates it into its own trajectories; summing the
    parameter gradients over ranks (dist.allreduce_gradients) gives the single-device gradient.
    Every rank runs the same attempts, so the backward collectives pair up in the same order."""

    @staticmethod
    def forward(ctx, v, group, cpu):
        ctx.group, ctx.cpu = group, cpu
        t = v.detach().cpu().clone() if cpu else v.detach().clone()   # never reduce into v itself
        torch.distributed.all_reduce(t, group=group)
        return t.to(v.device)

    @staticmethod
    def backward(ctx, g):
        t = g.detach().cpu().clone() if ctx.cpu else g.detach().clone()
        torch.distributed.all_reduce(t, group=ctx.group)
        return t.to(g.device), None, None


def _ptrs(ts):
    return (_lib.ctypes.c_void_p * len(ts))(*[t.data_ptr() if t is not None else None for t in ts])


class _CombFn(torch.autograd.Function):
    """y0 + sum_j ks[j] * c[j] (y0 may be None) with c a device vector carrying a gradient (beta dt):
    one fetode_comb_forward launch, and one fetode_comb_backward (+ its dot-product finish) for every
    input's gradient — where the torch expression ran ~2 m kernels forward and ~5 m backward (a
    select, its zero fill and copy, a product and a reduction per term), ≈ 20 % of the ETT dopri5
    training iteration (profiles/r05_ett_train_flat_kernel_stats.csv).  Forward rounding is the torch
    expression's (fetode.h); <g, k_j> is an fp32 sum in a fixed order instead of torch's."""

    @staticmethod
    def forward(ctx, y0, c, *ks):
        lib = _lib.load()
        n = ks[0].numel()
        out = torch.empty_like(ks[0])
        _lib.check(lib.fetode_comb_forward(_lib.ptr(y0), _ptrs(ks), len(ks), c.data_ptr(), out.data_ptr(), n,
                                           _lib.stream_handle(out.device)), "fetode_comb_forward")
        ctx.save_for_backward(c, *ks)
        ctx.y0_shape = None if y0 is None else y0.shape   # y0 may share k's size, not its shape
        return out

    @staticmethod
    def backward(ctx, g):
        c, *ks = ctx.saved_tensors
        lib = _lib.load()
        n = ks[0].numel()
        g = g.contiguous()
        want_y0, want_c, want_k = ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.needs_input_grad[2:]
        gks = [torch.empty_like(k) if w else None for k, w in zip(ks, want_k)]
        gc = ws = None
        if want_c:
            gc = torch.empty_like(c)
            ws = torch.empty(max(1, lib.fetode_comb_workspace(n) // 4), device=g.device, dtype=torch.float32)
        if want_c or any(want_k):
            _lib.check(lib.fetode_comb_backward(g.data_ptr(), _ptrs(ks), len(ks), c.data_ptr(), _ptrs(gks),
                                                _lib.ptr(gc), _lib.ptr(ws), n, _lib.stream_handle(g.device)),
                       "fetode_comb_backward")
        return (g.view(ctx.y0_shape) if want_y0 else None, gc, *gks)


_FUSED_COMB = True   # tests flip it to compare with the torch expression


class _Dopri5Grad:
    """dopri5 with torchdiffeq's direct backpropagation (no adjoint): the solve is recorded by
    autograd through every stage of every attempt, the RMS error ratios and the adaptive step
    sizes (rk_common._optimal_step_size and misc._select_initial_step are tensor expressions in
    torchdiffeq, so d(loss)/d(theta) includes d(dt)/d(theta)).  Same control flow and call order
    as _Dopri5; the field's own HIP VJP serves each evaluation, the O(B*D) stage algebra is torch
    on the device, and t / dt are float64 device tensors like torchdiffeq's."""

    def __init__(self, func, y0, rtol, atol, options, reversed_, check_device=True):
        unsupported = [k for k in ("step_t", "jump_t", "norm", "perturb") if options.get(k) is not None]
        if unsupported:
            raise NotImplementedError(f"dopri5 options not supported with autograd: {unsupported}")
        self.func_user, self.sign, self.y0 = func, (-1.0 if reversed_ else 1.0), y0
        # the field's output must come from the HIP path; the CPU gloo tests of the sharded-norm
        # logic drive this class with a plain torch field in fp64 (check_device=False)
        self.check_device = check_device
        # trajectory-sharded solve (dist.odeint_sharded): norms over the global batch, see
        # _NormAllReduce for the gradient through them
        group = options.get("norm_group")
        self.distributed = group is not None
        if self.distributed:
            import torch.distributed as dist
            self.group = None if group == "world" else group
            self.cpu_reduce = dist.get_backend(self.group) != "nccl"
            cnt = torch.tensor([float(y0.numel())], dtype=torch.float64,
                               device="cpu" if self.cpu_reduce else y0.device)
            dist.all_reduce(cnt, group=self.group)
            self.n_global = float(cnt.item())
        self.dev, self.sdt = y0.device, y0.dtype
        f64 = dict(dtype=torch.float64, device=self.dev)
        self.rtol, self.atol = torch.as_tensor(rtol, **f64), torch.as_tensor(atol, **f64)
        self.first_step = options.get("first_step")
        self.safety = torch.as_tensor(options.get("safety", 0.9), **f64)
        self.ifactor = torch.as_tensor(options.get("ifactor", 10.0), **f64)
        self.dfactor = torch.as_tensor(options.get("dfactor", 0.2), **f64)
        # host copies for _host_next_dt (no device read-back)
        self._h = {k: np.float64(float(options.get(k, v))) for k, v in
                   (("safety", 0.9), ("ifactor", 10.0), ("dfactor", 0.2))}
        self.min_step = float(options.get("min_step", 0.0))
        self.max_step = float(options.get("max_step", math.inf))
        self.max_num_steps = int(options.get("max_num_steps", 2 ** 31 - 1))
        sd = dict(dtype=self.sdt, device=self.dev)
        self.alpha = [float(a) for a in A32]
        self.alpha_t = torch.as_tensor(np.asarray(_A, dtype=np.float64), dtype=torch.float64).to(**sd)
        self.beta = [torch.as_tensor(np.asarray(b, dtype=np.float64)).to(**sd) for b in _BETA]
        self.c_err = torch.as_tensor(np.asarray(_C_ERR, dtype=np.float64)).to(**sd)
        self.c_mid = torch.as_tensor(np.asarray(_C_MID, dtype=np.float64)).to(**sd)
        self.nfev = 0
        self.attempts = []

    def f(self, t, y):
        """_PerturbFunc (t cast to the state dtype) + _ReverseFunc (-f(-t, y))."""
        self.nfev += 1
        out = self.func_user((self.sign * t).to(y.dtype), y)
        if self.check_device:
            _lib.require_gpu_tensor(out, "odeint func output")
        return -out if self.sign < 0 else out

    @property
    def n_attempts(self) -> int:
        return len(self.attempts)

    def rms(self, x, finite_of=None):
        """misc._rms_norm; sharded: RMS over the global batch.  With ``finite_of`` also returns
        whether that tensor is finite on every rank (one collective for both)."""
        if not self.distributed:
            # single device: the loop-top assert already checked this y (no second read-back)
            r = x.abs().pow(2).mean().sqrt()
            return r if finite_of is None else (r, True)
        bad = torch.zeros((), dtype=torch.float64, device=x.device)
        if finite_of is not None:
            bad = (~torch.isfinite(finite_of)).any().to(torch.float64)
        v = _NormAllReduce.apply(torch.stack([x.abs().pow(2).sum().to(torch.float64), bad]), self.group,
                                 self.cpu_reduce)
        r = (v[0] / self.n_global).sqrt().to(x.dtype)
        return r if finite_of is None else (r, bool(v[1] == 0))

    def select_initial_step(self, t0, y0, f0):
        scale = self.atol + torch.abs(y0) * self.rtol
        d0, d1 = self.rms(y0 / scale).abs(), self.rms(f0 / scale).abs()
        if d0 < 1e-5 or d1 < 1e-5:
            h0 = torch.tensor(1e-6, dtype=self.sdt, device=self.dev)
        else:
            h0 = 0.01 * d0 / d1
        h0 = h0.abs()
        f1 = self.f(t0 + h0, y0 + h0 * f0)
        d2 = torch.abs(self.rms((f1 - f0) / scale) / h0)
        if d1 <= 1e-15 and d2 <= 1e-15:
            h1 = torch.max(torch.tensor(1e-6, dtype=self.sdt, device=self.dev), h0 * 1e-3)
        else:
            h1 = (0.01 / max(d1, d2)) ** (1. / float(ORDER))
        return torch.min(100 * h0, h1.abs()).to(torch.float64)

    def _stage(self, y0, ks, c):
        """(y0 +) sum_j ks[j] c[j]: _CombFn for fp32 GPU states, the torch expression otherwise (the
        CPU tests of the sharded norm drive this class in fp64 on the CPU)."""
        k0 = ks[0]
        if (_FUSED_COMB and k0.is_cuda and k0.dtype == torch.float32 and len(ks) <= 8 and c.is_contiguous()
                and all(k.is_contiguous() and k.shape == k0.shape for k in ks)
                and (y0 is None or (y0.is_contiguous() and y0.numel() == k0.numel()))):
            out = _CombFn.apply(y0, c, *ks)
            return out if y0 is None else out.view_as(y0)
        acc = self._comb(ks, c)
        return acc if y0 is None else y0 + acc.view_as(y0)

    @staticmethod
    def _comb(ks, c):
        """sum_j ks[j] * c[j] (torchdiffeq: torch.stack(ks, -1).matmul(c)).  As elementwise device ops,
        not the matmul: a (B*D, s) x (s,) product runs as a rocBLAS gemv with a leading dimension of
        s <= 7, ~4.5 ms per call at the ETT batch (B*D = 524 288) — 55 % of a training iteration
        (profiles/r04_ett_dopri5_train_kernel_stats_gemv.csv).  Autograd differentiates it the same way
        (d/d k_j = c_j g, d/d c_j = <g, k_j>: the gradient through dt is kept)."""
        acc = ks[0] * c[0]
        for j in range(1, len(ks)):
            acc = acc + ks[j] * c[j]
        return acc

    def step(self, y0, f0, t0, dt):
        """One attempt (rk_common._runge_kutta_step): y1, f1, the error estimate and k."""
        t0c, dtc, t1c = t0.to(self.sdt), dt.to(self.sdt), (t0 + dt).to(self.sdt)
        ks = [f0]
        yi = None
        for s in range(6):
            ti = t1c if self.alpha[s] == 1.0 else t0c + self.alpha_t[s] * dtc
            yi = self._stage(y0, ks, self.beta[s] * dtc)
            ks.append(self.f(ti, yi))
        return yi, ks[-1], self._stage(None, ks, dtc * self.c_err), ks

    def optimal_step(self, dt, ratio, ratio_host=None):
        """rk_common._optimal_step_size; ratio_host: the ratio's value already read back (the
        single-device loop reads it once per attempt), for the two branch decisions."""
        rv = ratio if ratio_host is None else ratio_host
        if rv == 0:
            return dt * self.ifactor
        dfactor = self.dfactor if rv >= 1 else torch.ones((), dtype=torch.float64, device=self.dev)
        er = ratio.type_as(dt)
        factor = torch.min(self.ifactor, torch.max(self.safety / er ** (1.0 / ORDER), dfactor))
        return dt * factor

    def _host_next_dt(self, dth, rh):
        """optimal_step + clamp on host floats (numpy fp64, IEEE NaN / inf semantics): the next dt
        up to the ulps of the device pow, NaN exactly when the device dt is NaN."""
        h = self._h
        with np.errstate(all="ignore"):
            d, r = np.float64(dth), np.float64(rh)
            if r == 0:
                nxt = d * h["ifactor"]
            else:
                dfac = h["dfactor"] if r >= 1 else np.float64(1.0)
                f = h["safety"] / r ** np.float64(1.0 / ORDER)
                factor = f if np.isnan(f) else min(h["ifactor"], max(f, dfac))
                nxt = d * factor
            if not np.isnan(nxt):
                nxt = min(max(nxt, np.float64(self.min_step)), np.float64(self.max_step))
        return float(nxt)

    def integrate(self, tp):
        t = tp.to(device=self.dev, dtype=torch.float64)
        y = self.y0
        sol = [y]
        f0 = self.f(t[0], y)
        dt = (torch.as_tensor(float(self.first_step), dtype=torch.float64, device=self.dev)
              if self.first_step is not None else self.select_initial_step(t[0], y, f0))
        t0s = t1s = t[0]
        coeff = [y] * 5
        pending = None
        # single device: the control flow runs on host copies of t, t1 and dt (fp64, the same IEEE
        # sums as the device tensors) and ONE read-back per attempt carries the ratio, the attempt's
        # dt and y1's finiteness (asserted at the next attempt's top if y1 is accepted, where
        # torchdiffeq asserts it); the tensors keep carrying the d/d dt terms.  One sync per attempt
        # instead of nine.  The dt-underflow assert stays BEFORE the attempt's evaluations, as
        # torchdiffeq's: the next dt is predicted on the host from the ratio just read
        # (_host_next_dt, the same formula in fp64); only when the prediction is NaN or within a
        # factor 2 of underflowing is the device dt read first (an extra sync in that rare case), so
        # a failing check never advances a stateful field's hysteresis by six evaluations.  The
        # dense-output coefficients of an accepted step are formed only when an output time needs them (torchdiffeq forms them at every accept; the ones a later accept
        # replaces before any output feed nothing: same solution, same gradient).
        host = not self.distributed
        if host:
            th = [float(v) for v in t.detach().cpu()]
            t1h, dth = th[0], float(dt.detach())
            dt_est = dth
            yfin = bool(torch.isfinite(y).all())
        for i in range(1, len(t)):
            n_steps = 0
            while (th[i] > t1h) if host else bool(t[i] > t1s):
                assert n_steps < self.max_num_steps, "max_num_steps exceeded"
                t0 = t1s
                if host:
                    t0h = t1h
                    if dth is None and not (dt_est == dt_est and t0h + 0.5 * dt_est > t0h):
                        dth = float(dt.detach())   # near underflow / NaN: check the real dt first
                    if dth is not None:
                        assert t0h + dth > t0h, "underflow in dt {}".format(dth)
                    assert yfin, "non-finite values in state `y`"
                else:
                    assert t0 + dt > t0, "underflow in dt {}".format(dt.item())
                y1, f1, err, k = self.step(y, f0, t0, dt)
                tol = self.atol + self.rtol * torch.max(y.abs(), y1.abs())
                if host:
                    ratio = self.rms(err / tol)
                    rv = torch.stack([ratio.detach().to(torch.float64), dt.detach(),
                                      torch.isfinite(y1.detach()).all().to(torch.float64)]).cpu()
                    rh, y1fin = float(rv[0]), bool(rv[2] != 0)
                    if dth is None:
                        dth = float(rv[1])
                        assert t0h + dth > t0h, "underflow in dt {}".format(dth)
                    accept = rh <= 1
                    self.attempts.append((t0h, dth, rh, accept))
                else:
                    # sharded: the finiteness of y on every rank travels with this attempt's norm
                    ratio, finite = self.rms(err / tol, finite_of=y)
                    assert finite, "non-finite values in state `y`"
                    accept = bool(ratio <= 1)
                    self.attempts.append((float(t0.detach()), float(dt.detach()), float(ratio.detach()), accept))
                    rh = None
                if accept:
                    pending = (y, y1, k, dt)
                    y, f0, t0s, t1s = y1, f1, t0, t0 + dt
                    if host:
                        t1h, yfin = t0h + dth, y1fin
                else:
                    t0s = t0
                dt = self.optimal_step(dt, ratio, rh).clamp(self.min_step, self.max_step)
                if host:
                    dt_est = self._host_next_dt(dth, rh)
                    dth = None   # read with the next attempt's ratio
                n_steps += 1
            if pending is not None:   # interp._interp_fit of the last accepted step
                yp, y1p, k, dtp = pending
                dtm = dtp.type_as(yp)
                ym = self._stage(yp, k, dtm * self.c_mid)
                fa, fb = k[0], k[-1]
                coeff = [yp, dtm * fa, dtm * (fb - 4 * fa) - 11 * yp - 5 * y1p + 16 * ym,
                         dtm * (5 * fa - 3 * fb) + 18 * yp + 14 * y1p - 32 * ym,
                         2 * dtm * (fb - fa) - 8 * (y1p + yp) + 16 * ym]
                pending = None
            x = ((t[i] - t0s) / (t1s - t0s)).to(self.sdt)   # interp._interp_evaluate
            total, xp = coeff[0] + x * coeff[1], x
            for c in coeff[2:]:
                xp = xp * x
                total = total + xp * c
            sol.append(total)
        return torch.stack(sol)


def _needs_grad(func, y0) -> bool:
    if not torch.is_grad_enabled():
        return False
    if y0.requires_grad:
        return True
    if isinstance(func, torch.nn.Module):
        return any(p.requires_grad for p in func.parameters())
    return True   # a plain callable may close over trainable tensors


def dopri5_solve(func, y0, tc, tp, reversed_, rtol, atol, options):
    if _RESIDENT:
        sol = _try_ecg_resident(func, y0, tp, reversed_, rtol, atol, options)
        if sol is None:
            sol = _try_field_resident(func, y0, tp, reversed_, rtol, atol, options)
        if sol is None and _WIDE_RESIDENT:
            sol = _try_wide_resident(func, y0, tp, reversed_, rtol, atol, options)
        if sol is not None:
            return sol
    if _needs_grad(func, y0):
        if _RESIDENT and _RESIDENT_TRAIN:
            sol = _try_field_resident_train(func, y0, tp, reversed_, rtol, atol, options)
            if sol is not None:
                return sol
        solver = _Dopri5Grad(func, y0, rtol, atol, options, reversed_)
        sol = solver.integrate(tp)
        dopri5_solve.last = solver
        return sol
    solver = _Dopri5(func, y0, rtol, atol, options, reversed_)
    sol = solver.integrate(tp)
    dopri5_solve.last = solver   # exposes nfev / attempts for tests and tooling
    return sol
