"""ctypes binding of libfetode.so (the C ABI in include/fetode.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).  There is
no fallback: if the library or a GPU is missing, every compute entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))

# Parameter generation: bumped after every torch optimizer step (any optimizer, global hook).
# The descriptor / plan / packed-weight caches key on (storage, version counter) of every
# parameter, but fused optimizers (torch.optim.Adam(fused=True): torch._fused_adam_) update
# parameters in place WITHOUT bumping version counters, so the generation is part of each key.
_PARAM_GEN = [0]


def _on_optimizer_step(optimizer, args, kwargs) -> None:
    _PARAM_GEN[0] += 1


from torch.optim.optimizer import register_optimizer_step_post_hook  # noqa: E402

register_optimizer_step_post_hook(_on_optimizer_step)


def param_generation() -> int:
    """Number of optimizer steps taken in this process (any optimizer)."""
    return _PARAM_GEN[0]
LIB_PATH = os.environ.get("FETODE_LIB", os.path.join(_HERE, "libfetode.so"))

FETODE_OK, FETODE_EINVAL, FETODE_EUNSUPPORTED, FETODE_EHIP = 0, 1, 2, 3
EULER, MIDPOINT, RK4, RK4_CLASSIC = 0, 1, 2, 3

_vp = ctypes.c_void_p
_fp = ctypes.c_void_p  # device float* passed as raw address


class KANLinearDesc(ctypes.Structure):
    _fields_ = [
        ("in_features", ctypes.c_int32), ("out_features", ctypes.c_int32),
        ("grid_size", ctypes.c_int32), ("spline_order", ctypes.c_int32),
        ("num_logistic", ctypes.c_int32), ("base_act", ctypes.c_int32),
        ("grid", _fp), ("base_weight", _fp), ("spline_weight", _fp), ("spline_scaler", _fp),
        ("logistic_a", _fp), ("logistic_b", _fp), ("logistic_weight", _fp),
        ("logistic_scaler", _fp), ("scale_logistic", ctypes.c_float),
    ]


class FerroDesc(ctypes.Structure):
    _fields_ = [
        ("in_dim", ctypes.c_int32), ("out_dim", ctypes.c_int32), ("num_basis", ctypes.c_int32),
        ("k", _fp), ("Ec", _fp), ("Ps", _fp), ("bias", _fp), ("coef", _fp),
        ("gate_slope", ctypes.c_double), ("alpha", ctypes.c_double),
        ("branch_sign", _fp), ("branch_sign_bstride", ctypes.c_int64),
    ]


class KANLinearGrad(ctypes.Structure):
    _fields_ = [(n, _fp) for n in ("base_weight", "spline_weight", "spline_scaler", "logistic_a",
                                   "logistic_b", "logistic_weight", "logistic_scaler")]


class FerroGrad(ctypes.Structure):
    _fields_ = [(n, _fp) for n in ("k", "Ec", "Ps", "bias", "coef")]


class HLogisticDesc(ctypes.Structure):
    _fields_ = [("in_dim", ctypes.c_int32), ("num_basis", ctypes.c_int32),
                ("k", _fp), ("Ec", _fp), ("Ps", _fp), ("bias", _fp),
                ("gate_slope", ctypes.c_double), ("breaking_point", ctypes.c_double)]


class KANRNNDesc(ctypes.Structure):
    _fields_ = [("num_features", ctypes.c_int32), ("hidden", ctypes.c_int32), ("num_basis", ctypes.c_int32),
                ("latent", ctypes.c_int32), ("ax", _fp), ("bx", _fp), ("ah", _fp), ("bh", _fp), ("w", _fp),
                ("bias", _fp)]


class XRankDesc(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int32), ("world", ctypes.c_int32), ("epoch", ctypes.c_uint32),
                ("inbox", _vp), ("peers", _vp), ("b_offset", ctypes.c_int64)]


class FieldDesc(ctypes.Structure):
    _fields_ = [
        ("n_layers", ctypes.c_int32),
        ("kan", ctypes.POINTER(KANLinearDesc)),
        ("ferro", ctypes.POINTER(FerroDesc)),
    ]


# exported symbol -> (restype, argtypes); mirrors include/fetode.h one to one
SIGNATURES = {
    "fetode_last_error": (ctypes.c_char_p, []),
    "fetode_abi_version": (ctypes.c_int, []),
    "fetode_resident_launch_mode": (ctypes.c_int32, [ctypes.c_int32]),
    "fetode_plan_bytes": (ctypes.c_int64, [ctypes.POINTER(FieldDesc)]),
    "fetode_plan_build": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, _vp]),
    "fetode_state_width": (ctypes.c_int32, [ctypes.POINTER(FieldDesc)]),
    "fetode_fused_supported": (ctypes.c_int, [ctypes.POINTER(FieldDesc)]),
    "fetode_fused_set_small_batch_max": (ctypes.c_int64, [ctypes.c_int64]),
    "fetode_fused_set_tpw1_range": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
    "fetode_fused_set_v8_range": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64]),
    "fetode_fused_get_batch_ranges": (ctypes.c_int, [ctypes.c_void_p]),
    "fetode_dopri5_set_spin_limit": (ctypes.c_uint32, [ctypes.c_uint32]),
    "fetode_integrate_dopri5": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, _vp, ctypes.c_int64, _vp,
                                               ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                               ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float), _vp,
                                               _vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int32, _vp]),
    "fetode_integrate_dopri5_workspace": (ctypes.c_int64, [ctypes.c_int64]),
    "fetode_integrate_dopri5_tape": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, _vp, ctypes.c_int64, _vp,
                                                    ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float),
                                                    _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int32, _vp,
                                                    ctypes.c_int64, _vp, _vp]),
    "fetode_integrate_dopri5_backward": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, ctypes.c_int64, _vp,
                                                        ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float),
                                                        _vp, _vp, ctypes.c_int32, _vp, ctypes.c_int32, _vp, _vp,
                                                        ctypes.c_uint32, _vp, ctypes.POINTER(KANLinearGrad),
                                                        ctypes.POINTER(FerroGrad), _vp, _vp, _vp]),
    "fetode_integrate_dopri5_backward_workspace": (ctypes.c_int64, [ctypes.POINTER(FieldDesc), ctypes.c_int64]),
    "fetode_integrate_dopri5_backward_workspace_ev": (ctypes.c_int64, [ctypes.POINTER(FieldDesc), ctypes.c_int64,
                                                                       ctypes.c_int32]),
    "fetode_integrate_dopri5_backward_max_batch": (ctypes.c_int64, [ctypes.POINTER(FieldDesc)]),
    "fetode_integrate_dopri5_xrank": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, _vp, ctypes.c_int64,
                                                     ctypes.c_int64, _vp, ctypes.c_int32, ctypes.c_double,
                                                     ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                                     ctypes.POINTER(ctypes.c_float), _vp, _vp, ctypes.c_uint32,
                                                     _vp, _vp, _vp, ctypes.c_int32, ctypes.POINTER(XRankDesc), _vp]),
    "fetode_xrank_inbox_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "fetode_integrate_dopri5_max_batch": (ctypes.c_int64, [ctypes.POINTER(FieldDesc), ctypes.c_int32]),
    "fetode_xrank_alloc": (ctypes.c_int, [ctypes.c_int64, ctypes.POINTER(ctypes.c_void_p), _vp]),
    "fetode_xrank_open": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p)]),
    "fetode_xrank_close": (ctypes.c_int, [_vp]),
    "fetode_xrank_free": (ctypes.c_int, [_vp]),
    "fetode_wide_layer_supported": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc)]),
    "fetode_wide_layer_plan_bytes": (ctypes.c_int64, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc)]),
    "fetode_wide_layer_plan_build": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp, _vp]),
    "fetode_wide_layer_forward": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp, _vp,
                                                 ctypes.c_int64, _vp, ctypes.c_int32, _vp, _vp]),
    "fetode_wide_dopri5": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp,
                                          ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp, _vp,
                                          ctypes.c_int64, _vp, _vp, ctypes.c_uint32, _vp, ctypes.c_int32,
                                          ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_float), _vp, _vp, _vp, _vp, _vp, _vp,
                                          ctypes.c_int32, _vp]),
    "fetode_wide_dopri5_workspace": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "fetode_kuramoto_set_lds": (ctypes.c_int, [ctypes.c_int]),
    "fetode_wide_dopri5_xrank": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp,
                                                ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp, _vp,
                                                ctypes.c_int64, ctypes.c_int64, _vp, _vp, ctypes.c_uint32, _vp,
                                                ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                                ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float), _vp,
                                                _vp, _vp, _vp, _vp, _vp, ctypes.c_int32, ctypes.POINTER(XRankDesc),
                                                _vp]),
    "fetode_wide_dopri5_xrank_workspace": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                                            ctypes.c_int32, ctypes.c_int32]),
    "fetode_field_forward": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, _vp, ctypes.c_int64, _vp,
                                            ctypes.c_uint32, _vp, _vp]),
    "fetode_integrate_fixed": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, ctypes.c_int32, _vp,
                                              ctypes.c_int64, _vp, ctypes.c_int32, _vp, _vp, _vp,
                                              ctypes.c_int32, _vp, _vp, ctypes.c_uint32, _vp, _vp]),
    "fetode_kanlinear_forward": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), _vp, ctypes.c_int64, _vp, _vp]),
    "fetode_kanlinear_bsplines": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), _vp, ctypes.c_int64, _vp, _vp]),
    "fetode_ferro_forward": (ctypes.c_int, [ctypes.POINTER(FerroDesc), _vp, ctypes.c_int64, _vp, ctypes.c_int32,
                                            ctypes.c_int32, _vp, _vp, _vp, _vp]),
    "fetode_rk_combine": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, _vp, _vp, _vp, _vp, _vp,
                                         ctypes.c_float, _vp, ctypes.c_int64, _vp]),
    "fetode_axpby": (ctypes.c_int, [ctypes.c_int64, ctypes.c_float, _vp, ctypes.c_float, _vp, _vp, _vp]),
    "fetode_lincomb": (ctypes.c_int, [_vp, _vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_float), ctypes.c_int32,
                                      _vp, ctypes.c_int64, _vp]),
    "fetode_scaled_rms": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double, ctypes.c_int64,
                                         _vp, _vp, _vp]),
    "fetode_scaled_rms_workspace": (ctypes.c_int64, [ctypes.c_int64]),
    "fetode_comb_forward": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, _vp, _vp,
                                           ctypes.c_int64, _vp]),
    "fetode_comb_backward": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32, _vp,
                                            ctypes.POINTER(ctypes.c_void_p), _vp, _vp, ctypes.c_int64, _vp]),
    "fetode_comb_workspace": (ctypes.c_int64, [ctypes.c_int64]),
    "fetode_scaled_sumsq": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_double, ctypes.c_double, ctypes.c_int64,
                                           _vp, _vp, _vp]),
    "fetode_interp_fit": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_float),
                                         ctypes.c_float, _vp, ctypes.c_int64, _vp]),
    "fetode_interp_eval": (ctypes.c_int, [_vp, ctypes.c_float, _vp, ctypes.c_int64, _vp]),
    "fetode_kanlinear_backward_workspace": (ctypes.c_int64, [ctypes.POINTER(KANLinearDesc)]),
    "fetode_kanlinear_backward": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), _vp, ctypes.c_int64, _vp, _vp,
                                                 ctypes.POINTER(KANLinearGrad), _vp, ctypes.c_int32, _vp]),
    "fetode_ferro_backward": (ctypes.c_int, [ctypes.POINTER(FerroDesc), _vp, ctypes.c_int64, _vp, ctypes.c_int32,
                                             _vp, _vp, ctypes.POINTER(FerroGrad), ctypes.c_int32, _vp]),
    "fetode_kanlinear_backward_wide_workspace": (ctypes.c_int64, [ctypes.POINTER(KANLinearDesc),
                                                                  ctypes.POINTER(FerroDesc), ctypes.c_int64]),
    "fetode_kanlinear_backward_wide": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), ctypes.POINTER(FerroDesc), _vp,
                                                      _vp, ctypes.c_int64, _vp, _vp, ctypes.POINTER(KANLinearGrad),
                                                      ctypes.c_int32, _vp, _vp]),
    "fetode_ferro_backward_wide_workspace": (ctypes.c_int64, [ctypes.POINTER(FerroDesc), ctypes.c_int64]),
    "fetode_ferro_backward_wide": (ctypes.c_int, [ctypes.POINTER(FerroDesc), _vp, _vp, ctypes.c_int64, _vp,
                                                  ctypes.c_int32, _vp, _vp, ctypes.POINTER(FerroGrad),
                                                  ctypes.c_int32, _vp, _vp]),
    "fetode_fused_backward_supported": (ctypes.c_int, [ctypes.POINTER(FieldDesc)]),
    "fetode_backward_set_split": (ctypes.c_int, [ctypes.c_int32]),
    "fetode_backward_set_v7": (ctypes.c_int, [ctypes.c_int32]),
    "fetode_integrate_fixed_backward_workspace": (ctypes.c_int64, [ctypes.POINTER(FieldDesc), ctypes.c_int32,
                                                                  ctypes.c_int32, ctypes.c_int64]),
    "fetode_integrate_fixed_backward": (ctypes.c_int, [ctypes.POINTER(FieldDesc), _vp, ctypes.c_int32, ctypes.c_int64,
                                                       _vp, ctypes.c_int32, _vp, _vp, _vp, ctypes.c_int32,
                                                       _vp, _vp, _vp, ctypes.c_uint32, _vp,
                                                       ctypes.POINTER(KANLinearGrad), ctypes.POINTER(FerroGrad),
                                                       _vp, _vp]),
    "fetode_hlogistic_mixer_forward": (ctypes.c_int, [ctypes.POINTER(HLogisticDesc), _vp, ctypes.c_int64, _vp,
                                                      ctypes.c_int32, _vp, _vp, ctypes.c_int32, _vp, _vp, _vp,
                                                      _vp, _vp]),
    "fetode_hlogistic_mixer_backward_workspace": (ctypes.c_int64, [ctypes.POINTER(HLogisticDesc), ctypes.c_int64]),
    "fetode_ecg_dopri5": (ctypes.c_int, [ctypes.POINTER(HLogisticDesc), _vp, _vp, ctypes.c_int32, _vp, _vp,
                                         ctypes.c_int64, _vp, ctypes.c_int32, ctypes.c_double, ctypes.c_double,
                                         ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_float), _vp, _vp,
                                         _vp, _vp, _vp, _vp, ctypes.c_int32, _vp]),
    "fetode_ecg_dopri5_workspace": (ctypes.c_int64, [ctypes.c_int64]),
    "fetode_tanh_bound": (ctypes.c_int, [ctypes.c_int64, ctypes.c_float, _vp, _vp, _vp, _vp]),
    "fetode_tanh_bound_backward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_float, _vp, _vp, _vp, _vp]),
    "fetode_tanh": (ctypes.c_int, [ctypes.c_int64, _vp, _vp, _vp]),
    "fetode_tanh_backward": (ctypes.c_int, [ctypes.c_int64, _vp, _vp, _vp, _vp]),
    "fetode_nan_clamp": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_float] * 5 + [_vp, _vp, _vp]),
    "fetode_nan_clamp_backward": (ctypes.c_int, [ctypes.c_int64] + [ctypes.c_float] * 5 + [_vp, _vp, _vp, _vp]),
    "fetode_kuramoto_forward": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_float, _vp, _vp, _vp, _vp, _vp]),
    "fetode_kuramoto_backward_workspace": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32]),
    "fetode_kanlinear_wide_supported": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc)]),
    "fetode_kanlinear_wide_pack_bytes": (ctypes.c_int64, [ctypes.POINTER(KANLinearDesc)]),
    "fetode_kanlinear_wide_pack": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), _vp, _vp]),
    "fetode_kanlinear_wide_workspace": (ctypes.c_int64, [ctypes.POINTER(KANLinearDesc), ctypes.c_int64]),
    "fetode_kanlinear_wide_forward": (ctypes.c_int, [ctypes.POINTER(KANLinearDesc), _vp, _vp, _vp, ctypes.c_int64, _vp,
                                                     _vp, _vp]),
    "fetode_kuramoto_backward": (ctypes.c_int, [ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                ctypes.c_float, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fetode_hlogistic_mixer_backward": (ctypes.c_int, [ctypes.POINTER(HLogisticDesc), _vp, ctypes.c_int64, _vp,
                                                       ctypes.c_int32, _vp, _vp, ctypes.c_int32, _vp, _vp, _vp, _vp,
                                                       _vp, _vp, _vp, _vp, _vp, _vp]),
    "fetode_kanrnn_forward": (ctypes.c_int, [ctypes.POINTER(KANRNNDesc), _vp, ctypes.c_int64, ctypes.c_int32, _vp,
                                             _vp, _vp, _vp, ctypes.c_int32, _vp]),
    "fetode_kanrnn_depth": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "fetode_kanrnn_backward_workspace": (ctypes.c_int64, [ctypes.POINTER(KANRNNDesc), ctypes.c_int64]),
    "fetode_kanrnn_backward": (ctypes.c_int, [ctypes.POINTER(KANRNNDesc), _vp, ctypes.c_int64, ctypes.c_int32, _vp,
                                              _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fetode_logistic_basis_forward": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _vp, _vp,
                                                     _vp, _vp]),
    "fetode_logistic_basis_backward_workspace": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int64]),
    "fetode_logistic_basis_backward": (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, _vp, _vp,
                                                      _vp, _vp, _vp, _vp, _vp, _vp]),
}

_lib: Optional[ctypes.CDLL] = None
_load_error: Optional[str] = None


class FetodeError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load libfetode.so (once).  Raises if it is absent: there is no CPU fallback."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FetodeError(f"libfetode.so not found at {LIB_PATH}; run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fetode_abi_version() != 2:
        raise FetodeError("libfetode ABI version mismatch")
    _lib = lib
    return lib


def last_error() -> str:
    return load().fetode_last_error().decode(errors="replace")


def check(rc: int, what: str = ""):
    if rc != FETODE_OK:
        msg = load().fetode_last_error().decode(errors="replace")
        if rc == FETODE_EINVAL:
            raise ValueError(f"{what}: {msg}")
        if rc == FETODE_EUNSUPPORTED:
            raise NotImplementedError(f"{what}: {msg}")
        raise FetodeError(f"{what}: {msg} (code {rc})")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_gpu_tensor(x: torch.Tensor, what: str):
    if not x.is_cuda:
        raise RuntimeError(f"{what}: fet_ode_amd computes on the MI355X (HIP) only; got a {x.device} "
                           "tensor. Move the module and inputs to 'cuda'.")
    if x.dtype != torch.float32:
        raise TypeError(f"{what}: expected float32, got {x.dtype}")


def f32c(t: torch.Tensor) -> torch.Tensor:
    """fp32 contiguous view/copy for passing to the ABI."""
    return t.detach().to(torch.float32).contiguous()


class FieldHandle:
    """Keeps the ctypes descriptors (and the tensors they point to) alive for one call."""

    def __init__(self, kan_descs: Sequence[KANLinearDesc], ferro_descs: Optional[Sequence[FerroDesc]],
                 keep: List[torch.Tensor]):
        n = len(kan_descs)
        self._kan = (KANLinearDesc * n)(*kan_descs)
        self._ferro = (FerroDesc * n)(*ferro_descs) if ferro_descs is not None else None
        self.desc = FieldDesc(n, ctypes.cast(self._kan, ctypes.POINTER(KANLinearDesc)),
                              ctypes.cast(self._ferro, ctypes.POINTER(FerroDesc)) if self._ferro is not None
                              else ctypes.POINTER(FerroDesc)())
        self.keep = keep

    @property
    def ref(self):
        return ctypes.byref(self.desc)

    def supported(self, lib) -> bool:
        """fetode_fused_supported for this descriptor (asked once per handle)."""
        s = self.__dict__.get("_supported")
        if s is None:
            s = self._supported = bool(lib.fetode_fused_supported(self.ref))
        return s


_CACHE_PREFIXES = ("_fetode", "_t_eval", "_rhs")


class CacheFreeState:
    """Module mixin: copy.deepcopy / pickle leave out the HIP caches kept in the instance __dict__
    (ctypes descriptors holding raw pointers, packed plans, pinned state views, closures over the
    module).  They describe THIS instance's tensors — a copy must not inherit them — and are
    rebuilt on the copy's first call."""

    def __getstate__(self):
        st = super().__getstate__()
        return {k: v for k, v in st.items() if not k.startswith(_CACHE_PREFIXES)}
