"""Drop-in ``ferro_class.FerroelectricBasis`` (reference: ferro_class.py:329-424).

Same constructor, parameters (k, Ec, Ps, bias, coef), RNG consumption order, forward
semantics and state_dict keys/shapes as the reference.  The difference is the state
layout: the reference stores ``prev_x`` as ``x.expand(B, in, out, K)`` (ferro_class.py:372,409)
and ``branch_sign`` as a tensor that is never written after being reset to ones
(:366, :377-378).  Here the state is the compact ``(B, in)`` prev_x plus an optional
explicit branch_sign; ``.prev_x`` / ``.branch_sign`` return the reference-shaped
(expanded) views and ``state_dict()`` emits/accepts the reference-shaped tensors.

Forward runs the HIP kernel (libfetode ``fetode_ferro_forward``); there is no CPU path.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from ._lib import CacheFreeState
from .autograd_ops import ferro_apply


class FerroelectricBasis(CacheFreeState, nn.Module):
    """P = Ps*tanh(k*(E + Ec*m)) + bias, m from the hysteresis direction/crossing gates."""

    def __init__(self, in_dim, out_dim, num_basis, use_noise=False, gate_slope=10.0, alpha=0.8,
                 noise_std=0.05):
        super().__init__()
        self.in_dim = in_dim
        self.out_dim = out_dim
        self.num_basis = num_basis
        self.use_noise = use_noise
        self.noise_std = noise_std
        self.gate_slope = gate_slope
        self.alpha = alpha
        # same init distributions and RNG order as ferro_class.py:358-362
        self.k = nn.Parameter(torch.rand(in_dim, out_dim, num_basis) * 2 + 0.5)
        self.Ec = nn.Parameter(torch.rand(in_dim, out_dim, num_basis) * 2 + 0.5)
        self.Ps = nn.Parameter(torch.rand(in_dim, out_dim, num_basis) * 1.5 + 0.5)
        self.bias = nn.Parameter(torch.randn(in_dim, out_dim, num_basis) * 0.1)
        self.coef = nn.Parameter(torch.randn(in_dim, out_dim, num_basis))
        # compact state (non-persistent: state_dict carries the reference-shaped tensors instead)
        self.register_buffer("_prev", torch.zeros(1, in_dim), persistent=False)
        self.register_buffer("_bsign", None, persistent=False)   # None == all ones

    # -- reference-shaped views ------------------------------------------------------------
    @property
    def prev_x(self) -> torch.Tensor:
        p = self._prev
        return p[:, :, None, None].expand(p.shape[0], self.in_dim, self.out_dim, self.num_basis)

    @property
    def branch_sign(self) -> torch.Tensor:
        if self._bsign is not None:
            return self._bsign
        return torch.ones(1, 1, 1, 1, dtype=self._prev.dtype, device=self._prev.device).expand(
            self._prev.shape[0], self.in_dim, self.out_dim, self.num_basis)

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        destination[prefix + "prev_x"] = self.prev_x.contiguous() if keep_vars else self.prev_x.detach().contiguous()
        destination[prefix + "branch_sign"] = self.branch_sign.detach().contiguous()

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys,
                              unexpected_keys, error_msgs):
        pk, bk = prefix + "prev_x", prefix + "branch_sign"
        for key in (pk, bk):
            if key not in state_dict and strict:
                missing_keys.append(key)
        if pk in state_dict:
            v = state_dict[pk]
            if v.dim() == 4 and v.shape[1] == self.in_dim:
                if v.numel() and not bool((v == v[:, :, :1, :1]).all()):
                    error_msgs.append(f"{pk}: prev_x is not constant over (out, K); the reference only "
                                      "ever stores x.expand(...) there (ferro_class.py:409)")
                with torch.no_grad():
                    self._prev = v[:, :, 0, 0].detach().clone().to(self._prev.device, self._prev.dtype) \
                        if v.shape[2] and v.shape[3] else torch.zeros(v.shape[0], self.in_dim)
            else:
                error_msgs.append(f"{pk}: expected (B,{self.in_dim},{self.out_dim},{self.num_basis}), got {tuple(v.shape)}")
        if bk in state_dict:
            v = state_dict[bk]
            if bool((v == 1).all()):
                self._bsign = None
            else:
                self._bsign = v.detach().clone().to(self._prev.device, self._prev.dtype)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys,
                                      unexpected_keys, error_msgs)
        for key in (pk, bk):
            while key in unexpected_keys:
                unexpected_keys.remove(key)

    # -- state rules (ferro_class.py:373-378) ---------------------------------------------
    def _needs_reinit(self, x: torch.Tensor) -> bool:
        p = self._prev
        return p.shape[0] != x.shape[0] or p.device != x.device or p.dtype != x.dtype

    def _branch_sign_for(self, x: torch.Tensor):
        """Explicit branch_sign tensor to use, or None for all-ones (the only value the
        reference ever holds unless a state_dict put something else there)."""
        b = self._bsign
        if b is None:
            return None
        if b.shape[0] != x.shape[0] or b.device != x.device or b.dtype != x.dtype:
            self._bsign = None  # :377-378 re-initialises to ones
            return None
        return b

    def _commit_state(self, x: torch.Tensor, reinit: bool):
        """prev_x <- x  (ferro_class.py:409)."""
        xd = x.detach()
        if reinit:
            self._prev = xd.clone()
        else:
            self._prev.copy_(xd)

    def forward(self, x, return_activations=False):
        if x.dim() > 2:
            x = x.view(x.shape[0], -1)
        _lib.require_gpu_tensor(x, "FerroelectricBasis.forward")
        if self.use_noise:
            raise NotImplementedError("use_noise=True is nondeterministic and not on the hot path "
                                      "(SURVEY §2); use the reference NoisyFerroelectricBasis")
        reinit = self._needs_reinit(x)
        bsign = self._branch_sign_for(x)
        out, basis = ferro_apply(self, x, reinit, bsign, return_activations)
        self._commit_state(x, reinit)
        if return_activations:
            return out, basis, self.coef.detach()
        return out

    def reset_state(self):
        """ferro_class.py:422-424: prev_x.zero_() AND branch_sign.fill_(1.0) — so a branch_sign
        loaded from a state_dict is reset to ones here too (None is the all-ones encoding)."""
        self._prev.zero_()
        self._bsign = None

    def desc(self, keep: list, bsign=None) -> _lib.FerroDesc:
        ps = [_lib.f32c(getattr(self, n)) for n in ("k", "Ec", "Ps", "bias", "coef")]
        keep.extend(ps)
        d = _lib.FerroDesc(self.in_dim, self.out_dim, self.num_basis, *[p.data_ptr() for p in ps],
                           float(self.gate_slope), float(self.alpha), None, 0)
        if bsign is not None:
            b = _lib.f32c(bsign)
            keep.append(b)
            d.branch_sign = b.data_ptr()
            d.branch_sign_bstride = self.in_dim * self.out_dim * self.num_basis
        return d
