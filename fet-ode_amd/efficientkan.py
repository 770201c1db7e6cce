"""Drop-in ``efficientkan`` (reference: efficient_kan/efficientkan.py) plus ``KANFET``.

``LogisticBasis``, ``KANLinear`` and ``KAN`` keep the reference constructors, parameter
names/shapes, init distributions and RNG consumption order (so ``torch.manual_seed(s)``
gives identical weights), and the same methods.  ``forward`` / ``b_splines`` on CUDA
tensors run the HIP kernels of libfetode.  ``KANFET`` is missing from the reference
snapshot; it is defined here as SURVEY §8a A9 recommends:
layer(x) = KANLinear(x) + FerroelectricBasis(x), stacked like ``KAN``.

Initialisation (``curve2coeff``) and ``update_grid`` are off the hot path (never called
by the reference training loops, predator_prey.py:151-152 is commented out); they use
plain torch ops on whatever device the module lives on.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib
from ._lib import CacheFreeState
from .autograd_ops import field_apply, kanlinear_apply
from .ferro_class import FerroelectricBasis


class LogisticBasis(CacheFreeState, nn.Module):
    """efficientkan.py:7-24: phi = 2/(1+exp(-a(x-b))), (B,in) -> (B,in,nb)."""

    def __init__(self, in_dim: int, num_basis: int):
        super().__init__()
        self.in_dim = in_dim
        self.num_basis = num_basis
        self.a = nn.Parameter(torch.randn(in_dim, num_basis))
        self.b = nn.Parameter(torch.randn(in_dim, num_basis))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.dim() == 2 and x.size(1) == self.in_dim
        x = x.unsqueeze(-1)
        return 2.0 / (1.0 + torch.exp(-self.a * (x - self.b)))


def _b_splines_torch(x, grid, spline_order):
    """Init-time Cox-de Boor (efficientkan.py:117-131) used by curve2coeff/update_grid."""
    x = x.unsqueeze(-1)
    bases = ((x >= grid[:, :-1]) & (x < grid[:, 1:])).to(x.dtype)
    for k in range(1, spline_order + 1):
        bases = ((x - grid[:, : -(k + 1)]) / (grid[:, k:-1] - grid[:, : -(k + 1)]) * bases[:, :, :-1]) + \
                ((grid[:, k + 1:] - x) / (grid[:, k + 1:] - grid[:, 1:(-k)]) * bases[:, :, 1:])
    return bases.contiguous()


class KANLinear(CacheFreeState, nn.Module):
    def __init__(self, in_features, out_features, grid_size=5, spline_order=3, scale_noise=0.1,
                 scale_base=1.0, scale_spline=1.0, enable_standalone_scale_spline=True,
                 base_activation=nn.SiLU, grid_eps=0.02, grid_range=[-1, 1],
                 enable_logistic_basis=True, num_basis=10, scale_logistic=1.0,
                 enable_standalone_scale_logistic=True):
        super().__init__()
        if base_activation is not nn.SiLU:
            raise NotImplementedError("only base_activation=nn.SiLU is on the hot path")
        if not 1 <= spline_order <= 3:
            raise NotImplementedError("spline_order must be 1..3")
        self.in_features = in_features
        self.out_features = out_features
        self.grid_size = grid_size
        self.spline_order = spline_order
        h = (grid_range[1] - grid_range[0]) / grid_size
        grid = ((torch.arange(-spline_order, grid_size + spline_order + 1) * h + grid_range[0])
                .expand(in_features, -1).contiguous())
        self.register_buffer("grid", grid)
        self.base_weight = nn.Parameter(torch.empty(out_features, in_features))
        self.spline_weight = nn.Parameter(torch.empty(out_features, in_features, grid_size + spline_order))
        if enable_standalone_scale_spline:
            self.spline_scaler = nn.Parameter(torch.empty(out_features, in_features))
        self.scale_noise = scale_noise
        self.scale_base = scale_base
        self.scale_spline = scale_spline
        self.enable_standalone_scale_spline = enable_standalone_scale_spline
        self.base_activation = base_activation()
        self.grid_eps = grid_eps
        self.enable_logistic_basis = enable_logistic_basis
        self.num_basis = num_basis
        self.scale_logistic = scale_logistic
        self.enable_standalone_scale_logistic = enable_standalone_scale_logistic
        if enable_logistic_basis:
            self.logistic_basis = LogisticBasis(in_features, num_basis)
            self.logistic_weight = nn.Parameter(torch.empty(out_features, in_features * num_basis))
            if enable_standalone_scale_logistic:
                self.logistic_scaler = nn.Parameter(torch.empty(out_features))
        self.reset_parameters()

    def reset_parameters(self):
        """efficientkan.py:92-115, same order of RNG draws."""
        nn.init.kaiming_uniform_(self.base_weight, a=math.sqrt(5) * self.scale_base)
        with torch.no_grad():
            noise = ((torch.rand(self.grid_size + 1, self.in_features, self.out_features) - 0.5)
                     * self.scale_noise / self.grid_size)
            self.spline_weight.data.copy_(
                (self.scale_spline if not self.enable_standalone_scale_spline else 1.0)
                * self.curve2coeff(self.grid.T[self.spline_order: -self.spline_order], noise))
            if self.enable_standalone_scale_spline:
                nn.init.kaiming_uniform_(self.spline_scaler, a=math.sqrt(5) * self.scale_spline)
        if self.enable_logistic_basis:
            nn.init.kaiming_uniform_(self.logistic_weight, a=math.sqrt(5) * self.scale_logistic)
            if self.enable_standalone_scale_logistic:
                nn.init.ones_(self.logistic_scaler)

    def b_splines(self, x: torch.Tensor):
        """efficientkan.py:117-131; HIP kernel (bitwise equal to the reference) on CUDA."""
        assert x.dim() == 2 and x.size(1) == self.in_features
        _lib.require_gpu_tensor(x, "KANLinear.b_splines")
        keep = []
        d = self.desc(keep)
        xc = _lib.f32c(x)
        out = torch.empty(x.shape[0], self.in_features, self.grid_size + self.spline_order,
                          device=x.device, dtype=torch.float32)
        _lib.check(_lib.load().fetode_kanlinear_bsplines(
            _lib.ctypes.byref(d), xc.data_ptr(), x.shape[0], out.data_ptr(),
            _lib.stream_handle(x.device)), "KANLinear.b_splines")
        return out

    def curve2coeff(self, x: torch.Tensor, y: torch.Tensor):
        """efficientkan.py:133-143 (init-time least squares)."""
        assert x.dim() == 2 and x.size(1) == self.in_features
        assert y.size() == (x.size(0), self.in_features, self.out_features)
        A = _b_splines_torch(x, self.grid, self.spline_order).transpose(0, 1)
        B = y.transpose(0, 1)
        solution = torch.linalg.lstsq(A, B).solution
        result = solution.permute(2, 0, 1)
        assert result.size() == (self.out_features, self.in_features, self.grid_size + self.spline_order)
        return result.contiguous()

    @property
    def scaled_spline_weight(self):
        return self.spline_weight * (self.spline_scaler.unsqueeze(-1) if self.enable_standalone_scale_spline else 1.0)

    @property
    def scaled_logistic_weight(self):
        if not self.enable_logistic_basis:
            return None
        w = self.logistic_weight * self.scale_logistic
        if self.enable_standalone_scale_logistic:
            w = w * self.logistic_scaler.unsqueeze(-1)
        return w

    def desc(self, keep: list) -> _lib.KANLinearDesc:
        """ABI descriptor (pointers stay valid while the tensors in ``keep`` live)."""
        def p(t):
            if t is None:
                return None
            t = _lib.f32c(t)
            keep.append(t)
            return t.data_ptr()
        lg = self.enable_logistic_basis
        return _lib.KANLinearDesc(
            self.in_features, self.out_features, self.grid_size, self.spline_order,
            self.num_basis if lg else 0, 0,
            p(self.grid), p(self.base_weight), p(self.spline_weight),
            p(self.spline_scaler) if self.enable_standalone_scale_spline else None,
            p(self.logistic_basis.a) if lg else None, p(self.logistic_basis.b) if lg else None,
            p(self.logistic_weight) if lg else None,
            p(self.logistic_scaler) if lg and self.enable_standalone_scale_logistic else None,
            float(self.scale_logistic))

    def forward(self, x: torch.Tensor):
        """efficientkan.py:160-182."""
        assert x.size(-1) == self.in_features
        original_shape = x.shape
        x2d = x.reshape(-1, self.in_features)
        _lib.require_gpu_tensor(x2d, "KANLinear.forward")
        out = kanlinear_apply(self, x2d)
        return out.reshape(*original_shape[:-1], self.out_features)

    @torch.no_grad()
    def update_grid(self, x: torch.Tensor, margin=0.01):
        """efficientkan.py:184-221 (off the hot path; torch ops)."""
        assert x.dim() == 2 and x.size(1) == self.in_features
        batch = x.size(0)
        splines = _b_splines_torch(x, self.grid, self.spline_order).permute(1, 0, 2)
        orig_coeff = self.scaled_spline_weight.permute(1, 2, 0)
        unreduced = torch.bmm(splines, orig_coeff).permute(1, 0, 2)
        x_sorted = torch.sort(x, dim=0)[0]
        grid_adaptive = x_sorted[torch.linspace(0, batch - 1, self.grid_size + 1, dtype=torch.int64,
                                                device=x.device)]
        uniform_step = (x_sorted[-1] - x_sorted[0] + 2 * margin) / self.grid_size
        grid_uniform = (torch.arange(self.grid_size + 1, dtype=torch.float32, device=x.device).unsqueeze(1)
                        * uniform_step + x_sorted[0] - margin)
        grid = self.grid_eps * grid_uniform + (1 - self.grid_eps) * grid_adaptive
        grid = torch.concatenate([
            grid[:1] - uniform_step * torch.arange(self.spline_order, 0, -1, device=x.device).unsqueeze(1),
            grid,
            grid[-1:] + uniform_step * torch.arange(1, self.spline_order + 1, device=x.device).unsqueeze(1),
        ], dim=0)
        self.grid.copy_(grid.T)
        self.spline_weight.data.copy_(self.curve2coeff(x, unreduced))

    def regularization_loss(self, regularize_activation=1.0, regularize_entropy=1.0,
                            regularize_logistic_l1=0.0):
        """efficientkan.py:223-237."""
        l1_fake = self.spline_weight.abs().mean(-1)
        reg_act = l1_fake.sum()
        p = l1_fake / (reg_act + 1e-12)
        reg_ent = -torch.sum(p * (p + 1e-12).log())
        reg = regularize_activation * reg_act + regularize_entropy * reg_ent
        if self.enable_logistic_basis and regularize_logistic_l1 != 0.0:
            reg = reg + regularize_logistic_l1 * self.logistic_weight.abs().mean()
        return reg


class _FieldMixin(CacheFreeState):
    """Shared by KAN and KANFET: the whole stack as one fetode field."""

    def as_ode_func(self):
        """A ``func(t, y)`` for ``odeint`` that takes the fused single-launch path."""
        return autonomous(self)


class KAN(_FieldMixin, nn.Module):
    """efficientkan.py:240-284."""
    has_ferro = False

    def __init__(self, layers_hidden, grid_size=5, spline_order=3, scale_noise=0.1, scale_base=1.0,
                 scale_spline=1.0, base_activation=torch.nn.SiLU, grid_eps=0.02, grid_range=[-1, 1]):
        super().__init__()
        self.grid_size = grid_size
        self.spline_order = spline_order
        self.layers = nn.ModuleList()
        for in_features, out_features in zip(layers_hidden, layers_hidden[1:]):
            self.layers.append(KANLinear(in_features, out_features, grid_size=grid_size,
                                         spline_order=spline_order, scale_noise=scale_noise,
                                         scale_base=scale_base, scale_spline=scale_spline,
                                         base_activation=base_activation, grid_eps=grid_eps,
                                         grid_range=grid_range))

    def forward(self, x: torch.Tensor, update_grid=False):
        if update_grid:
            for layer in self.layers:
                layer.update_grid(x)
                x = layer(x)
            return x
        return field_apply(self, x)

    def regularization_loss(self, regularize_activation=1.0, regularize_entropy=1.0):
        return sum(layer.regularization_loss(regularize_activation, regularize_entropy)
                   for layer in self.layers)


class KANFETLayer(CacheFreeState, nn.Module):
    """One KAN-FET layer: KANLinear(x) + FerroelectricBasis(x)."""

    def __init__(self, in_features, out_features, grid_size=5, spline_order=3, num_fet_basis=10,
                 gate_slope=10.0, alpha=0.8, **kan_kw):
        super().__init__()
        self.kan = KANLinear(in_features, out_features, grid_size=grid_size, spline_order=spline_order,
                             **kan_kw)
        self.ferro = FerroelectricBasis(in_features, out_features, num_fet_basis, gate_slope=gate_slope,
                                        alpha=alpha)

    def forward(self, x):
        return self.kan(x) + self.ferro(x)


class KANFET(_FieldMixin, nn.Module):
    """KAN with a ferroelectric hysteresis branch per layer (build-defined).

    Constructor mirrors ``KAN.__init__`` (efficientkan.py:241-272) with the extra
    ``num_fet_basis=10``, ``gate_slope=10.0``, ``alpha=0.8`` of ``FerroelectricBasis``
    (ferro_class.py:347).  state_dict keys: ``layers.{l}.kan.*`` and ``layers.{l}.ferro.*``.
    """
    has_ferro = True

    def __init__(self, layers_hidden, grid_size=5, spline_order=3, scale_noise=0.1, scale_base=1.0,
                 scale_spline=1.0, base_activation=torch.nn.SiLU, grid_eps=0.02, grid_range=[-1, 1],
                 num_fet_basis=10, gate_slope=10.0, alpha=0.8):
        super().__init__()
        self.grid_size = grid_size
        self.spline_order = spline_order
        self.layers = nn.ModuleList(
            KANFETLayer(i, o, grid_size=grid_size, spline_order=spline_order, num_fet_basis=num_fet_basis,
                        gate_slope=gate_slope, alpha=alpha, scale_noise=scale_noise, scale_base=scale_base,
                        scale_spline=scale_spline, base_activation=base_activation, grid_eps=grid_eps,
                        grid_range=grid_range)
            for i, o in zip(layers_hidden, layers_hidden[1:]))

    def forward(self, x: torch.Tensor):
        return field_apply(self, x)

    def reset_state(self):
        for l in self.layers:
            l.ferro.reset_state()

    def regularization_loss(self, regularize_activation=1.0, regularize_entropy=1.0):
        return sum(l.kan.regularization_loss(regularize_activation, regularize_entropy) for l in self.layers)


class ODEFunc(CacheFreeState, nn.Module):
    """``func(t, y) = field(y)`` (the reference's calDeriv, train_kanfet_node_predprey.py:159-161),
    tagged so that ``fet_ode_amd.odeint`` integrates it in one fused launch."""

    def __init__(self, field: nn.Module):
        super().__init__()
        self.field = field

    @property
    def _fetode_field(self):
        return self.field

    def forward(self, t, y):
        return self.field(y)


def autonomous(field: nn.Module) -> ODEFunc:
    return ODEFunc(field)
