"""Drop-in MNIST Kuramoto + KANLinear classifier, mnist_kuramoto_kan.py:
  * LogisticBasis          :11-22   phi = 2 / (1 + exp(-a (x - b))), a, b ~ N(0, 0.2^2)
  * KANLinear              :25-142  efficientkan's KANLinear with a logistic branch that has a bias
                                    and no scaler (out = base + spline + (phi Wl^T + bias))
  * Kuramoto2D             :145-199 phase oscillators on the pixel grid, `steps` Euler steps,
                                    features [cos theta | sin theta]
  * KuramotoKANClassifier  :202-221 Kuramoto2D -> KANLinear(2 H W -> classes)

Same constructor arguments, parameter / buffer names and shapes, init RNG order as the reference.
Kuramoto2D is one HIP launch per forward (a workgroup per image, all steps in LDS) with a HIP VJP
from a theta tape; the KANLinear head's forward is the MFMA kernel (fetode_kanlinear_wide_forward:
features once per (row, input), contraction on v_mfma_f32_16x16x4_f32, the logistic bias in its
epilogue), its backward the HIP KANLinear VJP kernels.  There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import _lib
from ._lib import CacheFreeState
from .autograd_ops import kan_backward, kan_params, kanlinear_apply


def _stream(x):
    return _lib.stream_handle(x.device)


class LogisticBasis(CacheFreeState, nn.Module):
    """mnist_kuramoto_kan.py:11-22 (used inside KANLinear's HIP kernel; standalone calls are the
    reference formula on the device)."""

    def __init__(self, in_dim: int, num_basis: int):
        super().__init__()
        self.in_dim = in_dim
        self.num_basis = num_basis
        self.a = nn.Parameter(torch.randn(in_dim, num_basis) * 0.2)
        self.b = nn.Parameter(torch.randn(in_dim, num_basis) * 0.2)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.dim() == 2 and x.size(1) == self.in_dim
        _lib.require_gpu_tensor(x, "LogisticBasis.forward")
        x = x.unsqueeze(-1)
        return 2.0 / (1.0 + torch.exp(-self.a * (x - self.b)))


class KANLinear(CacheFreeState, nn.Module):
    """mnist_kuramoto_kan.py:25-142."""

    def __init__(self, in_features, out_features, grid_size=5, spline_order=3, scale_noise=0.1, scale_base=1.0,
                 scale_spline=1.0, enable_standalone_scale_spline=True, base_activation=nn.SiLU, grid_eps=0.02,
                 grid_range=(-1.0, 1.0), use_logistic_basis=True, num_basis=10, scale_logistic=1.0):
        super().__init__()
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
        self.enable_standalone_scale_spline = enable_standalone_scale_spline
        if enable_standalone_scale_spline:
            self.spline_scaler = nn.Parameter(torch.empty(out_features, in_features))
        self.scale_noise = scale_noise
        self.scale_base = scale_base
        self.scale_spline = scale_spline
        self.base_activation = base_activation()
        self.grid_eps = grid_eps
        self.use_logistic_basis = use_logistic_basis
        self.num_basis = num_basis
        self.scale_logistic = scale_logistic
        if use_logistic_basis:
            self.logistic_basis = LogisticBasis(in_features, num_basis)   # draws a, b here (RNG order)
            self.logistic_weight = nn.Parameter(torch.empty(out_features, in_features * num_basis))
            self.logistic_bias = nn.Parameter(torch.zeros(out_features))
        self.reset_parameters()

    # the HIP KANLinear kernels' view of this variant: a logistic branch without scaler / scale
    enable_standalone_scale_logistic = False

    @property
    def enable_logistic_basis(self):
        return self.use_logistic_basis

    def reset_parameters(self):
        """:80-97 — same draws in the same order."""
        nn.init.kaiming_uniform_(self.base_weight, a=math.sqrt(5) * self.scale_base)
        with torch.no_grad():
            noise = ((torch.rand(self.grid_size + 1, self.in_features, self.out_features) - 0.5)
                     * self.scale_noise / self.grid_size)
            self.spline_weight.data.copy_(
                (self.scale_spline if not self.enable_standalone_scale_spline else 1.0)
                * self.curve2coeff(self.grid.T[self.spline_order:-self.spline_order], noise))
            if self.enable_standalone_scale_spline:
                nn.init.kaiming_uniform_(self.spline_scaler, a=math.sqrt(5) * self.scale_spline)
        if self.use_logistic_basis:
            nn.init.kaiming_uniform_(self.logistic_weight, a=math.sqrt(5) * self.scale_logistic)
            nn.init.zeros_(self.logistic_bias)

    def b_splines(self, x: torch.Tensor):
        """:99-109 (initialisation-time helper; the forward evaluates the bases in the kernel)."""
        assert x.dim() == 2 and x.size(1) == self.in_features
        grid = self.grid
        x = x.unsqueeze(-1)
        bases = ((x >= grid[:, :-1]) & (x < grid[:, 1:])).to(x.dtype)
        for k in range(1, self.spline_order + 1):
            left = (x - grid[:, :-(k + 1)]) / (grid[:, k:-1] - grid[:, :-(k + 1)])
            right = (grid[:, k + 1:] - x) / (grid[:, k + 1:] - grid[:, 1:(-k)])
            bases = left * bases[:, :, :-1] + right * bases[:, :, 1:]
        return bases.contiguous()

    def curve2coeff(self, x: torch.Tensor, y: torch.Tensor):
        """:111-117, least squares on the host at construction."""
        A = self.b_splines(x).transpose(0, 1)
        B = y.transpose(0, 1)
        solution = torch.linalg.lstsq(A, B).solution
        return solution.permute(2, 0, 1).contiguous()

    @property
    def scaled_spline_weight(self):
        if self.enable_standalone_scale_spline:
            return self.spline_weight * self.spline_scaler.unsqueeze(-1)
        return self.spline_weight

    def desc(self, keep: list) -> _lib.KANLinearDesc:
        def p(t):
            if t is None:
                return None
            t = _lib.f32c(t)
            keep.append(t)
            return t.data_ptr()
        lg = self.use_logistic_basis
        if not isinstance(self.base_activation, nn.SiLU):
            raise NotImplementedError("KANLinear: the HIP kernels implement base_activation=nn.SiLU")
        return _lib.KANLinearDesc(
            self.in_features, self.out_features, self.grid_size, self.spline_order, self.num_basis if lg else 0, 0,
            p(self.grid), p(self.base_weight), p(self.spline_weight),
            p(self.spline_scaler) if self.enable_standalone_scale_spline else None,
            p(self.logistic_basis.a) if lg else None, p(self.logistic_basis.b) if lg else None,
            p(self.logistic_weight) if lg else None, None, 1.0)

    def _wide_pack_for(self, d, keep):
        """The weights in the MFMA head's layout, re-packed whenever a weight tensor changes."""
        ws = [t for t in (self.base_weight, self.spline_weight, getattr(self, "spline_scaler", None),
                          getattr(self, "logistic_weight", None), self.grid) if t is not None]   # grid: basis tables
        key = (_lib.param_generation(), *((t.data_ptr(), t._version) for t in ws))
        cached = getattr(self, "_wide_cache", None)
        if cached is None or cached[0] != key:
            lib = _lib.load()
            wp = torch.empty(lib.fetode_kanlinear_wide_pack_bytes(_lib.ctypes.byref(d)) // 4, device=self.base_weight.device)
            _lib.check(lib.fetode_kanlinear_wide_pack(_lib.ctypes.byref(d), wp.data_ptr(), _stream(wp)),
                       "KANLinear wide pack")
            cached = (key, wp)
            self._wide_cache = cached
        return cached[1]

    def forward(self, x: torch.Tensor):
        assert x.size(-1) == self.in_features
        orig = x.shape
        x2 = x.reshape(-1, self.in_features)
        _lib.require_gpu_tensor(x2, "KANLinear.forward")
        keep = []
        if _lib.load().fetode_kanlinear_wide_supported(_lib.ctypes.byref(self.desc(keep))):
            bias = self.logistic_bias if self.use_logistic_basis else None
            out = _WideKANFn.apply(self, x2, bias, *kan_params(self))
        else:
            out = kanlinear_apply(self, x2)
            if self.use_logistic_basis:
                out = out + self.logistic_bias
        return out.reshape(*orig[:-1], self.out_features)


class _WideKANFn(torch.autograd.Function):
    """KANLinear + logistic bias, forward on the MFMA head kernel (fetode_kanlinear_wide_forward),
    backward on the HIP KANLinear VJP kernels."""

    @staticmethod
    def forward(ctx, mod, x, bias, *params):
        lib = _lib.load()
        keep = []
        d = mod.desc(keep)
        xc = _lib.f32c(x)
        B = xc.shape[0]
        wp = mod._wide_pack_for(d, keep)
        out = torch.empty(B, mod.out_features, device=x.device, dtype=torch.float32)
        ws = torch.empty(max(1, lib.fetode_kanlinear_wide_workspace(_lib.ctypes.byref(d), B) // 4), device=x.device)
        bc = _lib.f32c(bias) if bias is not None else None
        _lib.check(lib.fetode_kanlinear_wide_forward(_lib.ctypes.byref(d), wp.data_ptr(), _lib.ptr(bc), xc.data_ptr(), B,
                                                     out.data_ptr(), ws.data_ptr(), _stream(x)), "KANLinear.forward")
        ctx.mod = mod
        ctx.save_for_backward(xc)
        return out

    @staticmethod
    def backward(ctx, grad):
        (xc,) = ctx.saved_tensors
        gx, grads = kan_backward(ctx.mod, xc, grad, ctx.needs_input_grad[1], ctx.needs_input_grad[3:])
        gb = grad.sum(0) if ctx.needs_input_grad[2] else None
        return (None, gx, gb, *grads)


class _KuramotoFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, K, omega, steps, dt, training):
        lib = _lib.load()
        B, _, H, W = x.shape
        xc = _lib.f32c(x).view(B, H * W)
        Kc, oc = _lib.f32c(K).reshape(1), _lib.f32c(omega).reshape(H * W)
        feat = torch.empty(B, 2 * H * W, device=x.device, dtype=torch.float32)
        tape = torch.empty(B, steps + 1, H * W, device=x.device, dtype=torch.float32) if training else None
        _lib.check(lib.fetode_kuramoto_forward(xc.data_ptr(), B, H, W, steps, float(dt), Kc.data_ptr(), oc.data_ptr(),
                                               feat.data_ptr(), _lib.ptr(tape), _stream(x)), "Kuramoto2D.forward")
        if training:
            ctx.save_for_backward(tape, Kc)
            ctx.dims = (B, H, W, steps, float(dt))
        return feat

    @staticmethod
    def backward(ctx, gfeat):
        lib = _lib.load()
        tape, Kc = ctx.saved_tensors
        B, H, W, steps, dt = ctx.dims
        want = ctx.needs_input_grad
        g = _lib.f32c(gfeat)
        dev = g.device
        gx = torch.empty(B, 1, H, W, device=dev) if want[0] else None
        gK = torch.empty(1, device=dev) if want[1] else None
        gom = torch.empty(1, 1, H, W, device=dev) if want[2] else None
        ws = None
        if gK is not None or gom is not None:
            ws = torch.empty(max(1, lib.fetode_kuramoto_backward_workspace(B, H, W) // 4), device=dev)
        _lib.check(lib.fetode_kuramoto_backward(B, H, W, steps, dt, Kc.data_ptr(), tape.data_ptr(), g.data_ptr(),
                                                _lib.ptr(gx), _lib.ptr(gK), _lib.ptr(gom), _lib.ptr(ws), _stream(g)),
                   "Kuramoto2D backward")
        return gx, (gK.reshape(()) if gK is not None else None), gom, None, None, None


class Kuramoto2D(CacheFreeState, nn.Module):
    """mnist_kuramoto_kan.py:145-199."""

    def __init__(self, H=28, W=28, steps=10, dt=0.15, learn_K=True, learn_omega=True):
        super().__init__()
        self.H, self.W = H, W
        self.steps = steps
        self.dt = dt
        self.K = nn.Parameter(torch.tensor(0.5)) if learn_K else torch.tensor(0.5)
        if learn_omega:
            self.omega = nn.Parameter(torch.zeros(1, 1, H, W))
        else:
            self.register_buffer("omega", torch.zeros(1, 1, H, W))
        k = torch.zeros(1, 1, 3, 3)
        k[0, 0, 0, 1] = 1.0
        k[0, 0, 2, 1] = 1.0
        k[0, 0, 1, 0] = 1.0
        k[0, 0, 1, 2] = 1.0
        self.register_buffer("neighbor_kernel", k)
        self._cross = k.clone()

    def forward(self, x_img: torch.Tensor) -> torch.Tensor:
        B, C, H, W = x_img.shape
        assert C == 1 and H == self.H and W == self.W
        _lib.require_gpu_tensor(x_img, "Kuramoto2D.forward")
        if not torch.equal(self.neighbor_kernel.detach().cpu(), self._cross):
            raise NotImplementedError("Kuramoto2D: the HIP kernel implements the reference's fixed cross kernel")
        K = self.K if isinstance(self.K, torch.Tensor) else torch.tensor(self.K)
        K = K.to(x_img.device)
        training = torch.is_grad_enabled() and (x_img.requires_grad or K.requires_grad or self.omega.requires_grad)
        return _KuramotoFn.apply(x_img, K, self.omega, self.steps, self.dt, training)


class KuramotoKANClassifier(CacheFreeState, nn.Module):
    """mnist_kuramoto_kan.py:202-221."""

    def __init__(self, H=28, W=28, num_classes=10, kuramoto_steps=10, num_basis=8):
        super().__init__()
        self.osc = Kuramoto2D(H=H, W=W, steps=kuramoto_steps, dt=0.15, learn_K=True, learn_omega=True)
        in_dim = 2 * H * W
        self.head = KANLinear(in_dim, num_classes, grid_size=5, spline_order=3, base_activation=nn.SiLU,
                              use_logistic_basis=True, num_basis=num_basis)

    def forward(self, x_img):
        feat = self.osc(x_img)
        return self.head(feat)
