"""CPU ORACLE — test infrastructure only (see oracle/torch_ref.py for the rules).

Restatement of the MNIST Kuramoto + KANLinear classifier of the reference (SURVEY §8f rank 3,
BASELINE config "MNIST: Kuramoto + KANLinear(1568 -> 10)"), mnist_kuramoto_kan.py, in the
reference's own eager-op order, so that on CPU it reproduces the reference bit for bit (pinned by
tests/golden/mnist_*.npz, generated from the reference classes by tests/golden/make_golden_mnist.py):

  * LogisticBasis  :11-22   phi = 2 / (1 + exp(-a (x - b)))          (a, b: (in, nb))
  * KANLinear      :25-142  SiLU base + cubic B-spline branch (efficientkan's b_splines) +
                            logistic branch with a bias and no scaler:
                            out = (silu(x) Wb^T + B(x) (Ws * scaler)^T) + (phi Wl^T + bias)
  * Kuramoto2D     :145-199 theta = pi (2 x - 1); `steps` explicit Euler steps of
                            theta += dt (omega + K (cos(theta) S - sin(theta) C)), S / C the
                            4-neighbour sums of sin / cos (zero padded); features [cos, sin]
  * KuramotoKANClassifier :202-221  Kuramoto2D -> KANLinear(2 H W -> classes)
The product package never imports this module.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from . import torch_ref as O


@dataclass
class MnistKANParams:
    grid: torch.Tensor            # (in, G + 2k + 1)
    base_weight: torch.Tensor     # (out, in)
    spline_weight: torch.Tensor   # (out, in, G + k)
    spline_scaler: Optional[torch.Tensor]   # (out, in)
    a: Optional[torch.Tensor]     # (in, nb)
    b: Optional[torch.Tensor]
    logistic_weight: Optional[torch.Tensor]  # (out, in * nb)
    logistic_bias: Optional[torch.Tensor]    # (out,)
    spline_order: int = 3

    @classmethod
    def from_state_dict(cls, sd, prefix="", spline_order=3):
        g = lambda k: sd.get(prefix + k)
        return cls(g("grid"), g("base_weight"), g("spline_weight"), g("spline_scaler"), g("logistic_basis.a"),
                   g("logistic_basis.b"), g("logistic_weight"), g("logistic_bias"), spline_order)


def logistic_basis(x: torch.Tensor, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """mnist_kuramoto_kan.py:19-22."""
    x = x.unsqueeze(-1)
    return 2.0 / (1.0 + torch.exp(-a * (x - b)))


def kanlinear_forward(x: torch.Tensor, p: MnistKANParams) -> torch.Tensor:
    """mnist_kuramoto_kan.py:127-142 (base_activation = SiLU)."""
    out_f, in_f = p.base_weight.shape
    orig = x.shape
    x2 = x.reshape(-1, in_f)
    base_output = F.linear(F.silu(x2), p.base_weight)
    sw = p.spline_weight * p.spline_scaler.unsqueeze(-1) if p.spline_scaler is not None else p.spline_weight
    spline_output = F.linear(O.b_splines(x2, p.grid, p.spline_order).view(x2.size(0), -1), sw.view(out_f, -1))
    out = base_output + spline_output
    if p.logistic_weight is not None:
        phi = logistic_basis(x2, p.a, p.b).reshape(x2.size(0), -1)
        out = out + F.linear(phi, p.logistic_weight, p.logistic_bias)
    return out.reshape(*orig[:-1], out_f)


def neighbor_kernel(dtype=torch.float32) -> torch.Tensor:
    k = torch.zeros(1, 1, 3, 3, dtype=dtype)
    k[0, 0, 0, 1] = 1.0
    k[0, 0, 2, 1] = 1.0
    k[0, 0, 1, 0] = 1.0
    k[0, 0, 1, 2] = 1.0
    return k


def kuramoto_forward(x_img: torch.Tensor, K: torch.Tensor, omega: torch.Tensor, steps: int, dt: float,
                     kernel: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Kuramoto2D.forward, mnist_kuramoto_kan.py:179-199: (B, 1, H, W) -> (B, 2 H W)."""
    B = x_img.shape[0]
    kern = neighbor_kernel(x_img.dtype) if kernel is None else kernel
    theta = math.pi * (2.0 * x_img - 1.0)
    om = omega.expand(B, -1, -1, -1)
    for _ in range(steps):
        sin_t = torch.sin(theta)
        cos_t = torch.cos(theta)
        sin_n = F.conv2d(sin_t, kern, padding=1)
        cos_n = F.conv2d(cos_t, kern, padding=1)
        coupling = cos_t * sin_n - sin_t * cos_n
        theta = theta + dt * (om + K * coupling)
    feat = torch.cat([torch.cos(theta), torch.sin(theta)], dim=1)
    return feat.view(B, -1)


class ClassifierRef:
    """KuramotoKANClassifier.forward (:216-219)."""

    def __init__(self, sd, steps=10, dt=0.15):
        self.K, self.omega = sd["osc.K"], sd["osc.omega"]
        self.kernel = sd.get("osc.neighbor_kernel")
        self.head = MnistKANParams.from_state_dict(sd, "head.")
        self.steps, self.dt = steps, dt

    def __call__(self, x_img):
        feat = kuramoto_forward(x_img, self.K, self.omega, self.steps, self.dt, self.kernel)
        return kanlinear_forward(feat, self.head)


def mnist_x(batch: int, H: int = 28, W: int = 28, seed: int = 0, dtype=torch.float32) -> torch.Tensor:
    """Synthetic MNIST-shaped images in [0, 1] (the dataset is not in the image): a seeded blob
    per image plus noise, clamped like ToTensor's range."""
    g = torch.Generator().manual_seed(seed)
    yy = torch.linspace(-1, 1, H, dtype=torch.float64).view(1, H, 1)
    xx = torch.linspace(-1, 1, W, dtype=torch.float64).view(1, 1, W)
    c = (torch.rand(batch, 2, 1, 1, generator=g, dtype=torch.float64) - 0.5)
    r = 0.2 + 0.3 * torch.rand(batch, 1, 1, generator=g, dtype=torch.float64)
    d = ((yy - c[:, 0]) ** 2 + (xx - c[:, 1]) ** 2).sqrt()
    img = torch.exp(-((d - r) / 0.12) ** 2) + 0.05 * torch.rand(batch, H, W, generator=g, dtype=torch.float64)
    return img.clamp(0, 1).to(dtype).unsqueeze(1)
