"""Kuramoto front end (mnist_kuramoto_kan.py:145-199) at B = 8192, 28 x 28, 10 steps: forward and
backward kernel time by HIP events, lane-per-column kernels vs the LDS kernels
(fetode_kuramoto_set_lds)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402,F401
from fet_ode_amd import _lib, mnist  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
B = int(os.environ.get("B", "8192"))
torch.manual_seed(0)
m = mnist.Kuramoto2D(H=28, W=28, steps=10, dt=0.15).to(dev)
x = torch.rand(B, 1, 28, 28, device=dev).requires_grad_(True)
gy = torch.randn(B, 2 * 784, device=dev)


def ev_ms(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


for lds in (0, 1):
    lib.fetode_kuramoto_set_lds(lds)
    with torch.no_grad():
        f = ev_ms(lambda: m(x))

    def step():
        y = m(x)
        y.reshape(B, -1).backward(gy)
    fb = ev_ms(step)
    print(f"{'LDS ' if lds else 'lane'} kernels B={B}: forward {f * 1e3:.1f} us, fwd(tape)+bwd {fb * 1e3:.1f} us",
          flush=True)
lib.fetode_kuramoto_set_lds(0)
