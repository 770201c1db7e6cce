"""Wide KAN-FET layer VJP time at the ETT widths (B = 8192): forward under autograd and backward
(_WideLayerFn: the Ferro VJP + the KANLinear VJPs), HIP events over N calls; env B, N."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
B, N = int(os.environ.get("B", "8192")), int(os.environ.get("N", "10"))


def ev(fn, n=N):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for i, o in ((64, 128), (128, 64)):
    torch.manual_seed(1)
    x = (torch.rand(B, i, device=dev) * 6 - 3).requires_grad_(True)
    lay = F.KANFET([i, o], grid_size=5, num_fet_basis=10).to(dev)
    g = torch.randn(B, o, device=dev)
    lay(x.detach())                       # state for the stateful calls below
    fwd = ev(lambda: lay(x))
    ys = []

    def fb():
        y = lay(x)
        y.backward(g)
    tot = ev(fb)
    print(f"{i}->{o}: forward (autograd) {fwd:.1f} us, forward+backward {tot:.1f} us -> backward {tot - fwd:.1f} us",
          flush=True)
