"""Wide-layer kernel time split: KAN-FET layer vs Ferro alone vs KANLinear alone (B = 8192, ETT
widths), per call, HIP events over 20 calls."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")


def timed(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


with torch.no_grad():
    for i, o in ((64, 128), (128, 64)):
        torch.manual_seed(1)
        x = torch.rand(8192, i, device=dev) * 6 - 3
        lay = F.KANFET([i, o], grid_size=5, num_fet_basis=10).to(dev)
        fer = F.FerroelectricBasis(i, o, 10).to(dev)
        kan = F.KANLinear(i, o).to(dev)
        print(f"{i}->{o}: KANFET layer {timed(lambda: lay(x)):.1f} us, Ferro alone {timed(lambda: fer(x)):.1f} us, "
              f"KANLinear alone {timed(lambda: kan(x)):.1f} us", flush=True)
