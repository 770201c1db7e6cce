"""Small driver for rocprofv3 PMC passes: the wide KAN-FET layer kernels at the ETT widths
(B = 8192) and the MNIST KANLinear head (B = 8192), a few launches each."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import mnist  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else "all"
with torch.no_grad():
    if which in ("all", "wide"):
        for (i, o) in [(64, 128), (128, 64)]:
            torch.manual_seed(2)
            m = F.KANFET([i, o], grid_size=5, num_fet_basis=10).to(dev)
            x = torch.rand(8192, i, device=dev) * 6 - 3
            for _ in range(5):
                m(x)
    if which in ("all", "mnist"):
        torch.manual_seed(0)
        head = mnist.KANLinear(1568, 10).to(dev)
        xh = torch.rand(8192, 1568, device=dev) * 2 - 1
        for _ in range(5):
            head(xh)
    torch.cuda.synchronize()
print("done")
