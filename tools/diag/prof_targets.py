"""Small driver for rocprofv3 PMC passes: the wide KAN-FET layer kernels at the ETT widths
(B = 8192), the MNIST KANLinear head (B = 8192), the LV rk4 solve at the strong-scaling shard
(B = 512, v6) and the full batch (B = 4096, v4), the LV training step (B = 4096 rk4 forward
with tape + the fused reverse sweep) and the ETT KAN-RNN encoder (B = 8192), a few launches each.  argv[1] / $PROF_WHICH selects one."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import mnist  # noqa: E402

dev = torch.device("cuda:0")
which = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("PROF_WHICH", "all")
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
        clf = mnist.KuramotoKANClassifier().to(dev)          # the bench's classifier (head nb 8)
        xh = torch.rand(8192, 1568, device=dev) * 2 - 1
        img = torch.rand(8192, 1, 28, 28, device=dev)
        for _ in range(5):
            clf.head(xh)
            clf(img)
    torch.cuda.synchronize()
if which in ("all", "small"):   # the strong-scaling shard (v6, B = 512) next to the full batch (v4)
    import numpy as np
    import bench
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    with torch.no_grad():
        for B in (512, 1024, 4096):
            y0 = bench.lv_y0(B, 0).to(dev)
            for _ in range(4):
                F.odeint(F.autonomous(m), y0, t, method="rk4")
    torch.cuda.synchronize()
if which == "shard":   # the 8-way strong shard B = 512: v7 one trajectory per wave (default) then v6 forced
    import numpy as np
    import bench
    from fet_ode_amd import _lib
    lib = _lib.load()
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    y0 = bench.lv_y0(512, 0).to(dev)
    with torch.no_grad():
        for _ in range(4):
            F.odeint(F.autonomous(m), y0, t, method="rk4")
        lo = lib.fetode_fused_set_tpw1_range(-1, 0)
        prev = lib.fetode_fused_set_small_batch_max(1 << 40)
        for _ in range(4):
            F.odeint(F.autonomous(m), y0, t, method="rk4")
        lib.fetode_fused_set_small_batch_max(prev)
        lib.fetode_fused_set_tpw1_range(-1, lo)
    torch.cuda.synchronize()
if which in ("all", "train"):
    import numpy as np
    import bench
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
    y0 = bench.lv_y0(4096, 0).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    for _ in range(4):
        m.zero_grad()
        F.odeint(F.autonomous(m), y0, t, method="rk4").square().mean().backward()
    torch.cuda.synchronize()
if which in ("all", "enc"):   # the ETT KAN-RNN encoder at the bench size: forward (cone), training step
    from fet_ode_amd import ett
    torch.manual_seed(0)
    enc = ett.KANRNNEncoder(7, 64, 64, 10).to(dev)
    xe = torch.cumsum(torch.randn(8192, 96, 7, device=dev), 1) * 0.1
    with torch.no_grad():
        for _ in range(4):
            enc(xe)
    for _ in range(3):
        enc.zero_grad(set_to_none=True)
        enc(xe).square().mean().backward()
    torch.cuda.synchronize()
print("done")
