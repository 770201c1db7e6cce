"""cProfile of the host side of KanFet_NODE.forward (B = 200, the bench's ECG workload)."""
import cProfile
import os
import pstats
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from fet_ode_amd import ecg  # noqa: E402
from oracle import ecg_ref as E  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=64, num_basis=10).to(dev).eval()
x = E.ecg_x(200, seed=1).to(dev)
with torch.no_grad():
    for _ in range(5):
        m(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        m(x)
    torch.cuda.synchronize()
    print(f"wall {1e3 * (time.perf_counter() - t0) / 50:.3f} ms per forward")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(100):
        m(x)
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(22)
