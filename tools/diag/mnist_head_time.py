"""MNIST head (KANLinear 1568 -> 10, MFMA wide kernel) forward time at B = 8192 by HIP events, and
its output checksum (variants must agree).  FETODE_LIB selects the library build."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fet_ode_amd import mnist  # noqa: E402
from oracle import mnist_ref as M  # noqa: E402

dev = torch.device("cuda:0")
torch.set_num_threads(1)
torch.manual_seed(0)
m = mnist.KuramotoKANClassifier().to(dev)
x = M.mnist_x(8192, seed=3).to(dev)
with torch.no_grad():
    feat = m.osc(x)
    for _ in range(5):
        out = m.head(feat)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(50):
        out = m.head(feat)
    b.record()
    torch.cuda.synchronize()
print(f"{os.environ.get('FETODE_LIB', 'default')}: head {a.elapsed_time(b) / 50 * 1e3:.1f} us/call, "
      f"checksum {float(out.double().abs().sum()):.9e}", flush=True)
