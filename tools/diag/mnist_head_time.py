"""MNIST KANLinear head (1568 -> 10, mnist_kuramoto_kan.py:283) forward at B = 8192 by HIP events;
writes the output to gpurun_out/head_<tag>.pt for a bitwise A/B (env FETODE_WIDE_V1 picks the
kernel; TAG names the file)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402,F401
from fet_ode_amd import mnist  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", "8192"))
torch.manual_seed(0)
m = mnist.KuramotoKANClassifier()
# efficient_kan's init (curve2coeff's CPU lstsq) is not bitwise reproducible across processes: the
# first run saves its weights, later runs (the A/B) load them
sdp = "gpurun_out/head_sd.pt"
if os.path.exists(sdp):
    m.load_state_dict(torch.load(sdp, weights_only=True))
else:
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(m.state_dict(), sdp)
m = m.to(dev)
g = torch.Generator(device="cpu").manual_seed(1)
feat = (torch.rand(B, 1568, generator=g) * 2 - 1).to(dev)
with torch.no_grad():
    for _ in range(3):
        out = m.head(feat)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    a.record()
    for _ in range(n):
        out = m.head(feat)
    b.record()
    torch.cuda.synchronize()
tag = os.environ.get("TAG", "x")
os.makedirs("gpurun_out", exist_ok=True)
torch.save(out.cpu(), f"gpurun_out/head_{tag}.pt")
print(f"head B={B} [{tag}]: {a.elapsed_time(b) / n * 1e3:.1f} us per forward (head kernel + split reduce)", flush=True)
