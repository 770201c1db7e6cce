"""Wide KAN-FET layer forward (the ETT widths, B = 8192, K = 10) by HIP events, no autograd; the
outputs go to gpurun_out/wide_<TAG>_*.pt for a bitwise A/B across env settings (the weights are
saved by the first run and loaded by later ones: efficient_kan's lstsq init is not reproducible)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

dev = torch.device("cuda:0")
B, N, tag = int(os.environ.get("B", "8192")), int(os.environ.get("N", "20")), os.environ.get("TAG", "x")
os.makedirs("gpurun_out", exist_ok=True)
for i, o in ((64, 128), (128, 64)):
    torch.manual_seed(1)
    lay = F.KANFET([i, o], grid_size=5, num_fet_basis=10)
    sdp = f"gpurun_out/wide_sd_{i}_{o}.pt"
    if os.path.exists(sdp):
        lay.load_state_dict(torch.load(sdp, weights_only=True))
    else:
        torch.save(lay.state_dict(), sdp)
    lay = lay.to(dev)
    x = (torch.rand(B, i, generator=torch.Generator().manual_seed(2)) * 6 - 3).to(dev)
    with torch.no_grad():
        lay(x)  # the first call's reinit; later calls carry the state
        for _ in range(2):
            y = lay(x)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(N):
            y = lay(x)
        b.record()
        torch.cuda.synchronize()
    torch.save(y.cpu(), f"gpurun_out/wide_{tag}_{i}_{o}.pt")
    print(f"[{tag}] {i}->{o} B={B}: {a.elapsed_time(b) / N * 1e3:.1f} us per forward", flush=True)
