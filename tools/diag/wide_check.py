"""Quick GPU check + timing of the wide KAN-FET layer kernel (fetode_wide.hip) against the oracle,
and the ETT forward at B=8192."""
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import fet_ode_amd as F  # noqa: E402
from oracle import torch_ref as O  # noqa: E402

dev = torch.device("cuda:0")
for (i, o, K) in [(64, 128, 10), (128, 64, 10), (64, 128, 12)]:
    torch.manual_seed(1)
    m = F.KANFET([i, o], grid_size=5, num_fet_basis=K)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(dev)
    ref = O.KANFETRef.from_state_dict(sd, 1)
    x = torch.rand(300, i) * 6 - 3
    for call in range(2):
        xx = x * (1 + 0.1 * call)
        with torch.no_grad():
            got = m(xx.to(dev)).cpu()
        exp = ref(xx)
        rel = ((got - exp).norm(dim=1) / exp.norm(dim=1)).max().item()
        print(f"KANFET[{i},{o}] K={K} call {call}: max row rel {rel:.3e}", flush=True)
# timing of one layer at B=8192
for (i, o) in [(64, 128), (128, 64)]:
    torch.manual_seed(2)
    m = F.KANFET([i, o], grid_size=5, num_fet_basis=10).to(dev)
    x = (torch.rand(8192, i, device=dev) * 6 - 3)
    with torch.no_grad():
        for _ in range(3):
            m(x)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        n = 20
        for _ in range(n):
            m(x)
        ev[1].record()
        torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / n
    el = 8192 * i * o * 10
    print(f"layer {i}->{o} B=8192: {ms * 1e3:.1f} us per call (incl. state copy), {el / (ms * 1e-3) / 1e12:.2f} T Ferro elements/s", flush=True)
