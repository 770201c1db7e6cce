"""Host-side cost of one resident ECG dopri5 call (B=200, latent 64): the whole _try_ecg_resident,
the C-ABI launch call alone, and the status read, averaged over N calls."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from fet_ode_amd import dopri5 as D5
from fet_ode_amd import ecg, _lib

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = ecg.No_MLP_KANODEFunc(latent_dim=64, num_basis=10).to(dev)
h0 = torch.randn(200, 64, device=dev)
t = torch.tensor([0.0, 1.0])
lib = _lib.load()
acc = {"launch": 0.0}
real = lib.fetode_ecg_dopri5


class Timed:
    def __call__(self, *a):
        t0 = time.perf_counter()
        r = real(*a)
        acc["launch"] += time.perf_counter() - t0
        return r


lib.fetode_ecg_dopri5 = Timed()
n = 200
with torch.no_grad():
    for _ in range(20):
        D5._try_ecg_resident(m, h0, t, False, 1e-3, 1e-4, {})
    torch.cuda.synchronize()
    acc["launch"] = 0.0
    t0 = time.perf_counter()
    for _ in range(n):
        D5._try_ecg_resident(m, h0, t, False, 1e-3, 1e-4, {})
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
print(f"per call: total {tot / n * 1e6:.1f} us, C-ABI launch call {acc['launch'] / n * 1e6:.1f} us", flush=True)
