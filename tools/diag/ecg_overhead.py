"""Where the wall time of a resident ECG dopri5 solve goes (B=200, latent 64): full odeint call vs
the bare C-ABI launch, with and without a sync."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import fet_ode_amd as F
from fet_ode_amd import dopri5 as D5
from fet_ode_amd import ecg

dev = torch.device("cuda:0")
torch.manual_seed(0)
m = ecg.No_MLP_KANODEFunc(latent_dim=64, num_basis=10).to(dev)
h0 = torch.randn(200, 64, device=dev)
t = torch.tensor([0.0, 1.0])


def timeit(name, fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / n * 1e3:.3f} ms", flush=True)


with torch.no_grad():
    timeit("odeint (resident)", lambda: F.odeint(m, h0, t, method="dopri5", rtol=1e-3, atol=1e-4))
    timeit("_try_ecg_resident", lambda: D5._try_ecg_resident(m, h0, t, False, 1e-3, 1e-4, {}))
    timeit("field eval x1", lambda: m(0.0, h0))
    timeit("t.to(dev)", lambda: t.to(torch.float64).to(dev))
    # profile one call's host side
    import cProfile, pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        D5._try_ecg_resident(m, h0, t, False, 1e-3, 1e-4, {})
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(12)
