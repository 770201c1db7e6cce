"""ETT dopri5 training iteration (bench.ett_dopri5_train_rate's): host issue time vs GPU completion
for the forward and the backward, with the fused stage combine on / off (env-free: flips
dopri5._FUSED_COMB).  Host-bound when the call returns only just before the synchronize does."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import dopri5 as D, ett  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    c, P, batch = 96, 24, 2048
    torch.manual_seed(0)
    m = ett.LatentNeuralODEForecaster(num_features=7, context_len=c, pred_len=P, latent_dim=64, solver="dopri5",
                                      rtol=1e-3, atol=1e-4)
    with torch.no_grad():
        for n, p_ in m.dynamics.net.named_parameters():
            if n.endswith(("coef", "base_weight", "spline_weight", "logistic_weight")):
                p_.mul_(0.1)
    m = m.to(dev)
    g = torch.Generator().manual_seed(4)
    series = torch.cumsum(torch.randn(batch + c + P, 7, generator=g), 0) * 0.05
    ds = ett.EnergyWindowDataset(series, series[:, -1], c, P, device=dev)
    xb, yb = ds.batch(torch.arange(batch, device=dev))
    t_fut = torch.linspace(0.0, float(P - 1) * 0.05, steps=P, device=dev)
    for fused in (True, False, True):
        D._FUSED_COMB = fused
        sd = {k: v.clone() for k, v in m.state_dict().items()}
        rows = []
        for it in range(4):
            m.load_state_dict(sd)
            m.zero_grad(set_to_none=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c0 = time.process_time()
            loss = torch.nn.functional.mse_loss(m(xb, t_fut), yb)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            loss.backward()
            t3 = time.perf_counter()
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            c1 = time.process_time()
            if it:
                rows.append((t1 - t0, t2 - t0, t3 - t2, t4 - t2, c1 - c0, t4 - t0))
        mean = [sum(r[k] for r in rows) / len(rows) * 1e3 for k in range(6)]
        print(f"fused={fused}: fwd issue {mean[0]:.1f} / done {mean[1]:.1f} ms; bwd issue {mean[2]:.1f} / done "
              f"{mean[3]:.1f} ms; cpu {mean[4]:.1f} ms of wall {mean[5]:.1f} ms; nfev {F.dopri5.dopri5_solve.last.nfev}",
              flush=True)
    D._FUSED_COMB = True
    # where the host time goes: one iteration under cProfile
    import cProfile
    import pstats
    pr = cProfile.Profile()
    m.zero_grad(set_to_none=True)
    pr.enable()
    loss = torch.nn.functional.mse_loss(m(xb, t_fut), yb)
    loss.backward()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
