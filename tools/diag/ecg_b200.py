"""Batch-200 KanFet_NODE logits on the GPU (resident and host-driven dopri5) against the CPU
oracle in fp32 and fp64: per-row deviations, to tell a branch flip from a systematic error."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from fet_ode_amd import dopri5 as D5
from fet_ode_amd import ecg
from oracle import ecg_ref as E

dev = torch.device("cuda:0")
torch.manual_seed(0)
m0 = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=64, num_basis=10)
sd = {k: v.clone() for k, v in m0.state_dict().items()}
x = E.ecg_x(200, seed=1)
with torch.no_grad():
    l64 = E.ECGNodeRef({k: v.double() for k, v in sd.items()})(x.double())
    l32 = E.ECGNodeRef(sd)(x)
    for resident in (True, False):
        D5.set_resident_dopri5(resident)
        m = ecg.KanFet_NODE(T=96, num_classes=2, latent_dim=64, num_basis=10)
        m.load_state_dict(sd)
        m = m.to(dev).eval()
        lo = m(x.to(dev)).cpu().double()
        dr = (lo - l64).abs().max(dim=1).values
        top = torch.topk(dr, 5)
        print(f"resident={resident}: max {dr.max():.3e}, rows>1e-6: {(dr > 1e-6).sum().item()}, "
              f"top rows {top.indices.tolist()} {[f'{v:.2e}' for v in top.values.tolist()]}", flush=True)
        # the hidden state at t=1
        h0 = torch.nn.functional.linear(x.to(dev), m.encoder.weight, m.encoder.bias)
print("oracle fp32 vs fp64:", (l32.double() - l64).abs().max().item())
