"""Time the fused rk4 solve per kernel variant and batch (FETODE_FUSED_LPT is read once per
process, so run one process per variant)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import fet_ode_amd as F
from oracle import torch_ref as O

dev = torch.device("cuda:0")
tag = os.environ.get("FETODE_FUSED_LPT", "auto") + ("/" + os.path.basename(os.environ["FETODE_LIB"]) if "FETODE_LIB" in os.environ else "")
for B in [int(v) for v in os.environ.get("BATCHES", "1024,2048,4096,8192,16384,65536").split(",")]:
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2]).to(dev)
    f = F.autonomous(m)
    y0 = O.lv_y0(B).to(dev)
    t = torch.tensor(np.linspace(0, 3.5, 35))
    with torch.no_grad():
        for _ in range(3):
            F.odeint(f, y0, t, method="rk4")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            F.odeint(f, y0, t, method="rk4")
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
    print(f"{tag:>20s} B={B:6d}: {ms:7.3f} ms/solve  {34 * B / ms / 1e3:10.0f} traj-steps/ms", flush=True)
