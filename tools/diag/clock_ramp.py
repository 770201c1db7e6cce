"""Per-kernel time of the bench solve over a long back-to-back run (blocks of 100 calls timed with
HIP events): how much warm-up the GPU's clocks need before the timed steps."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, sd, y0, y0g, t = bench.make_problem(0, 1, "strong", dev)
y0d = y0.to(dev)
func = F.autonomous(model)
stream = torch.cuda.current_stream(dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(41)]
with torch.no_grad():
    F.odeint(func, y0d, t, method="rk4")
    torch.cuda.synchronize(dev)
    ev[0].record(stream)
    for blk in range(40):
        for _ in range(100):
            F.odeint(func, y0d, t, method="rk4")
        ev[blk + 1].record(stream)
    torch.cuda.synchronize(dev)
print(json.dumps([round(ev[i].elapsed_time(ev[i + 1]) / 100 * 1e3, 1) for i in range(40)]), flush=True)
