"""Is the bench's odeint call slower per kernel than a bare launch? HIP-event time per call of
(a) F.odeint on the bench workload, (b) bench.kernel_time_ms's direct fetode_integrate_fixed
launch, (c) odeint again — 20 back-to-back calls each, interleaved rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import fet_ode_amd as F  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, sd, y0, y0g, t = bench.make_problem(0, 1, "strong", dev)
y0d = y0.to(dev)
func = F.autonomous(model)
stream = torch.cuda.current_stream(dev)


def odeint_ms(reps=20):
    with torch.no_grad():
        for _ in range(3):
            F.odeint(func, y0d, t, method="rk4")
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            F.odeint(func, y0d, t, method="rk4")
        e1.record(stream)
        torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / reps


out = {}
for r in range(3):
    out[f"odeint_{r}"] = odeint_ms()
    out[f"launch_{r}"] = bench.kernel_time_ms(model, y0d, t)
print(json.dumps(out), flush=True)
