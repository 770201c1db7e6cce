"""Inference solve kernel time (bench.kernel_time_ms: HIP events around the launch) of the library
FETODE_LIB at B = 4096 and 1024, median of 3 rounds of 20 launches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import bench

dev = torch.device("cuda:0")
model, sd, y0, y0g, t = bench.make_problem(0, 1, "strong", dev)
res = []
for B in (4096, 1024):
    y = y0[:B].to(dev).contiguous()
    with torch.no_grad():
        ms = sorted(bench.kernel_time_ms(model, y, t) for _ in range(3))[1]
    res.append(f"B={B}: {ms * 1e3:.1f} us")
print(os.path.basename(os.environ.get("FETODE_LIB", "libfetode.so")), "; ".join(res), flush=True)
