"""Kernel time of one 34-step rk4 solve (LV KAN-FET, bench workload) per batch size for the v6
(one trajectory per 3-wave workgroup) and v4 (two trajectories per wave) fused kernels: picks the
small-batch switch point (fetode_fused_set_small_batch_max)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
rows = []
for B in [int(b) for b in os.environ.get("SWEEP_B", "1,64,256,512,1024,1536,2048,3072,4096,8192").split(",")]:
    y0 = bench.lv_y0(B, 0).to(dev)
    r = {"B": B}
    for name, sm, t1 in (("v6", 1 << 40, 0), ("v7x1", 0, 1 << 40), ("v7x2", 0, 0)):
        lib.fetode_fused_set_small_batch_max(sm)
        lib.fetode_fused_set_tpw1_range(0, t1)
        r[name + "_ms"] = bench.kernel_time_ms(m, y0, t)
    rows.append(r)
    print(json.dumps(r), flush=True)
lib.fetode_fused_set_small_batch_max(512)
lib.fetode_fused_set_tpw1_range(320, 1024)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(REPO, "gpurun_out", "batch_sweep.json"), "w"), indent=1)
