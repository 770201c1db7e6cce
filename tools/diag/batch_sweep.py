"""Kernel time of one 34-step rk4 solve (LV KAN-FET, bench workload) per batch size for the fused
rk4 kernels: v6 (one trajectory per 3-wave workgroup), v7 at one and two trajectories per wave and
v8 (one trajectory per two-wave workgroup): picks the switch points (fetode_fused_get_batch_ranges /
set_*).  The GPU clocks are settled first (~1 s of back-to-back B = 4096 solves)."""
import ctypes
import json
import os
import time
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
saved = (ctypes.c_int64 * 5)()
_lib.check(lib.fetode_fused_get_batch_ranges(ctypes.addressof(saved)), "ranges")
saved = list(saved)
with torch.no_grad():   # clock settle
    y4 = bench.lv_y0(4096, 0).to(dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for _ in range(20):
            F.odeint(F.autonomous(m), y4, t, method="rk4")
        torch.cuda.synchronize()
rows = []
for B in [int(b) for b in os.environ.get("SWEEP_B", "1,64,256,512,1024,1536,2048,3072,4096,8192").split(",")]:
    y0 = bench.lv_y0(B, 0).to(dev)
    r = {"B": B}
    for name, sm, t1, v8 in (("v6", 1 << 40, 0, 0), ("v7x1", 0, 1 << 40, 0), ("v7x2", 0, 0, 0),
                             ("v8", 0, 0, 1 << 40)):
        if name not in os.environ.get("SWEEP_K", "v6,v7x1,v7x2,v8").split(","):
            continue
        lib.fetode_fused_set_small_batch_max(sm)
        lib.fetode_fused_set_tpw1_range(0, t1)
        lib.fetode_fused_set_v8_range(0, v8)
        r[name + "_ms"] = bench.kernel_time_ms(m, y0, t, reps=50)
    rows.append(r)
    print(json.dumps(r), flush=True)
lib.fetode_fused_set_small_batch_max(saved[0])
lib.fetode_fused_set_tpw1_range(saved[1], saved[2])
lib.fetode_fused_set_v8_range(saved[3], saved[4])
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(REPO, "gpurun_out", "batch_sweep.json"), "w"), indent=1)
