"""ETT forecaster forward (bench.py ett_rate workload) wall time at B = 8192."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402

dev = torch.device("cuda:0")
r = bench.ett_rate(dev, batch=int(os.environ.get("ETT_B", "8192")), reps=2, with_cpu=False)
print({k: r[k] for k in ("value", "ms_per_batch", "finite")}, "CH", os.environ.get("FETODE_WIDE_CH", "8"), flush=True)
