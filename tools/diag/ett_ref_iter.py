"""The reference's own ETT training iteration (bench.ett_reference_iteration_rate) at a few field
scales / tolerances: attempts, nfev, ms per iteration, finiteness."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import bench
dev = torch.device("cuda:0")
for kw in [dict(rtol=1e-3, atol=1e-4, iters=1), dict(iters=1), dict(iters=2)]:
    print(json.dumps({**{k: v for k, v in kw.items()}, **bench.ett_reference_iteration_rate(dev, **kw)}), flush=True)
