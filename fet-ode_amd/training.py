"""One training iteration as ONE HIP graph replay (torch.cuda.CUDAGraph over the package's
launches): the reference's iteration (train_kanfet_node_predprey.py:252-257: odeint, MSE, backward,
Adam.step) issues ~40 host calls per iteration; on a slow or contended host their issue time
(0.64-0.67 ms measured against a 0.79 ms iteration) sets the rate.  Captured, the
host issues one graph launch.

The captured step must be shape-static and host-sync-free: inputs in fixed tensors (copy new data
into them between replays), an optimizer built with ``capturable=True`` (torch.optim.Adam(...,
fused=True, capturable=True)), no ``.item()``.  ``optimizer.zero_grad()`` may set the gradients to
None (torch's default, the reference's call): the captured backward then allocates them once from
the graph's pool and every replay writes the same buffers — and autograd keeps the fused backward's
gradient views as ``.grad`` instead of adding them into zeroed tensors (one add kernel per
parameter with ``set_to_none=False``: 24 of them per LV iteration, ≈ 10 % of it).  Every
replay re-runs everything the eager iteration runs, in the same order — the parameter plan rebuild
included (it is forced into the capture) — so replays are bitwise the eager iterations
(tools/diag/train_graph2.py).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from . import _lib


class CapturedStep:
    """``step = CapturedStep(fn)``; ``step()`` replays ``fn`` (one training iteration)."""

    def __init__(self, fn: Callable[[], Optional[torch.Tensor]], warmup: int = 3, device=None):
        self.fn = fn
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):      # warm-up: allocator pools, plans, cached schedules
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        # the iteration rebuilds the parameter plan after each optimizer step: make sure the
        # captured iteration contains that rebuild (the step counter invalidates cached plans)
        _lib._PARAM_GEN[0] += 1
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = fn()
        torch.cuda.synchronize(dev)

    def __call__(self):
        self.graph.replay()
        return self.out
