import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd as F  # noqa: E402

torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5)
h = hashlib.sha1()
for k, v in m.state_dict().items():
    h.update(v.numpy().tobytes())
print("pid", os.getpid(), "threads", torch.get_num_threads(), "param hash", h.hexdigest()[:16], flush=True)
