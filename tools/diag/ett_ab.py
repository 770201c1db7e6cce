"""ETT forecaster forward (bench.py ett_rate workload, B = 8192): time and the fp64-envelope parity
of windows 0-7, for A/B of the wide-layer builds (FETODE_LIB selects the library)."""
import json
import os
import sys
import threading
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402

def _beat():  # the CPU oracle legs print nothing for minutes: keep the run visibly alive
    while True:
        time.sleep(30)
        print("ett_ab: working", file=sys.stderr, flush=True)


threading.Thread(target=_beat, daemon=True).start()
dev = torch.device("cuda:0")
r = bench.ett_rate(dev, reps=4, with_cpu=True, cpu_seconds=1.0)
print(os.environ.get("AB_TAG", ""), json.dumps({"ms_per_batch": r["ms_per_batch"], "finite": r["finite"],
                                                 "parity": {k: v for k, v in r["parity"].items() if k != "note"}}),
      flush=True)
