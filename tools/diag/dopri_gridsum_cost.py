"""Where the LV resident dopri5 solve's time goes: bench.lv_dopri5_rate with the library FETODE_LIB
(the normal one, or a diagnostic build with -DFETODE_EXP_NO_GRIDSUM: every grid-wide norm replaced
by the workgroup's own value x grid size — no synchronisation, same evaluation count when the
control follows the same path) at rtol 1e-3 and 1e-7."""
import json, os, sys
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import bench  # noqa: E402

dev = torch.device("cuda:0")
model, sd, y0, y0g, t = bench.make_problem(0, 1, "strong", dev)
out = {"lib": os.environ.get("FETODE_LIB", "default")}
for rtol, atol in ((1e-3, 1e-4), (1e-7, 1e-9)):
    r = bench.lv_dopri5_rate(sd, y0.to(dev), t, reps=3, rtol=rtol, atol=atol)
    out[f"rtol{rtol:g}"] = {k: r[k] for k in ("ms_per_solve", "attempts", "nfev", "resident")}
print(json.dumps(out), flush=True)
