"""Host cost per field evaluation of KANFET([64, 128, 64]) under autograd (the ETT forecaster's
field in the dopri5 training forward, which is host-bound): B = 64 so the kernels are short, 500
evaluations, wall per evaluation; then the pieces of one wide layer call timed alone."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import fet_ode_amd as F  # noqa: E402
from fet_ode_amd import autograd_ops as A  # noqa: E402


def per_call(fn, n=500):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = F.KANFET([64, 128, 64], grid_size=5, num_fet_basis=10).to(dev)
    x = (torch.randn(64, 64, device=dev) * 0.5).requires_grad_(True)
    keep = []

    def ev():
        keep.append(m(x))
        if len(keep) > 40:
            keep.clear()
    print(f"field evaluation under autograd (2 wide layers): {per_call(ev):.1f} us", flush=True)
    with torch.no_grad():
        print(f"field evaluation, no_grad (fused or wide forward): {per_call(lambda: m(x)):.1f} us", flush=True)
    kan, fer = A.field_layers(m)[0]
    kp = [p for p in A.kan_params(kan) if p is not None]
    fp = [getattr(fer, n) for n in A.FERRO_PARAM_NAMES]
    xd = x.detach()
    print(f"wide_plans: {per_call(lambda: A.wide_plans(kan, fer, dev)):.1f} us", flush=True)
    print(f"_flat_params: {per_call(lambda: A._flat_params(kan, fer, kp + fp)):.1f} us", flush=True)
    ents = A.wide_plans(kan, fer, dev)
    print(f"wide_apply: {per_call(lambda: A.wide_apply(kan, fer, xd, False, entry=ents[0])):.1f} us", flush=True)
    print(f"_field_tensors grad check: {per_call(lambda: any(t.requires_grad for t in A._field_tensors(m))):.1f} us",
          flush=True)
    print(f"needs_reinit + branch_sign + commit: "
          f"{per_call(lambda: (fer._needs_reinit(xd), fer._branch_sign_for(xd), fer._commit_state(xd, False))):.1f} us",
          flush=True)

    def lg():
        keep.append(A.wide_layer_grad(kan, fer, x, False))
        if len(keep) > 40:
            keep.clear()
    print(f"wide_layer_grad (one layer): {per_call(lg):.1f} us", flush=True)


if __name__ == "__main__":
    main()
