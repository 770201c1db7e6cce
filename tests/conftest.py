import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libfetode.so")


def load_golden(name):
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def golden_sd(g, prefix="sd/"):
    import torch
    return {k[len(prefix):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(prefix)}


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test requested but torch.cuda.is_available() is False")
    return torch.device("cuda:0")


@pytest.fixture
def kernel_switch():
    """Force the fused integrator's kernel: small(True) -> v6 at any batch, small(False) -> v4 / v7 at
    two trajectories per wave (the one-per-wave range is switched off meanwhile)."""
    from fet_ode_amd import _lib
    lib = _lib.load()
    prev = lib.fetode_fused_set_small_batch_max(-1)
    prev_hi = lib.fetode_fused_set_tpw1_range(-1, 0)

    def small(on):
        lib.fetode_fused_set_small_batch_max(1 << 40 if on else 0)
    yield small
    lib.fetode_fused_set_small_batch_max(prev)
    lib.fetode_fused_set_tpw1_range(-1, prev_hi)


@pytest.fixture(params=[0, 1, 2, 6], ids=["one-kernel", "split", "lane-sweep", "lane-sweep-kansum"])
def bwd_split(request):
    """Run a fused-backward test through each sweep structure: the one-kernel sweep, the split
    (fetode_backward_set_split, diagnostic build), the lane-group sweep at every batch
    (fetode_backward_set_v7(2)) and the same with the KAN sums in kansum_kernel (mode 6)."""
    from fet_ode_amd import _lib
    lib = _lib.load()
    prev_v7 = lib.fetode_backward_set_v7(request.param if request.param in (2, 6) else 0)
    prev = lib.fetode_backward_set_split(1 if request.param == 1 else 0)
    if prev == -2:
        lib.fetode_backward_set_v7(prev_v7)
        pytest.skip("the split backward is in the diagnostic build only (make diag)")
    yield request.param
    lib.fetode_backward_set_split(prev)
    lib.fetode_backward_set_v7(prev_v7)
