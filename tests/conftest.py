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


class fused_ranges:
    """Save every fused-integrator kernel switch (fetode_fused_get_batch_ranges: small-batch max,
    one-trajectory-per-wave range, two-waves-per-trajectory range) and restore exactly those values
    on exit — not literals, so a value set through the environment survives the test."""

    def __init__(self):
        import ctypes
        from fet_ode_amd import _lib
        self.lib = _lib.load()
        self.saved = (ctypes.c_int64 * 5)()
        _lib.check(self.lib.fetode_fused_get_batch_ranges(ctypes.addressof(self.saved)), "get_batch_ranges")
        self.saved = list(self.saved)

    def set(self, small=None, tpw1=None, v8=None):
        if small is not None:
            self.lib.fetode_fused_set_small_batch_max(small)
        if tpw1 is not None:
            self.lib.fetode_fused_set_tpw1_range(*tpw1)
        if v8 is not None:
            self.lib.fetode_fused_set_v8_range(*v8)
        return self

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        sm, t_lo, t_hi, v_lo, v_hi = self.saved
        self.lib.fetode_fused_set_small_batch_max(sm)
        self.lib.fetode_fused_set_tpw1_range(t_lo, t_hi)
        self.lib.fetode_fused_set_v8_range(v_lo, v_hi)
        return False


@pytest.fixture
def kernel_switch():
    """Force the fused integrator's kernel: small(True) -> v6 at any batch, small(False) -> v4 / v7 at
    two trajectories per wave (the one-per-wave and two-waves-per-trajectory ranges are switched off
    meanwhile)."""
    with fused_ranges() as fr:
        fr.set(tpw1=(-1, 0), v8=(-1, 0))

        def small(on):
            fr.set(small=(1 << 40) if on else 0)
        yield small


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
