"""Host-side cache keys (no GPU): the descriptor / plan caches must follow every optimizer step,
including fused optimizers that update parameters without bumping version counters."""
import torch

import fet_ode_amd as F
from fet_ode_amd import _lib
from fet_ode_amd.autograd_ops import _handle_key


def _step(opt, m):
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    opt.step()


def test_fused_adam_does_not_bump_versions_but_invalidates_the_key():
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, fused=True)
    versions = [p._version for p in m.parameters()]
    k0 = _handle_key(m, 8, torch.device("cpu"))
    g0 = _lib.param_generation()
    _step(opt, m)
    assert [p._version for p in m.parameters()] == versions  # why the generation exists
    assert _lib.param_generation() == g0 + 1
    k1 = _handle_key(m, 8, torch.device("cpu"))
    assert k1[0] == k0[0] and k1[1] != k0[1]  # same descriptor, new values -> plan rebuilt


def test_plain_optimizers_invalidate_the_key():
    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5)
    for opt in (torch.optim.Adam(m.parameters(), lr=1e-3), torch.optim.SGD(m.parameters(), lr=1e-2)):
        k0 = _handle_key(m, 8, torch.device("cpu"))
        _step(opt, m)
        k1 = _handle_key(m, 8, torch.device("cpu"))
        assert k1[0] == k0[0] and k1[1] != k0[1]


def test_deepcopy_and_pickle_drop_hip_caches():
    """copy.deepcopy / pickle of the drop-in modules leave out the HIP caches of the instance
    (ctypes descriptors with raw pointers cannot be copied, and they describe the ORIGINAL's
    tensors); parameters and state come along (bench.py deep-copies the LV model)."""
    import copy
    import ctypes
    import pickle
    import fet_ode_amd as F
    from fet_ode_amd import ett

    class Desc(ctypes.Structure):
        _fields_ = [("p", ctypes.c_void_p)]

    torch.manual_seed(0)
    m = F.KANFET([2, 10, 2], grid_size=5)
    kan = m.layers[0].kan
    for mod in (m, kan, m.layers[0].ferro):
        mod.__dict__["_fetode_handle"] = (1, Desc())
    m2 = copy.deepcopy(m)
    m3 = pickle.loads(pickle.dumps(m))
    for c in (m2, m3):
        assert not [k for mod in c.modules() for k in mod.__dict__ if k.startswith("_fetode")]
        for (k1, v1), (k2, v2) in zip(m.state_dict().items(), c.state_dict().items()):
            assert k1 == k2 and torch.equal(v1, v2)
    f = ett.LatentNeuralODEForecaster(7, 96, 8)
    f.dynamics.net.__dict__["_fetode_wide_kf"] = (0, Desc())
    assert "_fetode_wide_kf" not in copy.deepcopy(f).dynamics.net.__dict__
    # the wide layers' flat parameter tensor of a live graph (autograd_ops._flat_params) is a
    # non-leaf tensor, which deepcopy refuses: it must not be copied either
    kan.__dict__["_fetode_flat"] = (kan.base_weight * 1.0, (), ([], 0), [True])
    assert "_fetode_flat" not in copy.deepcopy(m).layers[0].kan.__dict__
