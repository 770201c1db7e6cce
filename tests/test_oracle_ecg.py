"""CPU: the ECG oracle restatement (oracle/ecg_ref.py) reproduces the reference's ECG classes
bit for bit (fixtures made from the reference classes by tests/golden/make_golden_ecg.py)."""
import numpy as np
import torch

from conftest import golden_sd, load_golden


def test_hlogistic_sequence_bitwise():
    from oracle import ecg_ref as E
    g = load_golden("ecg_hlogistic")
    p = E.HLogisticParams.from_state_dict(golden_sd(g))
    for c in range(4):
        y = E.hlogistic_forward(torch.from_numpy(g[f"x{c}"]), p)
        assert torch.equal(y, torch.from_numpy(g[f"y{c}"])), c
        assert torch.equal(p.prev_x, torch.from_numpy(g[f"prev_x{c}"])), c
        assert torch.equal(p.branch_state, torch.from_numpy(g[f"branch_state{c}"])), c
    # the row equal to the stored last row (dx = 0) takes the down branch (g = 0.5 is not > 0.5)
    assert (g["branch_state3"][2] == 0).all()


def test_hlogistic_grads_bitwise():
    from oracle import ecg_ref as E
    g = load_golden("ecg_hlogistic")
    sd = golden_sd(g)
    ps = {k: v.clone().requires_grad_(k in ("k", "Ec", "Ps", "bias", "coef")) for k, v in sd.items()}
    p = E.HLogisticParams.from_state_dict(ps)
    for c in range(4):
        with torch.no_grad():
            E.hlogistic_forward(torch.from_numpy(g[f"x{c}"]), p)
    x = torch.from_numpy(g["x5"]).requires_grad_(True)
    (E.hlogistic_forward(x, p) * torch.from_numpy(g["w5"])).sum().backward()
    assert torch.equal(x.grad, torch.from_numpy(g["grad/x"]))
    for n in ("k", "Ec", "Ps", "bias"):
        assert torch.equal(ps[n].grad, torch.from_numpy(g["grad/" + n])), n
    assert ps["coef"].grad is None and np.isnan(g["grad/coef"]).all()   # unused by forward


def _one_thread():
    """The fixtures were made single-threaded: the CPU GEMM's summation order depends on the
    thread count (F.linear differs by ~2e-7 otherwise)."""
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    return n


def test_field_bitwise():
    from oracle import ecg_ref as E
    n = _one_thread()
    g = load_golden("ecg_field")
    f = E.ECGFieldRef.from_state_dict(golden_sd(g))
    t = torch.tensor(0.0)
    assert torch.equal(f(t, torch.from_numpy(g["h1"])), torch.from_numpy(g["y1"]))
    assert torch.equal(f(t, torch.from_numpy(g["h2"])), torch.from_numpy(g["y2"]))
    torch.set_num_threads(n)


def test_node_dopri5_bitwise():
    from oracle import ecg_ref as E
    n = _one_thread()
    for name in ("ecg_node64", "ecg_node1"):
        g = load_golden(name)
        ref = E.ECGNodeRef(golden_sd(g), rtol=float(g["rtol"]), atol=float(g["atol"]))
        with torch.no_grad():
            lo = ref(torch.from_numpy(g["x"]))
        assert torch.equal(lo, torch.from_numpy(g["logits"])), name
        assert ref.trace.nfev == int(g["nfev"])
        got = np.array([[a[0], a[1], a[2], float(a[3])] for a in ref.trace.attempts])
        assert np.array_equal(got, g["attempts"]), name
    torch.set_num_threads(n)


def test_ferronet_field_bitwise():
    """KANFetODEFunc (train_ecg.py:986-1013): batch calls with the B > 1 first-call rule, a
    carried-state call with gradients, batch-1 calls (incl. a 1-D h) and a field saturating the
    +-50 clamp, against the reference class driven with the reference ferro_class."""
    from oracle import ecg_ref as E
    n = _one_thread()
    g = load_golden("ecg_ferronet_field")
    t = torch.tensor(0.0)
    sd = {k: v.clone().requires_grad_(v.dtype.is_floating_point and "prev_x" not in k and "branch_sign" not in k)
          for k, v in golden_sd(g, "sd_a/").items()}
    f = E.FerroNetFieldRef.from_state_dict(sd)
    with torch.no_grad():
        assert torch.equal(f(t, torch.from_numpy(g["a/h1"])), torch.from_numpy(g["a/y1"]))
    h2 = torch.from_numpy(g["a/h2"]).requires_grad_(True)
    y2 = f(t, h2)
    assert torch.equal(y2.detach(), torch.from_numpy(g["a/y2"]))
    (y2 * torch.from_numpy(g["a/w"])).sum().backward()
    assert torch.equal(h2.grad, torch.from_numpy(g["a/grad/h"]))
    for k in ("fc1.k", "fc1.Ec", "fc1.Ps", "fc1.bias", "fc1.coef", "fc2.k", "fc2.coef"):
        assert torch.equal(sd[k].grad, torch.from_numpy(g["a/grad/" + k])), k
    f = E.FerroNetFieldRef.from_state_dict(golden_sd(g, "sd_b/"))
    for c in range(3):
        assert torch.equal(f(t, torch.from_numpy(g[f"b/h{c}"])), torch.from_numpy(g[f"b/y{c}"])), c
    f = E.FerroNetFieldRef.from_state_dict(golden_sd(g, "sd_c/"))
    h = torch.from_numpy(g["c/h"]).requires_grad_(True)
    y = f(t, h)
    assert torch.equal(y.detach(), torch.from_numpy(g["c/y"])) and bool((y.abs() == 50).any())
    (y * torch.from_numpy(g["c/w"])).sum().backward()
    assert torch.equal(h.grad, torch.from_numpy(g["c/grad/h"]))
    torch.set_num_threads(n)


def test_ferronet_node_bitwise():
    """KanFet_MLP_NODE (train_ecg.py:1017-1059): per-row batch-1 solves, logits of the last row,
    euler (the __main__ config) and dopri5 (the class default)."""
    from oracle import ecg_ref as E
    n = _one_thread()
    for name, solver in (("ecg_ferronet_euler", "euler"), ("ecg_ferronet_dopri5", "dopri5")):
        g = load_golden(name)
        ref = E.FerroNetNodeRef(golden_sd(g), solver=solver, rtol=float(g["rtol"]), atol=float(g["atol"]))
        with torch.no_grad():
            lo = ref(torch.from_numpy(g["x"]))
        assert lo.shape == (1, 2)
        assert torch.equal(lo, torch.from_numpy(g["logits"])), name
        assert torch.equal(ref.field.st1.prev_x, torch.from_numpy(g["fc1_prev_x"])), name
        assert torch.equal(ref.field.st2.prev_x, torch.from_numpy(g["fc2_prev_x"])), name
    torch.set_num_threads(n)
