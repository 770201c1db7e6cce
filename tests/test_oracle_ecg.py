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
