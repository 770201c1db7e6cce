"""Time the KAN-RNN encoder kernels at the ETT bench size (B = 8192, T = 96, F = 7, H = 64,
latent 64, 10 bases): no-grad forward (cone), full-recurrence forward, forward with tape, backward."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import fet_ode_amd  # noqa: E402,F401
from fet_ode_amd import _lib, ett  # noqa: E402

dev = torch.device("cuda:0")
B, T = int(os.environ.get("B", 8192)), 96
torch.manual_seed(0)
enc = ett.KANRNNEncoder(7, 64, 64, 10).to(dev)
x = torch.cumsum(torch.randn(B, T, 7, device=dev), 1) * 0.1
lib = _lib.load()
keep = []
d = ett._rnn_desc(enc.rnn_cell, enc.to_latent, keep)
z0 = torch.empty(B, 64, device=dev)
h = torch.empty(B, 64, device=dev)
tape = torch.empty(B, T, 64, device=dev)
s = _lib.stream_handle(dev)


def timed(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


us_cone = timed(lambda: lib.fetode_kanrnn_forward(_lib.ctypes.byref(d), x.data_ptr(), B, T, None, None,
                                                  z0.data_ptr(), None, 0, s))
us_full = timed(lambda: lib.fetode_kanrnn_forward(_lib.ctypes.byref(d), x.data_ptr(), B, T, None, None,
                                                  z0.data_ptr(), None, 1, s))
us_tape = timed(lambda: lib.fetode_kanrnn_forward(_lib.ctypes.byref(d), x.data_ptr(), B, T, None, h.data_ptr(),
                                                  z0.data_ptr(), tape.data_ptr(), 1, s))
g = torch.randn(B, 64, device=dev)
gp = [torch.empty_like(p) for p in (enc.rnn_cell.input_basis.a, enc.rnn_cell.input_basis.b,
                                    enc.rnn_cell.hidden_basis.a, enc.rnn_cell.hidden_basis.b)]
d2 = ett._rnn_desc(enc.rnn_cell, None, keep)
ws = torch.empty(lib.fetode_kanrnn_backward_workspace(_lib.ctypes.byref(d2), B) // 4 + 1, device=dev)
gx = torch.empty_like(x)
us_bwd = timed(lambda: lib.fetode_kanrnn_backward(_lib.ctypes.byref(d2), x.data_ptr(), B, T, None, tape.data_ptr(),
                                                  g.data_ptr(), gx.data_ptr(), None, *(t.data_ptr() for t in gp),
                                                  ws.data_ptr(), s))


def step():
    enc.zero_grad(set_to_none=True)
    z = enc(x)
    z.backward(g)


us_train = timed(step, 20)
print(f"B={B} T={T}: fwd cone {us_cone:.1f} us, fwd full {us_full:.1f} us, fwd+tape {us_tape:.1f} us, "
      f"bwd {us_bwd:.1f} us, module train step {us_train:.1f} us")
