"""fet_ode_amd — MI355X-native Neural-ODE integrator for KAN / KAN-FET vector fields.

Drop-in surface of the reference hot path (sallywang147/FET-ODE):
  * ``odeint``               — torchdiffeq.odeint (euler, midpoint, rk4, dopri5)
  * ``efficientkan``         — LogisticBasis, KANLinear, KAN (+ KANFET)
  * ``ferro_class``          — FerroelectricBasis
  * ``ecg``                  — the ECG KAN-FET NODE (hysteretic LogisticBasis, KANFeatureMixer,
                               No_MLP_KANODEFunc, KanFet_NODE; train_ecg_kan_fet_nn_ode.py)
  * ``mnist``                — the MNIST Kuramoto + KANLinear classifier (mnist_kuramoto_kan.py)
  * ``ett``                  — odeint_rk4, EnergyWindowDataset, the KAN-FET LatentNeuralODEForecaster
                               and the KAN-RNN encoder (KANRNNEncoder, FullyNonlinearKANCell,
                               LogisticBasis, LogisticBasisLinear; train_kan_fet_ett.py)
  * ``training.CapturedStep`` — one training iteration replayed as one HIP graph
  * ``autonomous(field)``    — calDeriv-style func(t, y) = field(y) that odeint integrates in a
                               single fused HIP launch; the reference's own unchanged
                               ``def calDeriv(t, X): return kan_fet_model(X)`` is recognised as
                               the same thing (``set_closure_fusion`` / ``closure_fusion`` switch it)
All compute runs in libfetode.so (HIP, gfx950) through the C ABI of include/fetode.h.
"""
from . import _lib
from . import ecg, efficientkan, ett, ferro_class, lv, mnist, training
from .efficientkan import KAN, KANFET, KANFETLayer, KANLinear, LogisticBasis, ODEFunc, autonomous
from .ferro_class import FerroelectricBasis
from .odeint import SOLVERS, closure_fusion, odeint, set_closure_fusion, set_fused_training

__all__ = ["odeint", "SOLVERS", "set_fused_training", "set_closure_fusion", "closure_fusion", "KAN", "KANFET", "KANFETLayer", "KANLinear", "LogisticBasis",
           "FerroelectricBasis", "ODEFunc", "autonomous", "ecg", "efficientkan", "ett", "ferro_class", "lv", "mnist",
           "training"]
__version__ = "0.1.0"
