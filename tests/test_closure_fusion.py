"""The reference's unchanged calDeriv closure (train_kanfet_node_predprey.py:159-161,
predator_prey.py:113-115) is recognised as the module call it is (fet_ode_amd.odeint.closure_field),
so odeint integrates it on the fused path; anything that does more than `return model(X)` is not.
Host-side only: the recognition inspects bytecode and module hooks, no GPU call."""
import torch

import fet_ode_amd as F
from fet_ode_amd.odeint import closure_field, fused_field

torch.manual_seed(0)
kan_fet_model = F.KANFET([2, 10, 2])
kan_model = F.KAN([2, 10, 2])


def calDeriv(t, X):  # the reference's exact shape
    dXdt = kan_fet_model(X)
    return dXdt


def calkan_model_Deriv(t, X):
    dXdt = kan_model(X)
    return dXdt


def test_reference_caldriv_shapes_recognised():
    assert closure_field(calDeriv) is kan_fet_model
    assert closure_field(calkan_model_Deriv) is kan_model
    assert closure_field(lambda tt, yy: kan_fet_model(yy)) is kan_fet_model
    m = F.KANFET([2, 10, 2])
    assert closure_field(lambda tt, yy: m(yy)) is m          # closure cell
    assert fused_field(calDeriv) is kan_fet_model
    assert fused_field(F.autonomous(m)) is m


def test_global_rebinding_followed():
    global kan_fet_model
    old = kan_fet_model
    try:
        kan_fet_model = F.KANFET([2, 10, 2])
        assert closure_field(calDeriv) is kan_fet_model
    finally:
        kan_fet_model = old


def test_other_closures_not_recognised():
    m = F.KANFET([2, 10, 2])
    assert closure_field(lambda tt, yy: m(yy) * 2.0) is None            # more than the call
    assert closure_field(lambda tt, yy: m(tt)) is None                  # called on t
    assert closure_field(lambda tt, yy, *a: m(yy)) is None              # *args
    assert closure_field(lambda tt, yy, *, k=1: m(yy)) is None          # keyword-only
    assert closure_field(lambda tt, yy: torch.tanh(yy)) is None         # not a field module
    lin = torch.nn.Linear(2, 2)
    assert closure_field(lambda tt, yy: lin(yy)) is None
    assert closure_field(m.forward) is None                             # bound method

    class Sub(F.KANFET):
        pass

    s = Sub([2, 10, 2])
    assert closure_field(lambda tt, yy: s(yy)) is None                  # a subclass may override forward

    def two_calls(t, X):
        h = m(X)
        return m(h)
    assert closure_field(two_calls) is None


def test_hooks_and_switch_disable_recognition():
    m = F.KANFET([2, 10, 2])
    f = lambda tt, yy: m(yy)  # noqa: E731
    h = m.register_forward_hook(lambda mod, i, o: None)
    assert closure_field(f) is None
    h.remove()
    assert closure_field(f) is m
    with F.closure_fusion(False):
        assert fused_field(f) is None
        assert fused_field(F.autonomous(m)) is m     # the explicit tag still fuses
    assert fused_field(f) is m


def test_unrecognised_closure_over_a_field_warns_once():
    """A closure that reaches a KAN / KANFET module but is not `return model(X)` runs per stage and
    says so once (per code object); closures over anything else stay silent."""
    import warnings
    m = F.KANFET([2, 10, 2])

    def scaled(t, X):
        return m(X) * 2.0

    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert closure_field(scaled) is None
        assert closure_field(scaled) is None
        lin = torch.nn.Linear(2, 2)
        assert closure_field(lambda tt, yy: lin(yy) * 2) is None
        h = m.register_forward_hook(lambda mod, i, o: None)
        hooked = lambda tt, yy: m(yy)  # noqa: E731
        assert closure_field(hooked) is None
        h.remove()
    msgs = [str(x.message) for x in w if issubclass(x.category, RuntimeWarning)]
    assert len(msgs) == 2, msgs
    assert "scaled" in msgs[0] and "stage by stage" in msgs[0]
    assert "hooks" in msgs[1]
