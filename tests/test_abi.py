"""The C-ABI library builds for gfx950, loads, and exports exactly what include/fetode.h declares.
Host-only entry points (sizes, shape validation) are exercised without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "fetode.h")
LIB = os.path.join(REPO, "fet-ode_amd", "libfetode.so")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fetode_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(REPO, "fet-ode_amd", "csrc")], check=True)
    return ctypes.CDLL(LIB)


def test_exports_every_declared_symbol(lib):
    syms = declared_symbols()
    assert len(syms) >= 10
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (fetode_\w+)", out))
    assert set(syms) <= exported, set(syms) - exported
    for s in syms:
        getattr(lib, s)


def test_python_binding_covers_header():
    import fet_ode_amd
    assert set(declared_symbols()) == set(fet_ode_amd._lib.SIGNATURES)


def test_gfx950_code_object_present():
    """The offload bundle names its target (amdgcn-amd-amdhsa--gfx950)."""
    assert b"gfx950" in open(LIB, "rb").read()


def _lv_field(F, with_ferro=True):
    """Descriptors with fake non-null device pointers: only host code runs."""
    L = F._lib
    fake = 0x1000
    kan = [L.KANLinearDesc(2, 10, 5, 3, 10, 0, *[fake] * 8, 1.0),
           L.KANLinearDesc(10, 2, 5, 3, 10, 0, *[fake] * 8, 1.0)]
    fer = [L.FerroDesc(2, 10, 10, *[fake] * 5, 10.0, 0.8, None, 0),
           L.FerroDesc(10, 2, 10, *[fake] * 5, 10.0, 0.8, None, 0)] if with_ferro else None
    return L.FieldHandle(kan, fer, [])


def test_host_queries_without_gpu():
    import fet_ode_amd as F
    lib = F._lib.load()
    h = _lv_field(F)
    assert lib.fetode_state_width(h.ref) == 12
    nb = lib.fetode_plan_bytes(h.ref)
    # per layer (fetode_common.h LayerPlan): 4*in*out*K + out + out*in*(1+nb) + 2*in*nb
    # + in*12 knots + in*11 spans, pad to 4; + out*in*12*4 spline table + 1 flag, pad to 4
    def lp(i, o):
        n = 4 * i * o * 10 + o + o * i * 11 + 2 * i * 10 + i * 12 + i * 11
        n = (n + 3) // 4 * 4 + o * i * 12 * 4 + 1
        return (n + 3) // 4 * 4
    assert nb == 4 * (lp(2, 10) + lp(10, 2))
    assert lib.fetode_fused_supported(h.ref) == 1
    assert lib.fetode_fused_supported(_lv_field(F, False).ref) == 1
    assert lib.fetode_state_width(_lv_field(F, False).ref) == 0


def test_shape_errors_are_reported():
    import fet_ode_amd as F
    L = F._lib
    lib = L.load()
    fake = 0x1000
    kan = [L.KANLinearDesc(2, 10, 5, 3, 10, 0, *[fake] * 8, 1.0),
           L.KANLinearDesc(9, 2, 5, 3, 10, 0, *[fake] * 8, 1.0)]   # 10 != 9
    h = L.FieldHandle(kan, None, [])
    assert lib.fetode_plan_bytes(h.ref) == -1
    assert b"in_features" in lib.fetode_last_error()
    rc = lib.fetode_integrate_fixed(h.ref, fake, 2, fake, 4, fake, 1, fake, fake, fake, 2, fake, None, 0,
                                    None, None)
    assert rc == L.FETODE_EINVAL
    with pytest.raises(ValueError):
        L.check(rc, "integrate")
