"""Import shim for the package directory ``fet-ode_amd/``.

The package lives in a hyphenated directory (repo layout), which Python cannot
name in an import statement; this module loads it under the importable name
``fet_ode_amd`` so that ``import fet_ode_amd`` and
``from fet_ode_amd import odeint, KANFET`` work from the repo root.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_dir = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "fet-ode_amd")
_spec = _ilu.spec_from_file_location(__name__, _os.path.join(_dir, "__init__.py"),
                                     submodule_search_locations=[_dir])
_mod = _ilu.module_from_spec(_spec)
_sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
