"""Reference-name shim: `from model_bl import D_VECTOR` (as make_metadata.py does) resolves to
the MI355X implementation autovc_amd.model_bl.  Put compat/ on PYTHONPATH."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from autovc_amd.model_bl import *  # noqa: F401,F403,E402
from autovc_amd import model_bl as _impl  # noqa: E402

_sys.modules[__name__] = _impl
