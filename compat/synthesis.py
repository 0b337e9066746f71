"""Reference-name shim: `from synthesis import build_model, wavegen` (as vocoder.py does)
resolves to the MI355X implementation autovc_amd.synthesis.  Put compat/ on PYTHONPATH
(INTEGRATION.md)."""
import os as _os
import sys as _sys

_sys.path.insert(0, _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
from autovc_amd.synthesis import *  # noqa: F401,F403,E402
from autovc_amd import synthesis as _impl  # noqa: E402

_sys.modules[__name__] = _impl
