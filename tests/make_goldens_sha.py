"""The op-log SHA-256 of tools/make_ref_goldens.py (log_sha), for tests that regenerate fixture logs."""
import importlib.util
import os

_spec = importlib.util.spec_from_file_location(
    "make_ref_goldens", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tools", "make_ref_goldens.py"))
_m = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_m)
log_sha = _m.log_sha
