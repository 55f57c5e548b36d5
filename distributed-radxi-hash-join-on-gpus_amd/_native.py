"""Loader for the in-tree native extension (``_C*.so`` next to this file).

On a machine with a GPU the extension is REQUIRED: ``require_native()`` raises
instead of silently falling back, so a GPU test can never pass on a Python
path.  ``HPCJOIN_AUTOBUILD=1`` builds it on first import if missing.
"""
from __future__ import annotations

import importlib.util
import os
import sysconfig

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_C" + sysconfig.get_config_var("EXT_SUFFIX"))
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    if not os.path.exists(_SO) and os.environ.get("HPCJOIN_AUTOBUILD") == "1":
        from . import _build
        _build.build()
    try:
        spec = importlib.util.spec_from_file_location(__package__ + "._C", _SO)
        if spec is None or not os.path.exists(_SO):
            raise ImportError(f"native extension not built: {_SO} (run `python __graft_entry__.py build`)")
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        _mod = m
    except Exception as e:  # pragma: no cover - reported by require_native()
        _err = e


def native_available() -> bool:
    _load()
    return _mod is not None


def native():
    return require_native()


def require_native():
    _load()
    if _mod is None:
        raise RuntimeError(f"hpcjoin native extension unavailable: {_err}")
    return _mod


def so_path() -> str:
    return _SO
