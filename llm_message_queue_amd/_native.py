"""Loader for the in-tree native modules (``_lib/*.so``).

Host modules (``_mlq``) are rebuilt on demand with g++ if missing, since the
queue core is required on every host.  The HIP module (``_hipops``) is NEVER
silently replaced by a Python fallback on a GPU host: ``require_hipops()``
raises if the extension is missing or fails to load while a GPU is visible.
"""
from __future__ import annotations

import importlib
import os
import sys
import threading

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib")
_lock = threading.Lock()
_cache = {}


def _import(name: str):
    if _LIB not in sys.path:
        sys.path.insert(0, _LIB)
    return importlib.import_module(name)


def load(name: str, autobuild: bool = True):
    with _lock:
        if name in _cache:
            return _cache[name]
        try:
            mod = _import(name)
        except ImportError:
            if not autobuild:
                raise
            from . import _build
            _build.build(only=[name])
            importlib.invalidate_caches()
            mod = _import(name)
        _cache[name] = mod
        return mod


def mlq():
    return load("_mlq")


def hipops_available() -> bool:
    try:
        require_hipops()
        return True
    except Exception:
        return False


def require_hipops():
    """The HIP kernel module.  torch must be imported first so the process
    shares torch's HIP runtime (same SONAME ``libamdhip64.so.7``)."""
    import torch  # noqa: F401  (load order matters)
    return load("_hipops", autobuild=False)


def telemetry():
    return load("_telemetry", autobuild=True)


def shmring():
    return load("_shmring", autobuild=True)


def textcpu():
    """CPU twin of the text_analyze kernel (csrc/text/text_cpu.h)."""
    return load("_textcpu", autobuild=True)


def ingress():
    return load("_ingress", autobuild=True)
