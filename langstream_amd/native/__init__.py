"""Host-side C++ runtime (``_lsnative.so``): in-memory topic log, tokenizers, KV block
allocator.  Built in-tree by ``langstream_amd._build``; built on demand if missing."""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_lsnative.so")
_lock = threading.Lock()
_mod = None


def lib():
    """Load (building first if needed) the native module."""
    global _mod
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is not None:
            return _mod
        if not os.path.exists(_SO):
            from .._build import build_native
            build_native()
        loader = importlib.machinery.ExtensionFileLoader("_lsnative", _SO)
        spec = importlib.util.spec_from_file_location("_lsnative", _SO, loader=loader)
        m = importlib.util.module_from_spec(spec)
        loader.exec_module(m)
        sys.modules["langstream_amd.native._lsnative"] = m
        _mod = m
    return _mod
