"""``dumps(obj)``: ``json.dumps(obj)`` (default options) through the native encoder
(``native/jsonenc.cpp``), byte-identical output; objects outside its type set fall back
to ``json.dumps``.  Used where records are serialised onto topics -- an embeddings
record's float vector costs ~0.7 us per float through ``json.dumps``."""
from __future__ import annotations

import json
from typing import Any

_native = None
_unsupported = None


def _load():
    global _native, _unsupported
    try:
        from ..native import lib
        m = lib()
        _native, _unsupported = m.json_dumps, m.JsonUnsupported
    except Exception:  # noqa: BLE001  (no toolchain: plain json)
        _native, _unsupported = False, None


def dumps(obj: Any) -> str:
    if _native is None:
        _load()
    if _native:
        try:
            return _native(obj)
        except _unsupported:
            pass
    return json.dumps(obj)
