"""``dumps(obj)``: the JSON text of a map / list record value as the reference runtime
writes it onto a topic (Jackson: compact separators, non-ASCII as itself) --
``json.dumps(obj, separators=(",", ":"), ensure_ascii=False)`` -- through the native
encoder (``native/jsonenc.cpp``), byte-identical output; objects outside its type set
fall back to ``json.dumps`` with the same options.  Used where records are serialised
onto topics -- an embeddings record's float vector costs ~0.7 us per float through
``json.dumps``.

``Float32List``: a list of floats that hold float32 values (a local model's embedding
row).  The native encoder writes each with its shortest float32 digits (~9 significant
digits instead of the ~17 a widened double needs): half the record bytes, a quarter of
the formatting time, and the same float32 after parsing -- the one place the output
differs from ``json.dumps`` text (not in value).  It is a mutable list: when any item is
not exactly a float32 value (user or EL code stored a double in it), the whole list is
written with double digits, byte-identical to ``json.dumps``.  Everywhere else it is a
plain list (json.dumps, msgpack, EL, the vector stores)."""
from __future__ import annotations

import datetime as _dt
import json
from typing import Any

_native = None
_unsupported = None
SEPARATORS = (",", ":")


class Float32List(list):
    """A list whose float items are float32 values (see the module docstring)."""
    __slots__ = ()


_f32_rows_native = None


def f32_rows(t) -> list:
    """Host float tensor / array [n, d] -> n Float32Lists (built natively: the PyFloat
    objects of a 384-wide row cost ~50 us through tolist() + a copy on a slow host)."""
    import numpy as np
    if _native is None:
        _load()
    if _f32_rows_native:
        a = t.numpy() if hasattr(t, "numpy") and not isinstance(t, np.ndarray) else t
        a = np.ascontiguousarray(a, dtype=np.float32)
        if a.ndim == 2:
            return _f32_rows_native(a)
    return [Float32List(r) for r in t.tolist()]


def f32_matrix(rows):
    """A list of equal-length number lists -> float32 [n, d] ndarray (native when built;
    numpy otherwise).  Raises ValueError on ragged or non-numeric rows."""
    import numpy as np
    if _native is None:
        _load()
    fn = _f32_matrix_native
    if fn is not None:
        return fn(rows)
    return np.asarray(rows, dtype=np.float32).reshape(len(rows), -1)


_f32_matrix_native = None


def _load():
    global _native, _unsupported
    try:
        from ..native import lib
        m = lib()
        _native, _unsupported = m.json_dumps, m.JsonUnsupported
        if hasattr(m, "json_register_f32list"):
            m.json_register_f32list(Float32List)
            global _f32_rows_native
            _f32_rows_native = getattr(m, "f32_rows", None)
        global _f32_matrix_native
        _f32_matrix_native = getattr(m, "f32_matrix", None)
    except Exception:  # noqa: BLE001  (no toolchain: plain json)
        _native, _unsupported = False, None


def _default(o: Any) -> Any:
    """Values the JSON writer has no form for: the Java date-time types of
    api/temporal.py -- java.util.Date / Timestamp / Time as epoch millis (Jackson's default
    for Date), the java.time ones as their ISO text; bytes as base64 (Jackson's byte[]),
    decimals as numbers."""
    from ..api import temporal
    if isinstance(o, (temporal.JDate, temporal.Timestamp, temporal.Time)):
        return o.get_time()
    if isinstance(o, (temporal.Instant, temporal.LocalTime, temporal.LocalDateTime, temporal.OffsetDateTime)):
        return str(o)
    if isinstance(o, (_dt.date, _dt.time)):
        return o.isoformat()
    if isinstance(o, (bytes, bytearray, memoryview)):   # Jackson: byte[] / ByteBuffer as base64
        import base64
        return base64.b64encode(bytes(o)).decode()
    from decimal import Decimal
    if isinstance(o, Decimal):
        return float(o)
    raise TypeError(f"Object of type {type(o).__name__} is not JSON serializable")


def dumps(obj: Any) -> str:
    if _native is None:
        _load()
    if _native:
        try:
            return _native(obj)
        except _unsupported:
            pass
    s = json.dumps(obj, default=_default, separators=SEPARATORS, ensure_ascii=False)
    try:
        s.encode("utf-8")
    except UnicodeEncodeError:   # lone surrogates: \u escapes keep the text encodable
        s = json.dumps(obj, default=_default, separators=SEPARATORS)
    return s
