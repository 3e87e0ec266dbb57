"""Command output in the reference CLI's formats (``langstream-cli/.../commands/BaseCmd.java``
``print`` / ``printRows``):

* ``json``: the pretty-printed layout of the reference's JSON printer -- two-space
  indent, ``"key" : value``, arrays inline as ``[ a, b ]`` (``[ ]`` / ``{ }`` when
  empty), key order as received;
* ``yaml``: a ``---`` document, every string double-quoted, block mappings and sequences
  (sequence items at their key's indentation), ``[]`` / ``{}`` when empty;
* ``raw``: a table whose header is the upper-cased column names; every column is padded
  to the longest cell of the whole table, columns two spaces apart.

Floating-point numbers print as Java's ``Double.toString`` does (``1.0E10``, ``0.001``);
strings keep non-ASCII characters as themselves.
"""
from __future__ import annotations

import json
import math
from typing import Any, Callable, List, Optional, Sequence

__all__ = ["jackson_json", "jackson_yaml", "table", "render"]


def _shortest(a: float):
    """(significant digits, decimal exponent of the first one) of repr(a), a > 0."""
    s = repr(a)
    m, _, e = s.partition("e")
    e = int(e) if e else 0
    ip, _, fp = m.partition(".")
    if ip.strip("0"):
        exp10 = len(ip.lstrip("0")) - 1 + e
    else:
        exp10 = -(len(fp) - len(fp.lstrip("0")) + 1) + e
    digits = (ip + fp).lstrip("0").rstrip("0") or "0"
    return digits, exp10


def java_double(x: float) -> str:
    """``Double.toString``: positional for 1e-3 <= |x| < 1e7, else d.dddE[-]n."""
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    a = abs(x)
    d, e = _shortest(a)
    if 1e-3 <= a < 1e7:
        if e >= 0:
            ip = d[:e + 1].ljust(e + 1, "0")
            fp = d[e + 1:] or "0"
        else:
            ip, fp = "0", "0" * (-e - 1) + d
        return f"{sign}{ip}.{fp}"
    return f"{sign}{d[0]}.{d[1:] or '0'}E{e}"


def _scalar_json(v: Any) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return java_double(v)
    return json.dumps(v, ensure_ascii=False)


def jackson_json(v: Any, level: int = 0) -> str:
    if isinstance(v, dict):
        if not v:
            return "{ }"
        pad = "  " * (level + 1)
        items = [f'{pad}{json.dumps(str(k), ensure_ascii=False)} : {jackson_json(x, level + 1)}' for k, x in v.items()]
        return "{\n" + ",\n".join(items) + "\n" + "  " * level + "}"
    if isinstance(v, (list, tuple)):
        if not v:
            return "[ ]"
        return "[ " + ", ".join(jackson_json(x, level) for x in v) + " ]"
    return _scalar_json(v)


def _yaml_str(s: str) -> str:
    return json.dumps(s, ensure_ascii=False)


def _yaml_scalar(v: Any) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return java_double(v)
    return _yaml_str(str(v))


def _yaml_block(v: Any, level: int, out: List[str]) -> None:
    pad = "  " * level
    if isinstance(v, dict):
        for k, x in v.items():
            key = _yaml_str(str(k)) if not str(k).replace("-", "").replace("_", "").isalnum() else str(k)
            if isinstance(x, dict) and x:
                out.append(f"{pad}{key}:")
                _yaml_block(x, level + 1, out)
            elif isinstance(x, (list, tuple)) and x:
                out.append(f"{pad}{key}:")
                _yaml_seq(x, level, out)
            else:
                out.append(f"{pad}{key}: {_yaml_inline(x)}")
    elif isinstance(v, (list, tuple)):
        _yaml_seq(v, level, out)
    else:
        out.append(pad + _yaml_scalar(v))


def _yaml_seq(v, level: int, out: List[str]) -> None:
    pad = "  " * level
    for x in v:
        if isinstance(x, dict) and x:
            sub: List[str] = []
            _yaml_block(x, level + 1, sub)
            first = sub[0][len("  " * (level + 1)):]
            out.append(f"{pad}- {first}")
            out.extend(sub[1:])
        elif isinstance(x, (list, tuple)) and x:
            sub = []
            _yaml_seq(x, level + 1, sub)
            out.append(f"{pad}- {sub[0].lstrip()}")
            out.extend(sub[1:])
        else:
            out.append(f"{pad}- {_yaml_inline(x)}")


def _yaml_inline(x: Any) -> str:
    if isinstance(x, dict):
        return "{}"
    if isinstance(x, (list, tuple)):
        return "[]"
    return _yaml_scalar(x)


def jackson_yaml(v: Any) -> str:
    if isinstance(v, (dict, list, tuple)) and not v:
        return "--- " + _yaml_inline(v)
    if not isinstance(v, (dict, list, tuple)):
        return "--- " + _yaml_scalar(v)
    out: List[str] = []
    _yaml_block(v, 0, out)
    return "---\n" + "\n".join(out)


def table(rows: Sequence[Sequence[str]]) -> List[str]:
    """``printRows``: every column padded (and cut) to the longest cell of the table."""
    width = max((len(c) for r in rows for c in r), default=0)
    return ["  ".join(c[:width].ljust(width) for c in r) for r in rows]


def render(fmt: str, body: Any, columns: Optional[Sequence[str]] = None,
           value: Optional[Callable[[Any, str], Any]] = None) -> str:
    """``print(format, body, columnsForRaw, valueSupplier)``: ``body`` is the JSON text (or
    the decoded value) of the response."""
    data = json.loads(body) if isinstance(body, (str, bytes)) else body
    if fmt == "json":
        return jackson_json(data)
    if fmt == "yaml":
        return jackson_yaml(data)
    cols = list(columns or [])
    rows = [[c.upper() for c in cols]]
    for item in (data if isinstance(data, list) else [data]):
        row = []
        for c in cols:
            x = value(item, c) if value is not None else (item.get(c) if isinstance(item, dict) else None)
            row.append("" if x is None else (x if isinstance(x, str) else _raw_text(x)))
        rows.append(row)
    return "\n".join(table(rows))


def _raw_text(x: Any) -> str:
    """JsonNode.asText(): scalars as text, containers as empty text."""
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, float):
        return java_double(x)
    if isinstance(x, (dict, list)):
        return ""
    return str(x)
