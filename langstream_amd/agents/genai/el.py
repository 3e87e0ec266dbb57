"""Expression language for ``compute`` / ``when`` / ``fields`` / ``dispatch`` etc.

A Jakarta-EL/JSTL-compatible subset (parity: CMN/jstl/JstlEvaluator.java:30-305,
CMN/jstl/JstlFunctions.java:49-537, CMN/jstl/predicate/JstlPredicate.java):
literals (numbers, 'str', "str", true/false/null), property access ``a.b``,
``a['b']``, ``a[0]``, arithmetic ``+ - * / div % mod``, comparisons
(``== != < > <= >= eq ne lt gt le ge``), logic (``&& || ! and or not``), ``empty``,
ternary ``? :``, string concatenation ``+=``, EL 3.0 collection literals (``[a, b]`` list,
``{a, b}`` set, ``{k: v}`` map) and the ``fn:`` function library.
Expressions may be wrapped in ``${...}``.  Compiled ASTs are cached.
"""
from __future__ import annotations

import base64
import datetime as _dt
import functools
import json
import math
import random
import re
import time
import uuid
from decimal import Decimal
from typing import Any, Callable, Dict, List, Optional

from ...api import temporal as _temporal

# ---------------------------------------------------------------- lexer
_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<num>\d+\.\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?|\d+(?:[eE][+-]?\d+)?)
  | (?P<str>'(?:[^'\\]|\\.)*'|"(?:[^"\\]|\\.)*")
  | (?P<op>\+=|==|!=|<=|>=|&&|\|\||[-+*/%<>!?:.,()\[\]{}])
  | (?P<name>[A-Za-z_][A-Za-z0-9_]*)
""", re.VERBOSE)

_WORD_OPS = {"and": "&&", "or": "||", "not": "!", "eq": "==", "ne": "!=", "lt": "<", "gt": ">", "le": "<=",
             "ge": ">=", "div": "/", "mod": "%"}


def _unescape(s: str) -> str:
    body = s[1:-1]
    return re.sub(r"\\(.)", lambda m: {"n": "\n", "t": "\t", "r": "\r"}.get(m.group(1), m.group(1)), body)


def tokenize(src: str) -> List[tuple]:
    out = []
    pos = 0
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m:
            raise ValueError(f"Invalid expression at {pos}: {src!r}")
        pos = m.end()
        kind = m.lastgroup
        text = m.group(kind)
        if kind == "ws":
            continue
        if kind == "num":
            out.append(("num", float(text) if any(c in text for c in ".eE") else int(text)))
        elif kind == "str":
            out.append(("str", _unescape(text)))
        elif kind == "name":
            if text in _WORD_OPS:
                out.append(("op", _WORD_OPS[text]))
            elif text in ("true", "false"):
                out.append(("lit", text == "true"))
            elif text == "null":
                out.append(("lit", None))
            elif text == "empty":
                out.append(("op", "empty"))
            else:
                out.append(("name", text))
        else:
            out.append(("op", text))
    out.append(("eof", None))
    return out


# ---------------------------------------------------------------- parser (Pratt)
_BP = {"?": 1, "||": 2, "&&": 3, "==": 4, "!=": 4, "<": 5, ">": 5, "<=": 5, ">=": 5, "+": 6, "-": 6, "+=": 6,
       "*": 7, "/": 7, "%": 7}


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self):
        return self.t[self.i]

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, op):
        tok = self.next()
        if tok != ("op", op):
            raise ValueError(f"expected {op!r}, got {tok[1]!r}")

    def parse(self, rbp=0):
        left = self.nud(self.next())
        while True:
            tok = self.peek()
            if tok[0] != "op" or tok[1] not in _BP or _BP[tok[1]] <= rbp:
                break
            self.next()
            op = tok[1]
            if op == "?":
                a = self.parse(0)
                self.expect(":")
                b = self.parse(0)
                left = ("?", left, a, b)
            else:
                left = ("bin", op, left, self.parse(_BP[op]))
        return left

    def nud(self, tok):
        kind, v = tok
        if kind in ("num", "str", "lit"):
            return self.postfix(("lit", v))
        if kind == "op" and v == "(":
            e = self.parse(0)
            self.expect(")")
            return self.postfix(e)
        if kind == "op" and v == "[":
            # EL 3.0 collection construction: [a, b, ...] is a List
            return self.postfix(("list", self._items("]")))
        if kind == "op" and v == "{":
            # {a, b} is a Set, {k: v, ...} a Map
            if self.peek() == ("op", "}"):
                self.next()
                return self.postfix(("set", []))
            first = self.parse(0)
            if self.peek() == ("op", ":"):
                self.next()
                pairs = [(first, self.parse(0))]
                while self.peek() == ("op", ","):
                    self.next()
                    k = self.parse(0)
                    self.expect(":")
                    pairs.append((k, self.parse(0)))
                self.expect("}")
                return self.postfix(("map", pairs))
            items = [first]
            while self.peek() == ("op", ","):
                self.next()
                items.append(self.parse(0))
            self.expect("}")
            return self.postfix(("set", items))
        if kind == "op" and v == "!":
            return ("not", self.parse(8))
        if kind == "op" and v == "-":
            return ("neg", self.parse(8))
        if kind == "op" and v == "empty":
            return ("empty", self.parse(8))
        if kind == "name":
            # namespaced function fn:name(...)
            if self.peek() == ("op", ":") and self.t[self.i + 1][0] == "name" and self.t[self.i + 2] == ("op", "("):
                self.next()
                fname = self.next()[1]
                self.expect("(")
                args = []
                if self.peek() != ("op", ")"):
                    while True:
                        args.append(self.parse(0))
                        if self.peek() == ("op", ","):
                            self.next()
                            continue
                        break
                self.expect(")")
                return self.postfix(("call", v, fname, args))
            return self.postfix(("var", v))
        raise ValueError(f"unexpected token {v!r}")

    def _items(self, close):
        items = []
        if self.peek() != ("op", close):
            while True:
                items.append(self.parse(0))
                if self.peek() == ("op", ","):
                    self.next()
                    continue
                break
        self.expect(close)
        return items

    def postfix(self, e):
        while True:
            tok = self.peek()
            if tok == ("op", "."):
                self.next()
                name = self.next()
                if name[0] not in ("name", "lit"):
                    raise ValueError("expected property name after '.'")
                prop = name[1] if name[0] == "name" else str(name[1]).lower()
                e = ("get", e, ("lit", prop))
            elif tok == ("op", "["):
                self.next()
                idx = self.parse(0)
                self.expect("]")
                e = ("get", e, idx)
            else:
                return e


@functools.lru_cache(maxsize=4096)
def compile_expression(expr: str):
    s = expr.strip()
    if s.startswith("${") and s.endswith("}"):
        s = s[2:-1]
    p = _Parser(tokenize(s))
    ast = p.parse(0)
    if p.peek()[0] != "eof":
        raise ValueError(f"unexpected trailing input in expression {expr!r}")
    return ast


# ---------------------------------------------------------------- evaluation
def _num(v):
    if isinstance(v, bool):
        return int(v)
    if v is None:
        return 0
    if isinstance(v, (int, float, Decimal)):
        return v
    if isinstance(v, str):
        try:
            return int(v)
        except ValueError:
            return float(v)
    raise ValueError(f"cannot coerce {v!r} to a number")


def _is_empty(v) -> bool:
    return v is None or (isinstance(v, (str, list, dict, tuple, set)) and len(v) == 0)


def _truthy(v) -> bool:
    if isinstance(v, str):
        return v.strip().lower() == "true"
    return bool(v)


def _cmp_coerce(a, b):
    if isinstance(a, str) and isinstance(b, (int, float)) and not isinstance(b, bool):
        try:
            return _num(a), b
        except ValueError:
            return a, str(b)
    if isinstance(b, str) and isinstance(a, (int, float)) and not isinstance(a, bool):
        try:
            return a, _num(b)
        except ValueError:
            return str(a), b
    return a, b


def _get(obj, key):
    if obj is None:
        return None
    if isinstance(obj, dict):
        return obj.get(key)
    if isinstance(obj, (list, tuple)):
        try:
            return obj[int(key)]
        except (IndexError, ValueError, TypeError):
            return None
    if isinstance(obj, str) and isinstance(key, str):
        # JSON-string values are transparently parsed (recordToMutableRecord behaviour)
        try:
            parsed = json.loads(obj)
            if isinstance(parsed, dict):
                return parsed.get(key)
        except ValueError:
            pass
        # String's bean properties through the EL's BeanELResolver: 'x'.bytes (getBytes,
        # UTF-8), 'x'.empty (isEmpty), 'x'.blank (isBlank)
        if key == "bytes":
            return obj.encode("utf-8")
        if key == "empty":
            return obj == ""
        if key == "blank":
            return obj.strip() == ""
        return None
    return getattr(obj, str(key), None)


def evaluate(ast, ctx: Dict[str, Any]) -> Any:
    t = ast[0]
    if t == "lit":
        return ast[1]
    if t == "var":
        return ctx.get(ast[1])
    if t == "get":
        return _get(evaluate(ast[1], ctx), evaluate(ast[2], ctx))
    if t == "list":
        return [evaluate(x, ctx) for x in ast[1]]
    if t == "set":
        out = []
        for x in ast[1]:
            v = evaluate(x, ctx)
            if v not in out:
                out.append(v)
        return out
    if t == "map":
        return {evaluate(k, ctx): evaluate(v, ctx) for k, v in ast[1]}
    if t == "not":
        return not _truthy(evaluate(ast[1], ctx))
    if t == "neg":
        return -_num(evaluate(ast[1], ctx))
    if t == "empty":
        return _is_empty(evaluate(ast[1], ctx))
    if t == "?":
        return evaluate(ast[2], ctx) if _truthy(evaluate(ast[1], ctx)) else evaluate(ast[3], ctx)
    if t == "call":
        fn = FUNCTIONS.get(ast[2])
        if fn is None:
            raise ValueError(f"Unknown function {ast[1]}:{ast[2]}")
        if ast[2] == "filter":
            return _fn_filter(evaluate(ast[3][0], ctx), evaluate(ast[3][1], ctx), ctx)
        return fn(*[evaluate(a, ctx) for a in ast[3]])
    if t == "bin":
        op = ast[1]
        if op == "&&":
            return _truthy(evaluate(ast[2], ctx)) and _truthy(evaluate(ast[3], ctx))
        if op == "||":
            return _truthy(evaluate(ast[2], ctx)) or _truthy(evaluate(ast[3], ctx))
        a, b = evaluate(ast[2], ctx), evaluate(ast[3], ctx)
        if op == "+=":
            return _fn_tostring(a) + _fn_tostring(b)
        if op == "==":
            a, b = _cmp_coerce(a, b)
            return a == b
        if op == "!=":
            a, b = _cmp_coerce(a, b)
            return a != b
        if op in ("<", ">", "<=", ">="):
            a, b = _cmp_coerce(a, b)
            if a is None or b is None:
                return False
            return {"<": a < b, ">": a > b, "<=": a <= b, ">=": a >= b}[op]
        if op == "+":
            return _num(a) + _num(b)
        if op == "-":
            return _num(a) - _num(b)
        if op == "*":
            return _num(a) * _num(b)
        if op == "/":
            return _num(a) / _num(b)
        if op == "%":
            return _num(a) % _num(b)
    raise ValueError(f"bad ast node {t}")


def eval_expression(expr: str, ctx: Dict[str, Any]) -> Any:
    return evaluate(compile_expression(expr), ctx)


def eval_predicate(expr: Optional[str], ctx: Dict[str, Any]) -> bool:
    if expr is None or (isinstance(expr, str) and not expr.strip()):
        return True
    return _truthy(eval_expression(expr, ctx))


# ---------------------------------------------------------------- fn: library
def _fn_tostring(v) -> str:
    """JstlFunctions.toString: String.valueOf semantics -- a map prints as Java's
    ``{k=v, ...}``, a list as ``[a, b]``, doubles as Double.toString."""
    if v is None:
        return ""
    if isinstance(v, bytes):
        return v.decode("utf-8", errors="replace")
    return _java_str(v)


def _java_str(v) -> str:
    if v is None:
        return "null"
    if isinstance(v, _TEMPORAL_TYPES):
        return _temporal.to_java_string(v)
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return _temporal.java_float_str(v) if isinstance(v, _temporal.Float32) else _temporal.java_double_str(v)
    if isinstance(v, dict):
        return "{" + ", ".join(f"{_java_str(k)}={_java_str(x)}" for k, x in v.items()) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ", ".join(_java_str(x) for x in v) + "]"
    return str(v)


def _fn_to_json(v):
    # Jackson's default writer: compact separators, non-ASCII as is (JstlFunctions.toJson)
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False, default=_json_default)


def _json_default(o):
    if isinstance(o, Decimal):
        return float(o)
    if isinstance(o, (bytes, bytearray)):
        import base64
        return base64.b64encode(bytes(o)).decode()
    raise TypeError(f"{type(o).__name__} is not JSON serializable")


def _fn_from_json(v):
    if v is None:
        return None
    if isinstance(v, bytes):
        v = v.decode()
    if isinstance(v, str) and not v.strip():
        return None                     # JstlFunctions.fromJson: empty text -> null
    return json.loads(v) if isinstance(v, str) else v


def _to_big_integer(v) -> int:
    """BigInteger conversion of JstlTypeConverter: byte[] two's complement, text, numbers."""
    if isinstance(v, (bytes, bytearray)):
        return int.from_bytes(bytes(v), "big", signed=True)
    if isinstance(v, str):
        return int(v.strip())
    return int(v)


def _fn_to_big_decimal(v, scale=None):
    """``toBigDecimal(value, scale)`` = new BigDecimal(BigInteger(value), scale) (exact);
    ``toBigDecimal(value)`` = BigDecimal.valueOf(double): the value goes through a double."""
    if v is None:
        return None
    if scale is None:
        return Decimal(repr(_to_double(v)))
    import decimal
    return Decimal(_to_big_integer(v)).scaleb(-int(_fn_tostring(scale)), context=decimal.Context(prec=1000))


def _fn_length(v):
    if v is None:
        return 0
    return len(v) if isinstance(v, (str, list, dict, tuple)) else len(_fn_tostring(v))


def _fn_to_list_of_float(v):
    if v is None:
        return None
    if isinstance(v, str):
        v = json.loads(v)
    return [float(x) for x in v]


def _to_int(v):
    if v is None:
        return None
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, str):
        return int(float(v)) if v.strip() else None
    return int(v)


def _to_double(v):
    if v is None:
        return None
    return float(v)


def _fn_split(v, sep):
    if v is None:
        return None
    s = _fn_tostring(v)
    if s == "":
        return []
    return re.split(_fn_tostring(sep), s)


def _fn_concat(*args):
    return "".join(_fn_tostring(a) for a in args)


def _fn_replace(v, regex, repl):
    if v is None:
        return None
    if regex is None or repl is None:      # JstlFunctions.replace: nothing to replace with
        return _fn_tostring(v)
    return re.sub(_fn_tostring(regex), _fn_tostring(repl).replace("$", "\\"), _fn_tostring(v))


def _fn_contains(v, s):
    if v is None or s is None:
        return False
    if isinstance(v, (list, tuple, dict)):
        return s in v
    return _fn_tostring(s) in _fn_tostring(v)


def _fn_coalesce(v, d):
    return d if v is None else v


def _fn_unpack(v, fields):
    if v is None:
        return None
    vals = ([] if v == "" else v.split(",")) if isinstance(v, str) else list(v)
    heads = _fn_tostring(fields).split(",")
    return {h: (vals[i] if i < len(vals) else None) for i, h in enumerate(heads)}


def _fn_list_add(lst, item):
    return list(lst or []) + [item]


def _fn_add_all(a, b):
    return list(a or []) + list(b or [])


def _fn_list_of(*args):
    return list(args)


def _fn_map_of(*args):
    if len(args) % 2:
        raise ValueError("fn:mapOf needs an even number of arguments")
    return {_fn_tostring(args[i]): args[i + 1] for i in range(0, len(args), 2)}


def _fn_map_put(m, k, v):
    d = dict(m or {})
    d[_fn_tostring(k)] = v
    return d


def _fn_map_remove(m, k):
    d = dict(m or {})
    d.pop(_fn_tostring(k), None)
    return d


def _fn_map_to_list_of_structs(m, fields):
    if m is None:
        raise ValueError("listOf doesn't allow a null value")
    if isinstance(m, str):
        m = json.loads(m)
    return [{f: m.get(f) for f in fields.split(",")}]


def _fn_list_to_list_of_structs(lst, field):
    if lst is None:
        raise ValueError("listOf doesn't allow a null value")
    return [{field: x} for x in lst]


_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
_TEMPORAL_TYPES = (_temporal.JDate, _temporal.Timestamp, _temporal.Time, _temporal.Instant, _temporal.LocalTime,
                   _temporal.LocalDateTime, _temporal.OffsetDateTime)


def _dt_millis(d: "_dt.datetime") -> int:
    # exact integer arithmetic (d.timestamp() * 1000 rounds .005 s down to 4 ms)
    if d.tzinfo is None:
        d = d.replace(tzinfo=_dt.timezone.utc)
    return (d - _EPOCH) // _dt.timedelta(milliseconds=1)


def _to_millis(v) -> int:
    """Instant conversion of JstlTypeConverter: epoch millis, ISO-8601 text (an offset is
    honoured, none means UTC), datetimes; byte / other types are refused."""
    if isinstance(v, bool):
        raise ValueError(f"Cannot convert [{v}] to an Instant")
    if isinstance(v, (int, float)):
        return int(v)
    if isinstance(v, _dt.datetime):
        return _dt_millis(v)
    if isinstance(v, (_temporal.JDate, _temporal.Timestamp, _temporal.Instant, _temporal.LocalDateTime,
                      _temporal.OffsetDateTime)) or (isinstance(v, _dt.date) and not isinstance(v, _dt.datetime)):
        return _temporal.coerce(v, "instant").to_epoch_milli()   # the cast step's date-time values
    if isinstance(v, (bytes, bytearray)):
        v = v.decode()
    if isinstance(v, str):
        return _dt_millis(_dt.datetime.fromisoformat(v.strip().replace("Z", "+00:00")))
    raise ValueError(f"Cannot convert [{v}] of type [{type(v).__name__}] to an Instant")


_UNIT_MS = {"days": 86400000, "hours": 3600000, "minutes": 60000, "seconds": 1000, "millis": 1}


def _delta_long(d) -> int:
    """The delta's long value (JstlTypeConverter): numbers, numeric text, and a
    LocalTime as its millisecond of day."""
    if isinstance(d, _dt.time):
        return ((d.hour * 60 + d.minute) * 60 + d.second) * 1000 + d.microsecond // 1000
    if isinstance(d, (bytes, bytearray)):
        d = d.decode()
    if isinstance(d, str):
        return int(float(d)) if not d.strip().lstrip("-").isdigit() else int(d)
    return int(d)


def _fn_timestamp_add(v, delta, unit):
    if v is None or unit is None:
        raise ValueError("timestampAdd requires input and unit")
    unit = _fn_tostring(unit)
    ms = _to_millis(v)
    d = _delta_long(delta)
    if unit in ("years", "months"):
        import calendar
        t = _EPOCH + _dt.timedelta(milliseconds=ms)
        months = d * (12 if unit == "years" else 1)
        y, mth = divmod(t.month - 1 + months, 12)
        # Instant.atZone(UTC).plusMonths: an out-of-range day clamps to the month's last day
        day = min(t.day, calendar.monthrange(t.year + y, mth + 1)[1])
        t = t.replace(year=t.year + y, month=mth + 1, day=day)
        return _dt_millis(t)
    if unit == "nanos":
        return ms + d // 1_000_000
    if unit not in _UNIT_MS:
        raise ValueError(f"Invalid unit: {unit}. Should be one of [years, months, days, hours, minutes, seconds, "
                         f"millis]")
    return ms + d * _UNIT_MS[unit]


def _fn_filter(lst, expr, ctx):
    if lst is None:
        return None
    out = []
    for o in lst:
        if o is None:
            continue
        c = dict(ctx)
        c["record"] = o
        if eval_predicate(expr, c):
            out.append(o)
    return out


FUNCTIONS: Dict[str, Callable] = {
    "length": _fn_length, "toJson": _fn_to_json, "fromJson": _fn_from_json, "toListOfFloat": _fn_to_list_of_float,
    "uppercase": lambda v: None if v is None else _fn_tostring(v).upper(),
    "lowercase": lambda v: None if v is None else _fn_tostring(v).lower(),
    "contains": _fn_contains, "trim": lambda v: None if v is None else _fn_tostring(v).strip(),
    "concat": _fn_concat, "concat3": _fn_concat, "coalesce": _fn_coalesce, "replace": _fn_replace,
    "str": _fn_tostring, "toString": _fn_tostring, "toDouble": _to_double, "toInt": _to_int, "toLong": _to_int,
    "toBigDecimal": _fn_to_big_decimal,
    "decimalFromUnscaled": lambda v, scale: Decimal(int(v)).scaleb(-int(scale)),
    "decimalFromNumber": lambda v: Decimal(str(v)),
    "split": _fn_split, "unpack": _fn_unpack, "listOf": _fn_list_of, "emptyList": lambda: [],
    "listAdd": _fn_list_add, "addAll": _fn_add_all, "mapOf": _fn_map_of, "emptyMap": lambda: {},
    "mapPut": _fn_map_put, "mapRemove": _fn_map_remove, "mapToListOfStructs": _fn_map_to_list_of_structs,
    "listToListOfStructs": _fn_list_to_list_of_structs, "filter": _fn_filter,
    "now": lambda: int(time.time() * 1000), "uuid": lambda: str(uuid.uuid4()),
    "random": lambda mx: random.randrange(int(mx)),
    "timestampAdd": _fn_timestamp_add, "dateadd": _fn_timestamp_add,
    "toSQLTimestamp": lambda v: _dt.datetime.fromtimestamp(_to_millis(v) / 1000, tz=_dt.timezone.utc).isoformat(),
}
