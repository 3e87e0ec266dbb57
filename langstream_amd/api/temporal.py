"""Java value types of the toolkit's type converter, and the converter itself.

The reference's records carry Java objects, and its ``cast`` step and expression
language convert between them with ``JstlTypeConverter.coerceToType``
(langstream-agents-commons/.../jstl/JstlTypeConverter.java:48-521): numbers of four
widths, strings, byte[] in the Pulsar schema encodings (``BytesConverter``), and seven
date / time classes with nanosecond precision.  Python's ``datetime`` stops at
microseconds and has no counterpart of ``java.sql.Time`` or of a UTC ``Instant``, so the
temporal classes are modelled here:

=================  ============================================  ====================
Java               here                                           bytes (big-endian)
=================  ============================================  ====================
java.util.Date     ``JDate(millis)``                              int64 millis
java.sql.Timestamp ``Timestamp(seconds, nanos)``                  int64 millis
java.sql.Time      ``Time(millis)``                               int64 millis
LocalDate          ``datetime.date``                              int64 epoch day
LocalTime          ``LocalTime(nano_of_day)``                     int64 nano of day
LocalDateTime      ``LocalDateTime(date, LocalTime)``             epoch day + nano of day
Instant            ``Instant(seconds, nanos)``                    int64 s + int32 nanos
OffsetDateTime     ``OffsetDateTime(LocalDateTime, offset_s)``    as its Instant
=================  ============================================  ====================

Numbers follow api/types.py: a plain ``int`` is a Long, ``Int32`` an Integer, ``Int16`` a
Short, ``Int8`` a Byte; a plain ``float`` a Double, ``Float32`` a Float.  The default time
zone is UTC (the reference's tests pin it so).  Python ``datetime`` values are accepted
as inputs: naive -> LocalDateTime, aware -> OffsetDateTime, ``time`` -> LocalTime.

``coerce(value, target)`` mirrors ``coerceToType`` branch by branch (the order of the
instanceof checks matters: a Long is epoch MILLIS for an Instant but epoch DAYS for a
LocalDate); the test vectors are JstlTypeConverterTest.java's
(tests/test_ref_vectors_types.py)."""
from __future__ import annotations

import datetime as _dt
import math
import re
import struct
from decimal import Decimal
from typing import Any, Optional

from .types import Float32, Int8, Int16, Int32

_NANOS = 1_000_000_000
_DAY_NANOS = 86_400 * _NANOS
_EPOCH_DATE = _dt.date(1970, 1, 1)


class ConversionError(ValueError):
    pass


def _frac_groups(nanos: int) -> str:
    """Instant / LocalTime ``toString``: 0, 3, 6 or 9 fraction digits."""
    if nanos == 0:
        return ""
    if nanos % 1_000_000 == 0:
        return ".%03d" % (nanos // 1_000_000)
    if nanos % 1_000 == 0:
        return ".%06d" % (nanos // 1_000)
    return ".%09d" % nanos


def _frac_min(nanos: int) -> str:
    """``DateTimeFormatter.ISO_LOCAL_TIME``: as few digits as needed."""
    if nanos == 0:
        return ""
    return "." + ("%09d" % nanos).rstrip("0")


def _floordiv(a: int, b: int):
    return a // b, a % b


class LocalTime:
    __slots__ = ("nano_of_day",)

    def __init__(self, nano_of_day: int):
        if not 0 <= nano_of_day < _DAY_NANOS:
            raise ConversionError(f"nano of day out of range: {nano_of_day}")
        self.nano_of_day = int(nano_of_day)

    @classmethod
    def of(cls, h: int, m: int, s: int = 0, n: int = 0) -> "LocalTime":
        return cls(((h * 60 + m) * 60 + s) * _NANOS + n)

    @property
    def hms(self):
        sec, n = divmod(self.nano_of_day, _NANOS)
        h, rem = divmod(sec, 3600)
        m, s = divmod(rem, 60)
        return h, m, s, n

    def __eq__(self, o):
        return isinstance(o, LocalTime) and o.nano_of_day == self.nano_of_day

    def __hash__(self):
        return hash(("LocalTime", self.nano_of_day))

    def __str__(self):
        h, m, s, n = self.hms
        out = "%02d:%02d" % (h, m)
        if s or n:
            out += ":%02d" % s + _frac_groups(n)
        return out

    def iso(self) -> str:   # ISO_LOCAL_TIME
        h, m, s, n = self.hms
        return "%02d:%02d:%02d" % (h, m, s) + _frac_min(n)

    __repr__ = lambda self: f"LocalTime({self})"  # noqa: E731


class LocalDateTime:
    __slots__ = ("date", "time")

    def __init__(self, date: _dt.date, time: LocalTime):
        self.date, self.time = date, time

    def __eq__(self, o):
        return isinstance(o, LocalDateTime) and (o.date, o.time) == (self.date, self.time)

    def __hash__(self):
        return hash(("LocalDateTime", self.date, self.time))

    def __str__(self):
        return f"{self.date.isoformat()}T{self.time}"

    def epoch_second_utc(self):
        return (self.date - _EPOCH_DATE).days * 86_400 + self.time.nano_of_day // _NANOS

    __repr__ = lambda self: f"LocalDateTime({self})"  # noqa: E731


class Instant:
    __slots__ = ("seconds", "nanos")

    def __init__(self, seconds: int, nanos: int = 0):
        extra, n = _floordiv(int(nanos), _NANOS)
        self.seconds, self.nanos = int(seconds) + extra, n

    @classmethod
    def of_epoch_milli(cls, ms: int) -> "Instant":
        s, r = _floordiv(int(ms), 1000)
        return cls(s, r * 1_000_000)

    def to_epoch_milli(self) -> int:
        return self.seconds * 1000 + self.nanos // 1_000_000

    def at_utc(self) -> LocalDateTime:
        d, sod = _floordiv(self.seconds, 86_400)
        return LocalDateTime(_EPOCH_DATE + _dt.timedelta(days=d), LocalTime(sod * _NANOS + self.nanos))

    def __eq__(self, o):
        return type(o) is Instant and (o.seconds, o.nanos) == (self.seconds, self.nanos)

    def __hash__(self):
        return hash(("Instant", self.seconds, self.nanos))

    def __str__(self):   # ISO_INSTANT
        ldt = self.at_utc()
        h, m, s, n = ldt.time.hms
        return "%sT%02d:%02d:%02d%sZ" % (ldt.date.isoformat(), h, m, s, _frac_groups(n))

    __repr__ = lambda self: f"Instant({self})"  # noqa: E731


class OffsetDateTime:
    __slots__ = ("local", "offset")

    def __init__(self, local: LocalDateTime, offset_seconds: int = 0):
        self.local, self.offset = local, int(offset_seconds)

    def to_instant(self) -> Instant:
        return Instant(self.local.epoch_second_utc() - self.offset, self.local.time.nano_of_day % _NANOS)

    def __eq__(self, o):
        return isinstance(o, OffsetDateTime) and (o.local, o.offset) == (self.local, self.offset)

    def __hash__(self):
        return hash(("OffsetDateTime", self.local, self.offset))

    def __str__(self):
        if self.offset == 0:
            z = "Z"
        else:
            sign = "+" if self.offset > 0 else "-"
            h, rem = divmod(abs(self.offset), 3600)
            m, s = divmod(rem, 60)
            z = "%s%02d:%02d" % (sign, h, m) + (":%02d" % s if s else "")
        return f"{self.local}{z}"

    __repr__ = lambda self: f"OffsetDateTime({self})"  # noqa: E731


class JDate:
    """java.util.Date: epoch millis."""
    __slots__ = ("millis",)

    def __init__(self, millis: int):
        self.millis = int(millis)

    def get_time(self) -> int:
        return self.millis

    def to_instant(self) -> Instant:
        return Instant.of_epoch_milli(self.millis)

    def __eq__(self, o):
        return type(o) is JDate and o.millis == self.millis

    def __hash__(self):
        return hash(("Date", self.millis))

    def __str__(self):
        return str(self.to_instant())

    __repr__ = lambda self: f"Date({self})"  # noqa: E731


class Timestamp:
    """java.sql.Timestamp: whole seconds + nanos (``getTime()`` = the millis of both)."""
    __slots__ = ("seconds", "nanos")

    def __init__(self, seconds: int, nanos: int = 0):
        i = Instant(seconds, nanos)
        self.seconds, self.nanos = i.seconds, i.nanos

    @classmethod
    def of_millis(cls, ms: int) -> "Timestamp":
        i = Instant.of_epoch_milli(ms)
        return cls(i.seconds, i.nanos)

    def get_time(self) -> int:
        return self.seconds * 1000 + self.nanos // 1_000_000

    def to_instant(self) -> Instant:
        return Instant(self.seconds, self.nanos)

    def __eq__(self, o):
        return type(o) is Timestamp and (o.seconds, o.nanos) == (self.seconds, self.nanos)

    def __hash__(self):
        return hash(("Timestamp", self.seconds, self.nanos))

    def __str__(self):
        return str(self.to_instant())

    __repr__ = lambda self: f"Timestamp({self})"  # noqa: E731


class Time:
    """java.sql.Time: epoch millis; compared (and printed) by its time of day to the
    second, as ``Time.toLocalTime()`` does."""
    __slots__ = ("millis",)

    def __init__(self, millis: int):
        self.millis = int(millis)

    @classmethod
    def value_of(cls, lt: LocalTime) -> "Time":   # Time.valueOf(LocalTime): h, m, s only
        h, m, s, _ = lt.hms
        return cls(((h * 60 + m) * 60 + s) * 1000)

    def get_time(self) -> int:
        return self.millis

    def to_local_time(self) -> LocalTime:
        sod = (self.millis // 1000) % 86_400
        return LocalTime(sod * _NANOS)

    def __eq__(self, o):
        return type(o) is Time and o.to_local_time() == self.to_local_time()

    def __hash__(self):
        return hash(("Time", self.to_local_time().nano_of_day))

    def __str__(self):
        return self.to_local_time().iso()

    __repr__ = lambda self: f"Time({self})"  # noqa: E731


# ------------------------------------------------------------------ classification
def _is_long(v) -> bool:
    return type(v) is int

def _is_double(v) -> bool:
    return type(v) is float


def _is_number(v) -> bool:
    return isinstance(v, (int, float, Decimal)) and not isinstance(v, bool)


def _is_date(v) -> bool:          # java.util.Date and its subclasses
    return isinstance(v, (JDate, Timestamp, Time))


def _is_temporal(v) -> bool:      # java.time.temporal.TemporalAccessor
    return isinstance(v, (LocalTime, LocalDateTime, Instant, OffsetDateTime)) or _is_local_date(v)


def _is_local_date(v) -> bool:
    return isinstance(v, _dt.date) and not isinstance(v, _dt.datetime)


def _from_python(v):
    """Python datetime values as their Java counterparts."""
    if isinstance(v, _dt.datetime):
        lt = LocalTime.of(v.hour, v.minute, v.second, v.microsecond * 1000)
        ldt = LocalDateTime(v.date(), lt)
        if v.tzinfo is None:
            return ldt
        return OffsetDateTime(ldt, int(v.utcoffset().total_seconds()))
    if isinstance(v, _dt.time):
        return LocalTime.of(v.hour, v.minute, v.second, v.microsecond * 1000)
    return v


# ------------------------------------------------------------------ parsing
_TIME_RE = r"(\d{2}):(\d{2})(?::(\d{2})(?:\.(\d{1,9}))?)?"
_LT = re.compile(_TIME_RE + r"$")
_LD = re.compile(r"([+-]?\d{4,})-(\d{2})-(\d{2})$")
_LDT = re.compile(r"([+-]?\d{4,})-(\d{2})-(\d{2})T" + _TIME_RE + r"$")
_ODT = re.compile(r"([+-]?\d{4,})-(\d{2})-(\d{2})T" + _TIME_RE + r"(Z|[+-]\d{2}:\d{2}(?::\d{2})?)(?:\[[^\]]+\])?$")


def _lt_of(h, m, s, f) -> LocalTime:
    n = int((f or "").ljust(9, "0") or 0)
    return LocalTime.of(int(h), int(m), int(s or 0), n)


def parse_local_time(s: str) -> LocalTime:
    m = _LT.match(s.strip())
    if not m:
        raise ConversionError(f"Text '{s}' could not be parsed as a LocalTime")
    return _lt_of(*m.groups())


def parse_local_date(s: str) -> _dt.date:
    m = _LD.match(s.strip())
    if not m:
        raise ConversionError(f"Text '{s}' could not be parsed as a LocalDate")
    return _dt.date(int(m.group(1)), int(m.group(2)), int(m.group(3)))


def parse_local_date_time(s: str) -> LocalDateTime:
    m = _LDT.match(s.strip())
    if not m:
        raise ConversionError(f"Text '{s}' could not be parsed as a LocalDateTime")
    g = m.groups()
    return LocalDateTime(_dt.date(int(g[0]), int(g[1]), int(g[2])), _lt_of(*g[3:7]))


def _parse_offset_date_time(s: str) -> OffsetDateTime:
    s = s.strip()
    if len(s) == 10:
        return OffsetDateTime(LocalDateTime(parse_local_date(s), LocalTime(0)), 0)
    m = _ODT.match(s)
    if not m:
        raise ConversionError(f"Text '{s}' could not be parsed as an OffsetDateTime")
    g = m.groups()
    ldt = LocalDateTime(_dt.date(int(g[0]), int(g[1]), int(g[2])), _lt_of(*g[3:7]))
    z = g[7]
    off = 0
    if z != "Z":
        sign = -1 if z[0] == "-" else 1
        parts = [int(p) for p in z[1:].split(":")]
        off = sign * (parts[0] * 3600 + parts[1] * 60 + (parts[2] if len(parts) > 2 else 0))
    return OffsetDateTime(ldt, off)


# ------------------------------------------------------------------ bytes (Pulsar encodings)
def encode_bytes(v) -> bytes:
    """``BytesConverter`` of the value's own type (JstlTypeConverter.coerceToBytes)."""
    v = _from_python(v)
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if isinstance(v, OffsetDateTime):
        return encode_bytes(v.to_instant())
    if isinstance(v, str):
        return v.encode("utf-8")
    if isinstance(v, bool):
        return b"\x01" if v else b"\x00"
    if isinstance(v, Int8):
        return struct.pack(">b", v)
    if isinstance(v, Int16):
        return struct.pack(">h", v)
    if isinstance(v, Int32):
        return struct.pack(">i", v)
    if _is_long(v):
        return struct.pack(">q", v)
    if isinstance(v, Float32):
        return struct.pack(">f", v)
    if _is_double(v):
        return struct.pack(">d", v)
    if isinstance(v, (JDate, Timestamp, Time)):
        return struct.pack(">q", v.get_time())
    if _is_local_date(v):
        return struct.pack(">q", (v - _EPOCH_DATE).days)
    if isinstance(v, LocalTime):
        return struct.pack(">q", v.nano_of_day)
    if isinstance(v, LocalDateTime):
        return struct.pack(">qq", (v.date - _EPOCH_DATE).days, v.time.nano_of_day)
    if isinstance(v, Instant):
        return struct.pack(">qi", v.seconds, v.nanos)
    raise ConversionError(f"Cannot convert type {type(v).__name__} to byte[]")


def _dec(fmt: str, b: bytes, what: str):
    if len(b) != struct.calcsize(fmt):
        raise ConversionError(f"Size of data received by {what}BytesConverter is not {struct.calcsize(fmt)}")
    return struct.unpack(fmt, b)


def decode_bytes(b: bytes, target: str):
    t = target
    if t == "string":
        return b.decode("utf-8")
    if t == "boolean":
        return _dec(">b", b, "Boolean")[0] != 0
    if t == "int8":
        return Int8(_dec(">b", b, "Byte")[0])
    if t == "int16":
        return Int16(_dec(">h", b, "Short")[0])
    if t == "int32":
        return Int32(_dec(">i", b, "Integer")[0])
    if t == "int64":
        return _dec(">q", b, "Long")[0]
    if t == "float":
        return Float32(_dec(">f", b, "Float")[0])
    if t == "double":
        return _dec(">d", b, "Double")[0]
    if t == "date":
        return JDate(_dec(">q", b, "Date")[0])
    if t == "timestamp":
        return Timestamp.of_millis(_dec(">q", b, "Timestamp")[0])
    if t == "time":
        return Time(_dec(">q", b, "Time")[0])
    if t == "local_time":
        return LocalTime(_dec(">q", b, "LocalTime")[0])
    if t == "local_date":
        return _EPOCH_DATE + _dt.timedelta(days=_dec(">q", b, "LocalDate")[0])
    if t == "local_date_time":
        d, n = _dec(">qq", b, "LocalDateTime")
        return LocalDateTime(_EPOCH_DATE + _dt.timedelta(days=d), LocalTime(n))
    if t == "instant":
        s, n = _dec(">qi", b, "Instant")
        return Instant(s, n)
    raise ConversionError(f"no bytes decoding to {target}")


# ------------------------------------------------------------------ numbers (ELSupport)
def _el_number(v) -> float:
    """ELSupport.coerceToNumber(value, Double.class)."""
    if isinstance(v, bool):
        raise ConversionError(f"Cannot convert {v} of type Boolean to Double")
    if isinstance(v, (int, float, Decimal)):
        return float(v)
    if isinstance(v, str):
        try:
            return float(v.strip())
        except ValueError as e:
            raise ConversionError(f"Cannot convert {v!r} to Double") from e
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Double")


def _d2l(d: float, bits: int) -> int:
    """Java (long) / (int) of a double: truncation, NaN -> 0, saturation."""
    if math.isnan(d):
        return 0
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    if math.isinf(d):
        return hi if d > 0 else lo
    return max(lo, min(hi, int(d)))


def _wrap(x: int, bits: int) -> int:
    x &= (1 << bits) - 1
    return x - (1 << bits) if x >> (bits - 1) else x


def _instant_of_double(d: float) -> Instant:
    seconds = _d2l(d / 1000, 64)
    nanos = math.floor((d - seconds * 1000) * 1_000_000 + 0.5)   # Math.round
    return Instant(seconds, nanos)


# ------------------------------------------------------------------ java toString
def java_double_str(d: float) -> str:
    """Double.toString: plain in [1e-3, 1e7), else d.dddE[-]n; shortest digits."""
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0:
        return "-0.0" if math.copysign(1, d) < 0 else "0.0"
    r = repr(float(d))
    return _java_float_fmt(r, abs(d))


def java_float_str(f: float) -> str:
    """Float.toString of a float32 value: the shortest digits that round-trip float32."""
    import numpy as np
    if math.isnan(f) or math.isinf(f) or f == 0:
        return java_double_str(f)
    r = np.format_float_positional(np.float32(f), unique=True, trim="-") if 1e-3 <= abs(f) < 1e7 else \
        np.format_float_scientific(np.float32(f), unique=True, trim="-")
    return _java_float_fmt(r, abs(f))


def _java_float_fmt(r: str, a: float) -> str:
    sign = "-" if r.startswith("-") else ""
    r = r.lstrip("-")
    if "e" in r or "E" in r:
        mant, exp = re.split("[eE]", r)
        exp = int(exp)
    else:
        mant, exp = r, 0
    digits = mant.replace(".", "")
    point = (mant.index(".") if "." in mant else len(mant)) + exp
    stripped = digits.lstrip("0")
    point -= len(digits) - len(stripped)
    digits = stripped.rstrip("0") or "0"
    if 1e-3 <= a < 1e7:
        if point <= 0:
            s = "0." + "0" * (-point) + digits
        elif point >= len(digits):
            s = digits + "0" * (point - len(digits)) + ".0"
        else:
            s = digits[:point] + "." + digits[point:]
        return sign + s
    e = point - 1
    frac = digits[1:] or "0"
    return f"{sign}{digits[0]}.{frac}E{e}"


def to_java_string(v) -> str:
    """JstlTypeConverter.coerceToString."""
    v = _from_python(v)
    if isinstance(v, Time):
        return v.to_local_time().iso()
    if isinstance(v, (JDate, Timestamp)):
        return str(v.to_instant())
    if isinstance(v, (bytes, bytearray)):
        return bytes(v).decode("utf-8")
    if isinstance(v, str):
        return v
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, Float32):
        return java_float_str(v)
    if isinstance(v, float):
        return java_double_str(v)
    if _is_local_date(v):
        return v.isoformat()
    return str(v)


# ------------------------------------------------------------------ temporal coercions
def _to_instant(v) -> Instant:
    if isinstance(v, Instant):
        return v
    if isinstance(v, (JDate, Timestamp)):
        return v.to_instant()
    if _is_long(v):
        return Instant.of_epoch_milli(v)
    if _is_double(v):
        return _instant_of_double(v)
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "instant")
    if _is_temporal(v) or isinstance(v, str):
        return _to_offset_date_time(v).to_instant()
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Instant")


def _to_offset_date_time(v) -> OffsetDateTime:
    if isinstance(v, OffsetDateTime):
        return v
    if _is_local_date(v):
        return OffsetDateTime(LocalDateTime(v, LocalTime(0)), 0)
    if isinstance(v, LocalDateTime):
        return OffsetDateTime(v, 0)
    if isinstance(v, Instant):
        return OffsetDateTime(v.at_utc(), 0)
    if isinstance(v, str):
        return _parse_offset_date_time(v)
    if _is_number(v) or _is_date(v) or isinstance(v, (bytes, bytearray)):
        return OffsetDateTime(_to_instant(v).at_utc(), 0)
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to OffsetDateTime")


def _to_date(v) -> JDate:
    if isinstance(v, Timestamp):
        return JDate(v.get_time())
    if isinstance(v, JDate):
        return v
    if _is_long(v) or _is_double(v):
        return JDate(_d2l(v, 64) if _is_double(v) else v)
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "date")
    if _is_temporal(v) or isinstance(v, str):
        return JDate(_to_instant(v).to_epoch_milli())
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Date")


def _to_timestamp(v) -> Timestamp:
    if isinstance(v, Timestamp):
        return v
    if isinstance(v, JDate):
        return Timestamp.of_millis(v.millis)
    if _is_long(v) or _is_double(v):
        return Timestamp.of_millis(_d2l(v, 64) if _is_double(v) else v)
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "timestamp")
    if _is_temporal(v) or isinstance(v, str):
        i = _to_instant(v)
        return Timestamp(i.seconds, i.nanos)
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Timestamp")


def _to_time(v) -> Time:
    if isinstance(v, Time):
        return v
    if _is_long(v) or _is_double(v):
        return Time(_d2l(v, 64) if _is_double(v) else v)
    if isinstance(v, LocalTime):
        return Time.value_of(v)
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "time")
    if isinstance(v, str):
        return Time.value_of(parse_local_time(v))
    if _is_temporal(v) or _is_date(v):
        return Time(_to_instant(v).to_epoch_milli())
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Time")


def _to_local_time(v) -> LocalTime:
    if isinstance(v, LocalTime):
        return v
    if isinstance(v, Time):
        return v.to_local_time()
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "local_time")
    if isinstance(v, str):
        return parse_local_time(v)
    if _is_temporal(v) or _is_number(v) or _is_date(v):
        return _to_instant(v).at_utc().time
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to LocalTime")


def _to_local_date(v) -> _dt.date:
    if _is_local_date(v):
        return v
    if isinstance(v, LocalDateTime):
        return v.date
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "local_date")
    if isinstance(v, str):
        return parse_local_date(v)
    if _is_number(v):
        return _EPOCH_DATE + _dt.timedelta(days=_d2l(float(v), 64) if not isinstance(v, int) else int(v))
    if _is_temporal(v) or _is_date(v):
        return _to_instant(v).at_utc().date
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to LocalDate")


def _to_local_date_time(v) -> LocalDateTime:
    if isinstance(v, LocalDateTime):
        return v
    if _is_local_date(v):
        return LocalDateTime(v, LocalTime(0))
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "local_date_time")
    if isinstance(v, str):
        return parse_local_date_time(v)
    if _is_temporal(v) or _is_number(v) or _is_date(v):
        return _to_instant(v).at_utc()
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to LocalDateTime")


# ------------------------------------------------------------------ numeric coercions
def _ms_of_day(v) -> int:
    lt = v.to_local_time() if isinstance(v, Time) else v
    return lt.nano_of_day // 1_000_000


def _to_double(v) -> float:
    if isinstance(v, LocalTime):
        return v.nano_of_day / 1_000_000
    if isinstance(v, Time):
        return v.to_local_time().nano_of_day / 1_000_000
    if isinstance(v, Timestamp):
        t = v.get_time()
        whole = (t // 1000 if t >= 0 else -((-t) // 1000)) * 1000   # Java long division
        return float(whole) + v.nanos / 1_000_000_000   # (sic) nanos / 1e9, as the reference
    if isinstance(v, JDate):
        return float(v.millis)
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "double")
    if _is_local_date(v):
        return float((v - _EPOCH_DATE).days)
    if _is_temporal(v):
        i = _to_instant(v)
        return float(i.seconds) * 1000 + i.nanos / 1_000_000
    return _el_number(v)


def _to_float(v) -> Float32:
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "float")
    if _is_local_date(v):
        return Float32(float((v - _EPOCH_DATE).days))
    import numpy as np
    return Float32(float(np.float32(_el_number(v))))


def _to_long(v) -> int:
    if isinstance(v, (LocalTime, Time)):
        return _ms_of_day(v)
    if isinstance(v, (JDate, Timestamp)):
        return v.get_time()
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "int64")
    if _is_local_date(v):
        return (v - _EPOCH_DATE).days
    if _is_temporal(v):
        return _to_instant(v).to_epoch_milli()
    return _d2l(_el_number(v), 64)


def _to_integer(v) -> Int32:
    if isinstance(v, (LocalTime, Time)):
        return Int32(_ms_of_day(v))
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "int32")
    if _is_local_date(v):
        d = (v - _EPOCH_DATE).days
        if not -(1 << 31) <= d < (1 << 31):
            raise ConversionError("integer overflow")
        return Int32(d)
    return Int32(_d2l(_el_number(v), 32))


def _to_short(v) -> Int16:
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "int16")
    return Int16(_wrap(_d2l(_el_number(v), 32), 16))


def _to_byte(v) -> Int8:
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "int8")
    if isinstance(v, bool):
        raise ConversionError(f"Cannot convert {v} of type Boolean to Byte")
    if isinstance(v, str):
        try:
            x = int(v.strip())
        except ValueError as e:
            raise ConversionError(f"Cannot convert {v!r} to Byte") from e
        if not -128 <= x <= 127:
            raise ConversionError(f"Value out of range. Value:\"{v}\" Radix:10")
        return Int8(x)
    if isinstance(v, (int, float, Decimal)):
        return Int8(_wrap(_d2l(float(v), 32) if not isinstance(v, int) else int(v), 8))
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Byte")


def _to_boolean(v) -> bool:
    if isinstance(v, (bytes, bytearray)):
        return decode_bytes(bytes(v), "boolean")
    if isinstance(v, bool):
        return v
    if isinstance(v, str):
        return v.strip().lower() == "true" if v else False
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to Boolean")


def _to_big_integer(v) -> int:
    if isinstance(v, int) and not isinstance(v, bool):
        return int(v)
    if isinstance(v, str):
        return int(v)
    if isinstance(v, (bytes, bytearray)):
        return int.from_bytes(bytes(v), "big", signed=True)
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to BigInteger")


def _to_big_decimal(v) -> Decimal:
    if isinstance(v, Decimal):
        return v
    if isinstance(v, str):
        return Decimal(v)
    if isinstance(v, int) and not isinstance(v, bool):
        return Decimal(int(v))
    if isinstance(v, float):   # BigDecimal.valueOf(double): Double.toString's digits
        return Decimal(java_double_str(float(v)).replace("E", "e"))
    raise ConversionError(f"Cannot convert {v!r} of type {type(v).__name__} to BigDecimal")


_TARGETS = {
    "boolean": _to_boolean, "double": _to_double, "float": _to_float, "int64": _to_long, "int16": _to_short,
    "int32": _to_integer, "int8": _to_byte, "string": to_java_string, "bytes": encode_bytes,
    "timestamp": _to_timestamp, "time": _to_time, "date": _to_date, "local_date_time": _to_local_date_time,
    "local_date": _to_local_date, "local_time": _to_local_time, "instant": _to_instant,
    "offset_date_time": _to_offset_date_time, "big_integer": _to_big_integer, "big_decimal": _to_big_decimal,
}
TARGETS = tuple(_TARGETS)


def coerce(value: Any, target: str) -> Optional[Any]:
    """JstlTypeConverter.coerceToType(value, target) -- target one of ``TARGETS``
    (schema-type spellings such as ``LOCAL_DATE_TIME`` / ``local-date-time`` accepted)."""
    if value is None:
        return None
    t = target.lower().replace("-", "_")
    t = {"long": "int64", "integer": "int32", "short": "int16", "byte": "int8", "bool": "boolean"}.get(t, t)
    fn = _TARGETS.get(t)
    if fn is None:
        raise ConversionError(f"Unsupported target type {target}")
    v = _from_python(value)
    if isinstance(v, bytearray):
        v = bytes(v)
    return fn(v)
