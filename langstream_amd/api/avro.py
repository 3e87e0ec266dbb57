"""In-tree Apache Avro codec + Confluent wire format (no fastavro / avro package offline).

What the reference uses Avro for, and what this module gives the runtime:
* topics whose ``keySchema`` / ``valueSchema`` is ``type: avro`` are read with
  ``KafkaAvroDeserializer`` and written with ``KafkaAvroSerializer``
  (KAFKA/KafkaTopic.java:90-126, KRT/KafkaProducerWrapper.java:236-241): Avro binary
  encoding behind the Confluent framing ``0x00 | schema id (4 B big-endian) | payload``;
* schemas are registered in a Confluent schema registry on deploy under the
  TopicNameStrategy subjects ``<topic>-key`` / ``<topic>-value``
  (KRT/KafkaTopicConnectionsRuntime.java:232-325);
* Python agents exchange ``AvroValue(schema, value)`` (RTPY/langstream_grpc/grpc_service.py:
  184-305, which uses fastavro.schemaless_reader / writer and parsing canonical form).

Records decode to :class:`AvroRecord`, a ``dict`` that remembers its schema, so the
expression language reaches fields as ``value.x`` (CMN AvroUtil / MutableRecord) and a
record read from one Avro topic re-encodes unchanged on another.

Covered: null, boolean, int, long, float, double, bytes, string, record, enum, array,
map, union, fixed, named-type references and namespaces, field defaults, logical types
(carried on their underlying type), Parsing Canonical Form and its CRC-64-AVRO
fingerprint (the schema identity fastavro / Java use).
"""
from __future__ import annotations

import io
import json
import struct
from typing import Any, Dict, List, Optional, Tuple, Union

__all__ = ["AvroSchema", "AvroRecord", "parse_schema", "encode", "decode", "canonical_form", "fingerprint64",
           "wire_encode", "wire_decode", "MAGIC_BYTE"]

PRIMITIVES = ("null", "boolean", "int", "long", "float", "double", "bytes", "string")
NAMED = ("record", "error", "enum", "fixed")
MAGIC_BYTE = 0


class AvroError(ValueError):
    pass


# ------------------------------------------------------------------ schema parsing
class AvroSchema:
    """A parsed schema: ``root`` is the normalized JSON form (named types by full name,
    references as strings), ``names`` maps full names to their definitions."""

    def __init__(self, schema: Union[str, dict, list]):
        if isinstance(schema, AvroSchema):
            self.root, self.names = schema.root, schema.names
            self._canon = schema._canon
            return
        if isinstance(schema, (bytes, bytearray)):
            schema = schema.decode()
        if isinstance(schema, str):
            s = schema.strip()
            schema = json.loads(s) if s[:1] in "{[\"" else s
        self.names: Dict[str, dict] = {}
        self.root = self._parse(schema, None)
        self._canon: Optional[str] = None

    def _fullname(self, name: str, ns: Optional[str]) -> str:
        if "." in name or not ns:
            return name
        return f"{ns}.{name}"

    def _parse(self, s: Any, ns: Optional[str]) -> Any:
        if isinstance(s, str):
            if s in PRIMITIVES:
                return s
            full = self._fullname(s, ns)
            if full in self.names:
                return full
            if s in self.names:
                return s
            raise AvroError(f"unknown Avro type {s!r}")
        if isinstance(s, list):
            return [self._parse(b, ns) for b in s]
        if not isinstance(s, dict) or "type" not in s:
            raise AvroError(f"invalid Avro schema {s!r}")
        t = s["type"]
        if t in PRIMITIVES and "logicalType" not in s:
            return t
        if t in NAMED:
            name = s.get("name")
            if not name:
                raise AvroError(f"{t} needs a name")
            nns = s.get("namespace", ns) if "." not in name else name.rsplit(".", 1)[0]
            full = self._fullname(name, nns)
            node: Dict[str, Any] = {"type": "record" if t == "error" else t, "name": full}
            self.names[full] = node                    # before the fields: recursive types
            if t in ("record", "error"):
                fields = []
                for f in s.get("fields", []):
                    fd = {"name": f["name"], "type": self._parse(f["type"], nns)}
                    if "default" in f:
                        fd["default"] = f["default"]
                    fields.append(fd)
                node["fields"] = fields
            elif t == "enum":
                node["symbols"] = list(s["symbols"])
                if "default" in s:
                    node["default"] = s["default"]
            else:
                node["size"] = int(s["size"])
            if "logicalType" in s:
                node["logicalType"] = s["logicalType"]
            return full
        if t == "array":
            return {"type": "array", "items": self._parse(s["items"], ns)}
        if t == "map":
            return {"type": "map", "values": self._parse(s["values"], ns)}
        if t in PRIMITIVES:                            # with a logical type annotation
            out = {"type": t, "logicalType": s["logicalType"]}
            for k in ("precision", "scale"):
                if k in s:
                    out[k] = s[k]
            return out
        if isinstance(t, (dict, list)) or t in self.names or self._fullname(str(t), ns) in self.names:
            return self._parse(t, ns)
        raise AvroError(f"unsupported Avro type {t!r}")

    def resolve(self, t: Any) -> Any:
        while isinstance(t, str) and t not in PRIMITIVES:
            t = self.names[t]
        return t

    def to_json(self) -> Any:
        """The schema as JSON (named types defined at first use, by full name)."""
        seen = set()

        def go(t):
            if isinstance(t, str):
                if t in PRIMITIVES:
                    return t
                if t in seen:
                    return t
                seen.add(t)
                d = dict(self.names[t])
                if d["type"] == "record":
                    d["fields"] = [dict(f, type=go(f["type"])) for f in d["fields"]]
                return d
            if isinstance(t, list):
                return [go(b) for b in t]
            d = dict(t)
            if d["type"] == "array":
                d["items"] = go(d["items"])
            elif d["type"] == "map":
                d["values"] = go(d["values"])
            return d
        return go(self.root)

    def canonical(self) -> str:
        if self._canon is None:
            self._canon = canonical_form(self)
        return self._canon

    def __eq__(self, other):
        return isinstance(other, AvroSchema) and self.canonical() == other.canonical()

    def __hash__(self):
        return hash(self.canonical())

    def __repr__(self):
        return f"AvroSchema({self.canonical()})"


def parse_schema(schema: Any) -> AvroSchema:
    return schema if isinstance(schema, AvroSchema) else AvroSchema(schema)


def canonical_form(schema: Any) -> str:
    """Avro Parsing Canonical Form (spec "Transforming into Parsing Canonical Form"):
    full names, only the attributes that affect parsing, fixed attribute order, no
    whitespace; named types are written in full at first occurrence only."""
    sc = parse_schema(schema)
    seen = set()

    def go(t) -> str:
        if isinstance(t, str):
            if t in PRIMITIVES:
                return json.dumps(t)
            if t in seen:
                return json.dumps(t)
            seen.add(t)
            d = sc.names[t]
            parts = [f'"name":{json.dumps(d["name"])}', f'"type":{json.dumps(d["type"])}']
            if d["type"] == "record":
                fs = ",".join("{" + f'"name":{json.dumps(f["name"])},"type":{go(f["type"])}' + "}" for f in d["fields"])
                parts.append(f'"fields":[{fs}]')
            elif d["type"] == "enum":
                parts.append('"symbols":[' + ",".join(json.dumps(x) for x in d["symbols"]) + "]")
            else:
                parts.append(f'"size":{d["size"]}')
            return "{" + ",".join(parts) + "}"
        if isinstance(t, list):
            return "[" + ",".join(go(b) for b in t) + "]"
        if t["type"] == "array":
            return '{"type":"array","items":' + go(t["items"]) + "}"
        if t["type"] == "map":
            return '{"type":"map","values":' + go(t["values"]) + "}"
        return json.dumps(t["type"])                   # primitive with a logical type
    return go(sc.root)


_CRC64_EMPTY = 0xC15D213AA4D7A795
_CRC64_TABLE: List[int] = []


def fingerprint64(schema: Any) -> int:
    """CRC-64-AVRO (Rabin) fingerprint of the Parsing Canonical Form."""
    if not _CRC64_TABLE:
        for i in range(256):
            fp = i
            for _ in range(8):
                fp = (fp >> 1) ^ (_CRC64_EMPTY & -(fp & 1))
            _CRC64_TABLE.append(fp)
    fp = _CRC64_EMPTY
    for b in canonical_form(schema).encode():
        fp = (fp >> 8) ^ _CRC64_TABLE[(fp ^ b) & 0xFF]
    return fp


# ------------------------------------------------------------------ values
class AvroRecord(dict):
    """A decoded Avro record (GenericRecord equivalent): the field dict plus its schema.
    JSON-serialisable and EL-addressable like any dict value."""

    __slots__ = ("schema",)

    def __init__(self, fields: Optional[dict] = None, schema: Any = None):
        super().__init__(fields or {})
        self.schema = parse_schema(schema) if schema is not None else None

    def __repr__(self):
        name = ""
        if self.schema is not None and isinstance(self.schema.root, str):
            name = self.schema.root
        return f"AvroRecord<{name}>({dict.__repr__(self)})"

    def __reduce__(self):
        return (AvroRecord, (dict(self), self.schema.to_json() if self.schema is not None else None))


# ------------------------------------------------------------------ binary encoding
def _write_long(buf: io.BytesIO, n: int) -> None:
    n = (n << 1) ^ (n >> 63)
    n &= 0xFFFFFFFFFFFFFFFF
    while n & ~0x7F:
        buf.write(bytes(((n & 0x7F) | 0x80,)))
        n >>= 7
    buf.write(bytes((n,)))


def _read_long(data: memoryview, pos: int) -> Tuple[int, int]:
    b = data[pos]
    pos += 1
    n = b & 0x7F
    shift = 7
    while b & 0x80:
        if pos >= len(data):
            raise AvroError("truncated varint")
        b = data[pos]
        pos += 1
        n |= (b & 0x7F) << shift
        shift += 7
        if shift > 70:
            raise AvroError("varint too long")
    return (n >> 1) ^ -(n & 1), pos


def _matches(sc: AvroSchema, t: Any, v: Any) -> bool:
    t = sc.resolve(t)
    tt = t if isinstance(t, str) else t["type"] if isinstance(t, dict) else "union"
    if tt == "null":
        return v is None
    if tt == "boolean":
        return isinstance(v, bool)
    if tt == "int":
        return isinstance(v, int) and not isinstance(v, bool) and -(1 << 31) <= v < (1 << 31)
    if tt == "long":
        return isinstance(v, int) and not isinstance(v, bool) and -(1 << 63) <= v < (1 << 63)
    if tt in ("float", "double"):
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    if tt == "bytes":
        return isinstance(v, (bytes, bytearray))
    if tt == "string":
        return isinstance(v, str)
    if tt == "fixed":
        return isinstance(v, (bytes, bytearray)) and len(v) == t["size"]
    if tt == "enum":
        return isinstance(v, str) and v in t["symbols"]
    if tt == "array":
        return isinstance(v, (list, tuple))
    if tt == "map":
        return isinstance(v, dict) and not (isinstance(v, AvroRecord) and v.schema is not None)
    if tt == "record":
        if not isinstance(v, dict):
            return False
        if isinstance(v, AvroRecord) and v.schema is not None and isinstance(v.schema.root, str):
            return v.schema.root == t["name"]
        return all(f["name"] in v or "default" in f for f in t["fields"])
    return False


def _branch_name(sc: AvroSchema, t: Any) -> str:
    t = sc.resolve(t)
    if isinstance(t, str):
        return t
    return t.get("name") or t["type"]


def _enc(sc: AvroSchema, t: Any, v: Any, buf: io.BytesIO) -> None:
    if isinstance(t, list):                            # union
        idx = None
        if isinstance(v, tuple) and len(v) == 2 and isinstance(v[0], str):
            # explicit branch (fastavro's (name, value) tuple notation)
            for i, b in enumerate(t):
                if _branch_name(sc, b) in (v[0], v[0].rsplit(".", 1)[-1]):
                    idx, v = i, v[1]
                    break
        if idx is None:
            for i, b in enumerate(t):
                if _matches(sc, b, v):
                    idx = i
                    break
        if idx is None:
            raise AvroError(f"value {v!r} matches no branch of union {canonical_form_of(sc, t)}")
        _write_long(buf, idx)
        _enc(sc, t[idx], v, buf)
        return
    rt = sc.resolve(t)
    tt = rt if isinstance(rt, str) else rt["type"]
    if tt == "null":
        if v is not None:
            raise AvroError(f"null expected, got {v!r}")
    elif tt == "boolean":
        buf.write(b"\x01" if v else b"\x00")
    elif tt in ("int", "long"):
        if isinstance(v, bool) or not isinstance(v, int):
            raise AvroError(f"{tt} expected, got {v!r}")
        _write_long(buf, v)
    elif tt == "float":
        buf.write(struct.pack("<f", float(v)))
    elif tt == "double":
        buf.write(struct.pack("<d", float(v)))
    elif tt == "bytes":
        b = bytes(v)
        _write_long(buf, len(b))
        buf.write(b)
    elif tt == "string":
        if not isinstance(v, str):
            raise AvroError(f"string expected, got {v!r}")
        b = v.encode("utf-8")
        _write_long(buf, len(b))
        buf.write(b)
    elif tt == "fixed":
        b = bytes(v)
        if len(b) != rt["size"]:
            raise AvroError(f"fixed {rt['name']} needs {rt['size']} bytes, got {len(b)}")
        buf.write(b)
    elif tt == "enum":
        try:
            _write_long(buf, rt["symbols"].index(v))
        except ValueError:
            raise AvroError(f"{v!r} is not a symbol of enum {rt['name']}") from None
    elif tt == "array":
        items = list(v)
        if items:
            _write_long(buf, len(items))
            for it in items:
                _enc(sc, rt["items"], it, buf)
        _write_long(buf, 0)
    elif tt == "map":
        if v:
            _write_long(buf, len(v))
            for k, it in v.items():
                kb = str(k).encode("utf-8")
                _write_long(buf, len(kb))
                buf.write(kb)
                _enc(sc, rt["values"], it, buf)
        _write_long(buf, 0)
    elif tt == "record":
        if not isinstance(v, dict):
            raise AvroError(f"record {rt['name']} expected, got {v!r}")
        for f in rt["fields"]:
            if f["name"] in v:
                fv = v[f["name"]]
            elif "default" in f:
                fv = f["default"]
            else:
                raise AvroError(f"record {rt['name']}: field {f['name']} missing and has no default")
            _enc(sc, f["type"], fv, buf)
    else:
        raise AvroError(f"cannot encode type {tt}")


def canonical_form_of(sc: AvroSchema, t: Any) -> str:
    try:
        return json.dumps(t)
    except TypeError:
        return repr(t)


def _dec(sc: AvroSchema, t: Any, data: memoryview, pos: int) -> Tuple[Any, int]:
    if isinstance(t, list):
        idx, pos = _read_long(data, pos)
        if not 0 <= idx < len(t):
            raise AvroError(f"union index {idx} out of range")
        return _dec(sc, t[idx], data, pos)
    rt = sc.resolve(t)
    tt = rt if isinstance(rt, str) else rt["type"]
    if tt == "null":
        return None, pos
    if tt == "boolean":
        return data[pos] != 0, pos + 1
    if tt in ("int", "long"):
        return _read_long(data, pos)
    if tt == "float":
        return struct.unpack_from("<f", data, pos)[0], pos + 4
    if tt == "double":
        return struct.unpack_from("<d", data, pos)[0], pos + 8
    if tt in ("bytes", "string"):
        n, pos = _read_long(data, pos)
        if n < 0 or pos + n > len(data):
            raise AvroError("truncated bytes/string")
        raw = bytes(data[pos:pos + n])
        return (raw.decode("utf-8") if tt == "string" else raw), pos + n
    if tt == "fixed":
        n = rt["size"]
        return bytes(data[pos:pos + n]), pos + n
    if tt == "enum":
        i, pos = _read_long(data, pos)
        return rt["symbols"][i], pos
    if tt == "array":
        out = []
        while True:
            n, pos = _read_long(data, pos)
            if n == 0:
                return out, pos
            if n < 0:                                  # block with a byte size
                n = -n
                _, pos = _read_long(data, pos)
            for _ in range(n):
                v, pos = _dec(sc, rt["items"], data, pos)
                out.append(v)
    if tt == "map":
        out = {}
        while True:
            n, pos = _read_long(data, pos)
            if n == 0:
                return out, pos
            if n < 0:
                n = -n
                _, pos = _read_long(data, pos)
            for _ in range(n):
                k, pos = _dec(sc, "string", data, pos)
                v, pos = _dec(sc, rt["values"], data, pos)
                out[k] = v
    if tt == "record":
        rec = AvroRecord(schema=None)
        rec.schema = sc if t is sc.root else _sub_schema(sc, rt["name"])
        for f in rt["fields"]:
            rec[f["name"]], pos = _dec(sc, f["type"], data, pos)
        return rec, pos
    raise AvroError(f"cannot decode type {tt}")


def _sub_schema(sc: AvroSchema, name: str) -> AvroSchema:
    """The schema of a nested named record (shares the parent's name table)."""
    sub = AvroSchema.__new__(AvroSchema)
    sub.root, sub.names, sub._canon = name, sc.names, None
    return sub


def encode(schema: Any, value: Any) -> bytes:
    """Avro binary encoding of ``value`` (schemaless, like fastavro.schemaless_writer)."""
    sc = parse_schema(schema)
    buf = io.BytesIO()
    _enc(sc, sc.root, value, buf)
    return buf.getvalue()


def decode(schema: Any, data: bytes) -> Any:
    """Inverse of encode (fastavro.schemaless_reader); records come back as AvroRecord."""
    sc = parse_schema(schema)
    v, pos = _dec(sc, sc.root, memoryview(data), 0)
    if pos != len(data):
        raise AvroError(f"{len(data) - pos} trailing bytes after the Avro datum")
    return v


def wire_encode(schema_id: int, schema: Any, value: Any) -> bytes:
    """Confluent framing: magic byte 0, 4-byte big-endian schema id, Avro binary."""
    return bytes((MAGIC_BYTE,)) + int(schema_id).to_bytes(4, "big") + encode(schema, value)


def wire_decode(data: bytes, schema_for_id) -> Any:
    """Decode a Confluent-framed datum; ``schema_for_id(id)`` returns the writer schema."""
    if len(data) < 5 or data[0] != MAGIC_BYTE:
        raise AvroError("not a schema-registry framed Avro datum (magic byte 0 missing)")
    sid = int.from_bytes(data[1:5], "big")
    return decode(schema_for_id(sid), data[5:])
