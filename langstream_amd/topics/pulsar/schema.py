"""Pulsar schemas for the WebSocket/admin-REST adapter.

Parity with ``PulsarTopicConnectionsRuntimeProvider.java``:
* deploy (``:256-308``): a topic with a ``valueSchema`` and no registered schema gets one
  through the admin API -- ``SchemaInfo{type = schema type upper-cased, name, properties
  {}, schema = the definition's text}``; with a ``keySchema`` too, a KeyValue schema in
  the SEPARATED encoding;
* producer (``:595-731``): the topic's configured schema, else one inferred from the first
  record's types (``BASE_SCHEMAS``: String -> STRING, Boolean -> BOOLEAN, Integer ->
  INT32, Long -> INT64, Double -> DOUBLE, byte[] -> BYTES; a non-null key makes it
  ``KeyValue<key, value>`` SEPARATED); the Java client registers that schema when the
  producer is created, which the adapter does through the admin API;
* consumer / reader (``:536``, ``AUTO_CONSUME``): values decoded with the topic's
  registered schema (a KeyValue message yields its key and value).

Wire forms (the bytes Java producers / consumers of the same topic use): STRING UTF-8;
INT8/16/32/64 and FLOAT/DOUBLE big-endian fixed width; BOOLEAN one byte; BYTES raw; JSON
UTF-8 JSON; AVRO the Avro binary encoding (``api/avro.py``, no framing).  KeyValue
SEPARATED carries the key bytes in the message key (a STRING key as text, any other key
base64 -- the WebSocket API has no ``partitionKeyB64Encoded`` flag, so Java readers of a
non-STRING key see its base64 text) and the value bytes as the payload.
"""
from __future__ import annotations

import base64
import json
import struct
from typing import Any, Dict, Optional, Tuple

import datetime as _dt

from ...api import avro, temporal
from ...utils import fastjson
from ...api.types import Float32, Int8, Int16, Int32

TEMPORAL_TYPES = ("DATE", "TIME", "TIMESTAMP", "INSTANT", "LOCAL_DATE", "LOCAL_TIME", "LOCAL_DATE_TIME")
PRIMITIVE_TYPES = ("STRING", "BYTES", "BOOLEAN", "INT8", "INT16", "INT32", "INT64", "FLOAT", "DOUBLE") + TEMPORAL_TYPES
_FMT = {"INT8": ">b", "INT16": ">h", "INT32": ">i", "INT64": ">q", "FLOAT": ">f", "DOUBLE": ">d"}


class SchemaError(ValueError):
    pass


class PulsarSchema:
    """One (non-KeyValue) schema: ``type`` (Pulsar SchemaType name), ``definition`` (the
    schema text for AVRO / JSON), ``name``."""

    def __init__(self, type_: str, definition: Optional[str] = None, name: Optional[str] = None):
        self.type = type_.upper()
        if self.type not in PRIMITIVE_TYPES + ("AVRO", "JSON", "NONE"):
            raise SchemaError(f"unsupported Pulsar schema type {type_!r}")
        self.definition = definition or ""
        self.name = name or ""
        self._avro = avro.parse_schema(self.definition) if self.type == "AVRO" and self.definition else None

    @classmethod
    def from_definition(cls, d: Optional[Dict[str, Any]]) -> Optional["PulsarSchema"]:
        """A topic's ``keySchema`` / ``valueSchema`` as the planner passes it."""
        if not d:
            return None
        sch = d.get("schema")
        if isinstance(sch, (dict, list)):
            sch = json.dumps(sch)
        return cls(str(d.get("type") or "bytes"), sch, d.get("name"))

    def info(self) -> Dict[str, Any]:
        return {"type": self.type, "name": self.name, "schema": self.definition, "properties": {}}

    def __eq__(self, other) -> bool:
        return isinstance(other, PulsarSchema) and (self.type, self.definition) == (other.type, other.definition)

    def __repr__(self) -> str:
        return f"PulsarSchema({self.type})"

    # -- codec
    def encode(self, v: Any) -> bytes:
        t = self.type
        if v is None:
            return b""
        if t in ("BYTES", "NONE"):
            if isinstance(v, (bytes, bytearray)):
                return bytes(v)
            return (v if isinstance(v, str) else fastjson.dumps(v)).encode()
        if t == "STRING":
            if isinstance(v, (bytes, bytearray)):
                return bytes(v)
            return (v if isinstance(v, str) else fastjson.dumps(v)).encode()
        if t == "BOOLEAN":
            if isinstance(v, str):
                v = v.strip().lower() == "true"
            return b"\x01" if v else b"\x00"
        if t in _FMT:
            try:
                x = float(v) if t in ("FLOAT", "DOUBLE") else int(v)
                return struct.pack(_FMT[t], x)
            except (TypeError, ValueError, struct.error) as e:
                raise SchemaError(f"cannot encode {v!r} as {t}: {e}") from e
        if t in TEMPORAL_TYPES:
            # Pulsar's DateSchema / TimeSchema / TimestampSchema (int64 millis), InstantSchema
            # (int64 s + int32 nanos), LocalDate / LocalTime / LocalDateTime schemas (epoch
            # day, nano of day) -- the value converted to the type first (JstlTypeConverter)
            try:
                return temporal.encode_bytes(temporal.coerce(v, t))
            except ValueError as e:
                raise SchemaError(f"cannot encode {v!r} as {t}: {e}") from e
        if t == "JSON":
            if isinstance(v, (bytes, bytearray)):
                v = v.decode()
            if isinstance(v, str):
                json.loads(v)                      # must be a JSON document already
                return v.encode()
            return fastjson.dumps(v).encode()
        if t == "AVRO":
            if isinstance(v, (bytes, bytearray)):
                return bytes(v)
            if isinstance(v, str):
                v = json.loads(v)
            return avro.encode(self._avro, v)
        raise SchemaError(f"cannot encode as {t}")

    def decode(self, b: bytes) -> Any:
        t = self.type
        if t in ("BYTES", "NONE"):
            try:
                return b.decode()
            except UnicodeDecodeError:
                return b
        if t == "STRING":
            return b.decode()
        if t == "BOOLEAN":
            if len(b) != 1:
                raise SchemaError(f"BOOLEAN payload of {len(b)} bytes")
            return b != b"\x00"
        if t in _FMT:
            if len(b) != struct.calcsize(_FMT[t]):
                raise SchemaError(f"{t} payload of {len(b)} bytes")
            return struct.unpack(_FMT[t], b)[0]
        if t in TEMPORAL_TYPES:
            try:
                return temporal.decode_bytes(b, t.lower())
            except ValueError as e:
                raise SchemaError(f"{t} payload: {e}") from e
        if t == "JSON":
            return json.loads(b.decode())
        if t == "AVRO":
            return avro.decode(self._avro, b)
        raise SchemaError(f"cannot decode {t}")


class TopicSchema:
    """A topic's schema: a plain one, or KeyValue(key, value) SEPARATED."""

    def __init__(self, value: PulsarSchema, key: Optional[PulsarSchema] = None, name: Optional[str] = None):
        self.value, self.key = value, key
        self.name = name or value.name

    @property
    def is_kv(self) -> bool:
        return self.key is not None

    @classmethod
    def from_definitions(cls, key_def, value_def) -> Optional["TopicSchema"]:
        v = PulsarSchema.from_definition(value_def)
        if v is None:
            return None
        return cls(v, PulsarSchema.from_definition(key_def))

    # -- the admin REST forms (PostSchemaPayload / GetSchemaResponse)
    def rest_payload(self) -> Dict[str, Any]:
        if not self.is_kv:
            return {"type": self.value.type, "schema": self.value.definition, "properties": {}}

        def data(s: PulsarSchema):
            if s.type in ("AVRO", "JSON") and s.definition:
                return json.loads(s.definition)
            return ""

        props = {"key.schema.name": self.key.name, "key.schema.type": self.key.type, "key.schema.properties": "{}",
                 "value.schema.name": self.value.name, "value.schema.type": self.value.type,
                 "value.schema.properties": "{}", "kv.encoding.type": "SEPARATED"}
        return {"type": "KEY_VALUE", "schema": json.dumps({"key": data(self.key), "value": data(self.value)}),
                "properties": props}

    @classmethod
    def from_rest(cls, d: Dict[str, Any]) -> "TopicSchema":
        t = str(d.get("type", "BYTES")).upper()
        if t != "KEY_VALUE":
            return cls(PulsarSchema(t, d.get("data") if d.get("data") is not None else d.get("schema")))
        props = d.get("properties") or {}
        raw = d.get("data") if d.get("data") is not None else d.get("schema")
        doc = json.loads(raw) if raw else {}

        def part(which: str) -> PulsarSchema:
            sd = doc.get(which)
            return PulsarSchema(props.get(f"{which}.schema.type", "BYTES"),
                                json.dumps(sd) if isinstance(sd, (dict, list)) else (sd or None),
                                props.get(f"{which}.schema.name"))
        if props.get("kv.encoding.type", "SEPARATED") != "SEPARATED":
            raise SchemaError("only the SEPARATED KeyValue encoding is supported")
        return cls(part("value"), part("key"))

    def __eq__(self, other) -> bool:
        return isinstance(other, TopicSchema) and (self.value, self.key) == (other.value, other.key)

    # -- messages
    def encode_message(self, key: Any, value: Any) -> Tuple[Optional[str], bytes]:
        """(message key text, payload bytes)."""
        payload = self.value.encode(value)
        if self.is_kv:
            if key is None:
                return None, payload
            kb = self.key.encode(key)
            if self.key.type == "STRING":
                return kb.decode(), payload
            return base64.b64encode(kb).decode(), payload
        if key is None:
            return None, payload
        if isinstance(key, (bytes, bytearray)):
            return base64.b64encode(bytes(key)).decode(), payload
        return (key if isinstance(key, str) else json.dumps(key)), payload

    def decode_message(self, key: Optional[str], payload: bytes) -> Tuple[Any, Any]:
        value = self.value.decode(payload) if payload or self.value.type in ("STRING", "BYTES", "NONE") else None
        if self.is_kv and key is not None and self.key.type != "STRING":
            return self.key.decode(base64.b64decode(key)), value
        return key, value


# Java classes of BASE_SCHEMAS that Python values carry as tags (api/types.py,
# api/temporal.py): Byte / Short / Integer / Float and the date-time classes
_TAGGED = ((Int8, "INT8"), (Int16, "INT16"), (Int32, "INT32"), (Float32, "FLOAT"),
           (temporal.JDate, "DATE"), (temporal.Timestamp, "TIMESTAMP"), (temporal.Time, "TIME"),
           (temporal.Instant, "INSTANT"), (temporal.LocalTime, "LOCAL_TIME"),
           (temporal.LocalDateTime, "LOCAL_DATE_TIME"))


def infer(key: Any, value: Any) -> TopicSchema:
    """``BASE_SCHEMAS`` by the record's Python types (JSON-ish values: a str schema with
    JSON text -- the reference's ``getSchema`` has no entry for maps)."""
    def one(v: Any) -> PulsarSchema:
        if v is None or isinstance(v, (bytes, bytearray)):
            return PulsarSchema("BYTES")
        if isinstance(v, bool):
            return PulsarSchema("BOOLEAN")
        for cls, name in _TAGGED:
            if isinstance(v, cls):
                return PulsarSchema(name)
        if isinstance(v, int):
            return PulsarSchema("INT32" if -(1 << 31) <= v < (1 << 31) else "INT64")
        if isinstance(v, float):
            return PulsarSchema("DOUBLE")
        if isinstance(v, _dt.date) and not isinstance(v, _dt.datetime):
            return PulsarSchema("LOCAL_DATE")
        return PulsarSchema("STRING")
    if key is None:
        return TopicSchema(one(value))
    return TopicSchema(one(value), one(key))
