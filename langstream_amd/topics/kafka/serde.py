"""Kafka key / value / header serialisation with the reference's rules.

Producer (KRT/KafkaProducerWrapper.java:57-270):
* a topic with a ``keySchema`` / ``valueSchema`` forces the serializer
  (KAFKA/KafkaTopic.java:107-121): ``string`` -> StringSerializer, ``bytes`` ->
  ByteArraySerializer, ``avro`` -> KafkaAvroSerializer;
* otherwise the serializer follows the Java type of each value: String (UTF-8),
  Boolean (1 byte), Short / Integer / Long (2 / 4 / 8 bytes big-endian), Float / Double
  (IEEE-754 big-endian), byte[], UUID (its string form), Map / Collection (JSON), Avro
  GenericRecord (KafkaAvroSerializer; never for headers) -- anything else fails with
  "Cannot find a serializer".  Python ints are Longs and floats Doubles unless tagged
  with api/types.py (Int16 / Int32 / Float32, what the compute step's INT16 / INT32 /
  FLOAT produce).
Consumer (KAFKA/KafkaTopic.java:90-104): StringDeserializer unless the schema says
``bytes`` (ByteArrayDeserializer) or ``avro`` (KafkaAvroDeserializer -> AvroRecord).
"""
from __future__ import annotations

import struct
import uuid
from typing import Any, Callable, Dict, Optional

from ...api.avro import AvroRecord, AvroSchema, parse_schema, wire_decode, wire_encode
from ...api.types import Float32, Int8, Int16, Int32
from ...utils import fastjson
from .schema_registry import SchemaRegistryClient, subject_name

STRING_SER = "org.apache.kafka.common.serialization.StringSerializer"
BYTES_SER = "org.apache.kafka.common.serialization.ByteArraySerializer"
AVRO_SER = "io.confluent.kafka.serializers.KafkaAvroSerializer"
STRING_DESER = "org.apache.kafka.common.serialization.StringDeserializer"
BYTES_DESER = "org.apache.kafka.common.serialization.ByteArrayDeserializer"
AVRO_DESER = "io.confluent.kafka.serializers.KafkaAvroDeserializer"

_SER_FOR_SCHEMA = {"string": STRING_SER, "bytes": BYTES_SER, "avro": AVRO_SER}
_DESER_FOR_SCHEMA = {"string": STRING_DESER, "bytes": BYTES_DESER, "avro": AVRO_DESER}


def serializer_for_schema(schema: Optional[Dict[str, Any]]) -> str:
    if not schema:
        return BYTES_SER          # "configured without a serializer": reflection per value
    t = schema.get("type")
    if t not in _SER_FOR_SCHEMA:
        raise ValueError(f"Unsupported schema type: {t}")
    return _SER_FOR_SCHEMA[t]


def deserializer_for_schema(schema: Optional[Dict[str, Any]]) -> str:
    if not schema:
        return STRING_DESER       # the default: people usually use schemaless JSON
    t = schema.get("type")
    if t not in _DESER_FOR_SCHEMA:
        raise ValueError(f"Unsupported schema type: {t}")
    return _DESER_FOR_SCHEMA[t]


def serialize_typed(v: Any, avro: Optional[Callable[[AvroRecord], bytes]] = None) -> Optional[bytes]:
    """Reflection-based serialisation (the BASE_SERIALIZERS table + JSON + Avro)."""
    t = type(v)
    if t is dict:   # the common cases first, by exact type (one check instead of ~10)
        return fastjson.dumps(v).encode()
    if t is str:
        return v.encode("utf-8")
    if v is None:
        return None
    if isinstance(v, (bytes, bytearray, memoryview)):
        return bytes(v)
    if isinstance(v, str):
        return v.encode("utf-8")
    if isinstance(v, bool):
        return b"\x01" if v else b"\x00"
    if isinstance(v, int):
        if isinstance(v, Int8):
            raise ValueError("Cannot find a serializer for class java.lang.Byte")
        if isinstance(v, Int16):
            return struct.pack(">h", v)
        if isinstance(v, Int32):
            return struct.pack(">i", v)
        return struct.pack(">q", v)
    if isinstance(v, float):
        return struct.pack(">f", v) if isinstance(v, Float32) else struct.pack(">d", v)
    if isinstance(v, uuid.UUID):
        return str(v).encode()
    if isinstance(v, AvroRecord) and v.schema is not None:
        if avro is None:
            raise ValueError("Cannot find a serializer for an Avro GenericRecord in a header")
        return avro(v)
    if isinstance(v, (dict, list, tuple, set)):
        return fastjson.dumps(list(v) if isinstance(v, (tuple, set)) else v).encode()
    raise ValueError(f"Cannot find a serializer for {type(v).__name__}")


class AvroSerializer:
    """KafkaAvroSerializer: registers (auto.register.schemas, default true) or looks up
    the writer schema under the TopicNameStrategy subject and frames the datum."""

    def __init__(self, registry: Optional[SchemaRegistryClient], topic: str, is_key: bool,
                 topic_schema: Optional[AvroSchema] = None, auto_register: bool = True):
        self.registry, self.topic, self.is_key = registry, topic, is_key
        self.topic_schema, self.auto_register = topic_schema, auto_register
        self._ids: Dict[str, int] = {}

    def __call__(self, v: Any) -> bytes:
        if self.registry is None:
            raise ValueError("Avro serialisation needs schema.registry.url in the streaming cluster configuration")
        schema = v.schema if isinstance(v, AvroRecord) and v.schema is not None else self.topic_schema
        if schema is None:
            raise ValueError(f"no Avro schema for a {type(v).__name__} value on topic {self.topic}")
        canon = schema.canonical()
        sid = self._ids.get(canon)
        if sid is None:
            subj = subject_name(self.topic, self.is_key)
            sid = self.registry.register(subj, schema) if self.auto_register else self.registry.get_id(subj, schema)
            self._ids[canon] = sid
        return wire_encode(sid, schema, v)


class ValueSerializer:
    """One side (key or value) of a producer."""

    def __init__(self, cls: str, avro: Optional[AvroSerializer]):
        self.cls, self.avro = cls, avro

    def __call__(self, v: Any) -> Optional[bytes]:
        if v is None:
            return None
        if self.cls == STRING_SER:
            return (v if isinstance(v, str) else fastjson.dumps(v) if isinstance(v, (dict, list)) else str(v)).encode()
        if self.cls == AVRO_SER:
            return self.avro(v)
        # ByteArraySerializer configured (a "bytes" schema, or no schema at all) is
        # the reflection path in the reference: forced == not ByteArraySerializer
        return serialize_typed(v, self.avro)


class ValueDeserializer:
    def __init__(self, cls: str, registry: Optional[SchemaRegistryClient]):
        self.cls, self.registry = cls, registry

    def __call__(self, b: Optional[bytes]) -> Any:
        if b is None:
            return None
        if self.cls == BYTES_DESER:
            return bytes(b)
        if self.cls == AVRO_DESER:
            if self.registry is None:
                raise ValueError("Avro deserialisation needs schema.registry.url in the streaming cluster configuration")
            return wire_decode(bytes(b), self.registry.get_by_id)
        try:
            return bytes(b).decode("utf-8")
        except UnicodeDecodeError:
            return bytes(b)


def topic_schema(d: Optional[Dict[str, Any]]) -> Optional[AvroSchema]:
    if d and d.get("type") == "avro" and d.get("schema"):
        return parse_schema(d["schema"])
    return None
