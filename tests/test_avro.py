"""Avro + schema-registry topics (VERDICT r3 "missing" #2/#3): the in-tree Avro codec, the
Confluent wire format, the schema-registry REST client against the in-process registry,
Kafka serde selection from keySchema / valueSchema (KAFKA/KafkaTopic.java:90-126), schema
registration on deploy (KRT/KafkaTopicConnectionsRuntime.java:232-325), the Java binary
serializers for untyped values (KRT/KafkaProducerWrapper.java:57-67) and AvroValue in and
out of a Python agent (RTPY/langstream_grpc/grpc_service.py:184-305)."""
import json
import os
import struct
import textwrap
import uuid

import pytest

from langstream_amd.api.avro import (AvroRecord, AvroSchema, canonical_form, decode, encode, fingerprint64,
                                     wire_decode, wire_encode)
from langstream_amd.api.types import Float32, Int16, Int32
from langstream_amd.topics.kafka import serde
from langstream_amd.topics.kafka.broker import KafkaBroker
from langstream_amd.topics.kafka.schema_registry import (SchemaRegistryClient, SchemaRegistryError,
                                                         SchemaRegistryServer)

USER = {
    "type": "record", "name": "User", "namespace": "com.example",
    "fields": [
        {"name": "name", "type": "string"},
        {"name": "age", "type": "int"},
        {"name": "score", "type": "double", "default": 0.0},
        {"name": "email", "type": ["null", "string"], "default": None},
        {"name": "tags", "type": {"type": "array", "items": "string"}},
        {"name": "attrs", "type": {"type": "map", "values": "long"}},
        {"name": "kind", "type": {"type": "enum", "name": "Kind", "symbols": ["A", "B", "C"]}},
        {"name": "id", "type": {"type": "fixed", "name": "Id16", "size": 4}},
        {"name": "blob", "type": "bytes"},
        {"name": "address", "type": {"type": "record", "name": "Address",
                                     "fields": [{"name": "city", "type": "string"},
                                                {"name": "zip", "type": ["null", "int"]}]}},
        {"name": "previous", "type": ["null", "Address"], "default": None},
        {"name": "ratio", "type": "float"},
        {"name": "ok", "type": "boolean"},
    ]}


def _user():
    return {"name": "Ada", "age": 36, "score": 1.5, "email": "ada@example.com", "tags": ["x", "y"],
            "attrs": {"a": 1, "b": -(1 << 40)}, "kind": "B", "id": b"\x01\x02\x03\x04", "blob": b"\x00\xff",
            "address": {"city": "London", "zip": None}, "previous": {"city": "Paris", "zip": 75001},
            "ratio": 0.25, "ok": True}


def test_spec_byte_vectors():
    assert encode("long", 1) == b"\x02" and encode("long", -1) == b"\x01" and encode("long", 64) == b"\x80\x01"
    assert encode("string", "foo") == b"\x06foo"
    # the spec's record example: {"a": 27, "b": "foo"} -> 36 06 66 6f 6f
    rec = {"type": "record", "name": "test", "fields": [{"name": "a", "type": "long"}, {"name": "b", "type": "string"}]}
    assert encode(rec, {"a": 27, "b": "foo"}) == bytes.fromhex("3606666f6f")
    # union ["null","string"]: index then value
    assert encode(["null", "string"], "a") == b"\x02\x02a" and encode(["null", "string"], None) == b"\x00"
    # array of longs [3, 27]: count 2, items, end 0
    assert encode({"type": "array", "items": "long"}, [3, 27]) == bytes.fromhex("04063600")
    assert encode("double", 1.0) == struct.pack("<d", 1.0) and encode("boolean", True) == b"\x01"


def test_roundtrip_complex_record():
    v = _user()
    data = encode(USER, v)
    out = decode(USER, data)
    assert isinstance(out, AvroRecord) and out.schema.root == "com.example.User"
    assert dict(out) == {**v, "address": out["address"], "previous": out["previous"]}
    assert dict(out["address"]) == v["address"] and dict(out["previous"]) == v["previous"]
    assert out["address"].schema.root == "com.example.Address"
    # defaults fill missing fields; re-encoding a decoded record is byte-identical
    v2 = dict(v)
    del v2["score"], v2["email"], v2["previous"]
    assert decode(USER, encode(USER, v2))["score"] == 0.0
    assert encode(USER, out) == data
    with pytest.raises(ValueError):
        encode(USER, {**v, "kind": "Z"})
    with pytest.raises(ValueError):
        encode(USER, {k: x for k, x in v.items() if k != "name"})


def test_canonical_form_and_fingerprint():
    a = AvroSchema(json.dumps(USER, indent=2))
    b = AvroSchema({**USER, "doc": "ignored", "aliases": ["x"]})
    assert a == b and canonical_form(a) == canonical_form(b)
    pcf = canonical_form({"type": "record", "name": "R", "namespace": "ns", "doc": "d",
                          "fields": [{"name": "f", "type": {"type": "int"}, "default": 1}]})
    assert pcf == '{"name":"ns.R","type":"record","fields":[{"name":"f","type":"int"}]}'
    assert fingerprint64(a) == fingerprint64(b) != fingerprint64("int")
    assert canonical_form("int") == '"int"'


def test_wire_format():
    data = wire_encode(7, USER, _user())
    assert data[0] == 0 and int.from_bytes(data[1:5], "big") == 7
    assert wire_decode(data, lambda i: USER if i == 7 else None)["name"] == "Ada"
    with pytest.raises(ValueError):
        wire_decode(b"\x01" + data[1:], lambda i: USER)


def test_schema_registry_client_and_server():
    srv = SchemaRegistryServer(basic_auth="u:p")
    try:
        c = SchemaRegistryClient(srv.url, basic_auth="u:p")
        sid = c.register("t-value", USER)
        assert c.register("t-value", json.dumps(USER)) == sid          # idempotent, cached
        assert SchemaRegistryClient(srv.url, basic_auth="u:p").register("t-value", USER) == sid
        sid2 = c.register("t-key", "string")
        assert sid2 != sid
        assert SchemaRegistryClient(srv.url, basic_auth="u:p").get_by_id(sid) == AvroSchema(USER)
        assert set(c.subjects()) == {"t-value", "t-key"}
        assert c.latest("t-value")["id"] == sid
        assert c.get_id("t-value", USER) == sid
        with pytest.raises(SchemaRegistryError):
            SchemaRegistryClient(srv.url).register("x", USER)                 # no credentials
        with pytest.raises(SchemaRegistryError):
            c.get_by_id(999)
    finally:
        srv.close()


def test_java_binary_serializers_for_untyped_values():
    s = serde.serialize_typed
    assert s("héllo") == "héllo".encode()
    assert s(True) == b"\x01" and s(False) == b"\x00"
    assert s(5) == (5).to_bytes(8, "big") and s(-2) == struct.pack(">q", -2)      # Long
    assert s(Int32(5)) == b"\x00\x00\x00\x05" and s(Int16(-1)) == b"\xff\xff"
    assert s(1.5) == struct.pack(">d", 1.5) and s(Float32(1.5)) == struct.pack(">f", 1.5)
    assert s(uuid.UUID(int=1)) == b"00000000-0000-0000-0000-000000000001"
    assert json.loads(s({"a": [1, 2]})) == {"a": [1, 2]}
    with pytest.raises(ValueError):
        s(object())


def test_serde_selection_from_schemas():
    assert serde.deserializer_for_schema(None) == serde.STRING_DESER
    assert serde.deserializer_for_schema({"type": "bytes"}) == serde.BYTES_DESER
    assert serde.deserializer_for_schema({"type": "avro", "schema": "{}"}) == serde.AVRO_DESER
    assert serde.serializer_for_schema({"type": "string"}) == serde.STRING_SER
    assert serde.serializer_for_schema(None) == serde.BYTES_SER
    with pytest.raises(ValueError):
        serde.serializer_for_schema({"type": "protobuf"})


def test_compute_step_int32_is_four_bytes_on_kafka():
    from langstream_amd.agents.genai.steps import _compute_value
    v = _compute_value("12", "INT32")
    assert v == 12 and serde.serialize_typed(v) == b"\x00\x00\x00\x0c"
    assert serde.serialize_typed(_compute_value("12", "INT64")) == (12).to_bytes(8, "big")


PROC = textwrap.dedent('''
    from langstream import AvroValue, Processor, SimpleRecord


    class Enrich(Processor):
        def process(self, record):
            v = record.value()
            assert isinstance(v, AvroValue), type(v)
            schema = dict(v.schema)
            schema["fields"] = list(schema["fields"]) + [{"name": "greeting", "type": "string"}]
            out = dict(v.value)
            out["greeting"] = "hello " + out["name"]
            return [SimpleRecord(AvroValue(schema=schema, value=out), key=record.key())]
''')


def test_avro_topics_end_to_end_with_python_agent(tmp_path):
    """Avro in -> python-processor (AvroValue in, AvroValue with an extended schema out) ->
    compute on the Avro value (value.age) -> Avro out; schemas registered on deploy under
    the TopicNameStrategy subjects; the output decodes from the registry by id."""
    from langstream_amd.runtime.local import LocalApplicationRunner
    broker = KafkaBroker(default_partitions=1).start()
    reg = SchemaRegistryServer()
    try:
        tin, tmid, tout = ("avro-in-" + uuid.uuid4().hex[:6], "avro-mid-" + uuid.uuid4().hex[:6],
                           "avro-out-" + uuid.uuid4().hex[:6])
        in_schema = {"type": "record", "name": "Person", "fields": [{"name": "name", "type": "string"},
                                                                     {"name": "age", "type": "int"}]}
        mid_schema = {"type": "record", "name": "Person", "fields": [
            {"name": "name", "type": "string"}, {"name": "age", "type": "int"},
            {"name": "greeting", "type": "string"}]}
        out_schema = {"type": "record", "name": "Person", "fields": [
            {"name": "name", "type": "string"}, {"name": "age", "type": "int"},
            {"name": "greeting", "type": "string"}, {"name": "next_age", "type": "int"}]}
        os.makedirs(tmp_path / "python")
        (tmp_path / "python" / "enrich.py").write_text(PROC)
        pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
    schema:
      type: avro
      schema: '{json.dumps(in_schema)}'
  - name: {tmid}
    creation-mode: create-if-not-exists
    schema:
      type: avro
      schema: '{json.dumps(mid_schema)}'
  - name: {tout}
    creation-mode: create-if-not-exists
    keySchema:
      type: string
    schema:
      type: avro
      schema: '{json.dumps(out_schema)}'
pipeline:
  - name: enrich
    type: python-processor
    input: {tin}
    output: {tmid}
    configuration:
      className: enrich.Enrich
  - name: compute
    type: compute
    input: {tmid}
    output: {tout}
    configuration:
      fields:
        - name: "value.next_age"
          expression: "value.age + 1"
          type: INT32
"""
        instance = f"""
instance:
  streamingCluster:
    type: kafka
    configuration:
      admin:
        bootstrap.servers: "{broker.bootstrap}"
        schema.registry.url: "{reg.url}"
"""
        app = LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, instance=instance,
                                               code_directory=str(tmp_path)).start(wait=20)
        try:
            client = SchemaRegistryClient(reg.url)
            assert {f"{tin}-value", f"{tmid}-value", f"{tout}-value"} <= set(client.subjects())
            for i, (n, a) in enumerate([("Ada", 36), ("Alan", 41)]):
                app.produce(tin, AvroRecord({"name": n, "age": a}, in_schema), key=f"k{i}")
            out = app.consume(tout, 2, timeout=30)
            assert len(out) == 2
            got = sorted((r.key(), dict(r.value())) for r in out)
            assert got == [("k0", {"name": "Ada", "age": 36, "greeting": "hello Ada", "next_age": 37}),
                           ("k1", {"name": "Alan", "age": 41, "greeting": "hello Alan", "next_age": 42})]
            assert all(isinstance(r.value(), AvroRecord) for r in out)
            # the raw bytes on the output topic are Confluent-framed Avro of the declared schema
            raw = app.topic_runtime.create_reader(app.streaming_cluster, {"topic": tout,
                                                  "value.deserializer": serde.BYTES_DESER},
                                                  __import__("langstream_amd.api.topics",
                                                             fromlist=["x"]).TopicOffsetPosition.EARLIEST)
            raw.start()
            recs = []
            for _ in range(50):
                recs += raw.read().records
                if len(recs) >= 2:
                    break
            assert recs and recs[0].value()[0] == 0
            assert wire_decode(recs[0].value(), client.get_by_id)["greeting"].startswith("hello")
            assert client.get_by_id(int.from_bytes(recs[0].value()[1:5], "big")) == AvroSchema(out_schema)
        finally:
            app.stop(10)
    finally:
        reg.close()
        broker.stop()


def test_avro_topic_without_registry_fails_deploy():
    from langstream_amd.runtime.local import LocalApplicationRunner
    broker = KafkaBroker(default_partitions=1).start()
    try:
        t = "avro-noreg-" + uuid.uuid4().hex[:6]
        pipe = f"""
topics:
  - name: {t}
    creation-mode: create-if-not-exists
    schema:
      type: avro
      schema: '{{"type": "record", "name": "R", "fields": [{{"name": "a", "type": "int"}}]}}'
pipeline:
  - name: id
    type: identity
    input: {t}
"""
        instance = f"""
instance:
  streamingCluster:
    type: kafka
    configuration:
      admin:
        bootstrap.servers: "{broker.bootstrap}"
"""
        with pytest.raises(ValueError, match="schema.registry.url"):
            LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, instance=instance).start(wait=10)
    finally:
        broker.stop()
