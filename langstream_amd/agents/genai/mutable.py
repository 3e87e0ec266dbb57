"""MutableRecord: the working form of a record inside the GenAI toolkit.

Parity: CMN/MutableRecord.java:58-563 -- key/value objects (JSON strings are parsed to
maps when possible: ``recordToMutableRecord(record, attemptJsonConversion=true)``),
properties (= headers as strings), input/output topic, event time, drop flag;
``set_result_field`` targets value / key / value.x / key.x / properties.x /
destinationTopic / messageKey (:309-360); the expression-language context exposes
key, value, messageKey, topicName, destinationTopic, eventTime, properties, record.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional

from ...api.record import Header, Record, SimpleRecord


def attempt_json(v: Any) -> Any:
    if isinstance(v, bytes):
        try:
            v = v.decode("utf-8")
        except UnicodeDecodeError:
            return v
    if isinstance(v, str):
        s = v.strip()
        if s[:1] in ("{", "["):
            try:
                return json.loads(s)
            except ValueError:
                return v
    return v


def _text_origin(r: Record, i: int):
    """str / bytes when the record's key (i = 0) or value (i = 1) is, or was before an
    upstream agent parsed it, JSON text; else None."""
    v = r.key() if i == 0 else r.value()
    if type(v) in (str, bytes):
        return type(v)
    ref = getattr(r, "_source_ref", None)
    if isinstance(ref, dict) and "json_origin" in ref:
        return ref["json_origin"][i]
    return None


def text_form(v: Any, origin) -> Any:
    """A map in the text form it came in: compact JSON (Jackson's writeValueAsString /
    writeValueAsBytes); anything else unchanged."""
    if isinstance(v, dict) and origin in (str, bytes):
        t = json.dumps(v, separators=(",", ":"), ensure_ascii=False, default=_json_default)
        return t if origin is str else t.encode("utf-8")
    return v


def _json_default(o):
    from ...utils.fastjson import _default
    return _default(o)


def safe_clone(v: Any) -> Any:
    """Copy the top level of a map/list value.  Enough for isolation: every mutation a
    step performs replaces a top-level entry (``set_result_field`` writes flat keys,
    drop-fields / merge / flatten / cast build new containers), so nested objects --
    e.g. retrieved documents with 384-float vectors -- are shared, never written.
    A deep copy per step dominated the per-record host cost of the RAG pipeline."""
    if isinstance(v, dict):
        if type(v) is dict:
            return dict(v)
        # a decoded Avro record stays one (cast prints it differently) but without its
        # schema: steps add / drop fields, so the writer re-derives the schema as for a map
        from ...api.avro import AvroRecord
        return AvroRecord(v) if isinstance(v, AvroRecord) else dict(v)
    if isinstance(v, list):
        return list(v)
    return v


def java_hashmap_order(d: dict) -> dict:
    """``d`` with its keys in the iteration order of a ``java.util.HashMap`` the same
    entries were put into (default capacity 16, load factor 0.75): buckets in index order
    (``hash ^ hash >>> 16`` masked to the table size), insertion order within a bucket --
    resizes split buckets without reordering them.  MutableRecord.copy() in the reference
    clones maps into HashMaps (``MutableRecord.safeClone``), so a copied record's JSON
    fields come out in this order (LangServeInvokeAgentRunnerIT's ``{"answer":..,"topic":..}``)."""
    n = len(d)
    if n < 2 or type(d) is not dict:
        return d
    from ...api.util import java_hash
    cap = 16
    while n > cap * 3 // 4:
        cap *= 2
    mask = cap - 1

    def bucket(k):
        h = java_hash(k) & 0xFFFFFFFF
        return (h ^ (h >> 16)) & mask
    return {k: d[k] for k in sorted(d, key=bucket)}


class MutableRecord:
    __slots__ = ("key", "value", "properties", "input_topic", "output_topic", "event_time", "drop",
                 "message_key", "record_object", "source", "hashmap")

    def __init__(self, key=None, value=None, properties=None, input_topic=None, event_time=None, source=None):
        self.key = key
        self.value = value
        self.properties: Dict[str, str] = dict(properties or {})
        self.input_topic = input_topic
        self.output_topic: Optional[str] = None
        self.event_time = event_time
        self.drop = False
        self.message_key = None
        self.record_object = None
        self.source = source
        # a copy(): its maps are java.util.HashMaps in the reference, so fields added later
        # also land in hash order (see java_hashmap_order); applied when leaving as a record
        self.hashmap = False

    @staticmethod
    def from_record(r: Record, attempt_json_conversion: bool = True) -> "MutableRecord":
        props = {}
        for h in r.headers():
            if h.key is not None and h.value is not None:
                props[h.key] = h.value_as_string()
        k0, v0 = r.key(), r.value()
        k, v = (attempt_json(k0), attempt_json(v0)) if attempt_json_conversion else (k0, v0)
        # a value parsed from JSON text is already a fresh object: no copy needed
        m = MutableRecord(k if k is not k0 else safe_clone(k), v if v is not v0 else safe_clone(v), props,
                          r.origin(), r.timestamp(), r)
        return m

    def copy(self) -> "MutableRecord":
        m = MutableRecord(safe_clone(self.key), safe_clone(self.value), dict(self.properties), self.input_topic,
                          self.event_time, self.source)
        m.hashmap = True
        m.output_topic = self.output_topic
        m.drop = self.drop
        m.message_key = self.message_key
        return m

    def shallow_copy(self) -> "MutableRecord":
        """Copy sharing nested objects: only the top-level key/value maps and the
        properties are duplicated, enough for set_result_field on the copy (used for
        every streamed answer chunk, where a deep copy of embeddings-laden values
        would dominate the cost)."""
        m = MutableRecord(dict(self.key) if isinstance(self.key, dict) else self.key,
                          dict(self.value) if isinstance(self.value, dict) else self.value,
                          dict(self.properties), self.input_topic, self.event_time, self.source)
        m.output_topic = self.output_topic
        m.drop = self.drop
        m.message_key = self.message_key
        m.hashmap = True
        return m

    def to_record(self) -> Optional[Record]:
        if self.drop:
            return None
        headers = [Header(k, v) for k, v in self.properties.items()]
        key = self.message_key if self.message_key is not None else self.key
        value = self.value
        if self.hashmap:
            key, value = java_hashmap_order(key) if isinstance(key, dict) else key, \
                java_hashmap_order(value) if isinstance(value, dict) else value
        r = SimpleRecord(key, value, self.input_topic, self.event_time, headers)
        ref = None
        if self.output_topic is not None:
            ref = {"destination_topic": self.output_topic}
        if self.source is not None and (isinstance(key, dict) or isinstance(self.value, dict)):
            # maps parsed from JSON text stay maps on the way downstream (the next agent would
            # parse them again), but remember the text form they came in: the reference hands
            # them on as compact JSON strings / bytes (MutableRecord.convertMapToStringOrBytes),
            # which is what a Python agent then receives (python_agents._to_user)
            origin = (_text_origin(self.source, 0), _text_origin(self.source, 1))
            if origin != (None, None):
                ref = dict(ref or {}, json_origin=origin)
        if ref is not None:
            r._source_ref = ref
        return r

    def el_context(self) -> Dict[str, Any]:
        return {"key": self.key, "value": self.value, "messageKey": self.message_key or self.key,
                "topicName": self.input_topic, "destinationTopic": self.output_topic, "eventTime": self.event_time,
                "properties": self.properties, "header": self.properties,
                "record": self.record_object if self.record_object is not None else
                {"key": self.key, "value": self.value}}

    def json_context(self) -> Dict[str, Any]:
        """Context for mustache templates: MutableRecord.toJsonRecord's JsonRecord (topicName,
        destinationTopic, key, value, properties, eventTime), plus origin / timestamp /
        messageKey aliases."""
        return {"key": self.key, "value": self.value, "topicName": self.input_topic,
                "destinationTopic": self.output_topic, "eventTime": self.event_time, "properties": self.properties,
                "origin": self.input_topic, "timestamp": self.event_time, "messageKey": self.message_key or self.key}

    def set_result_field(self, content: Any, field: Optional[str]) -> None:
        if field is None or field == "value":
            self.value = content
        elif field == "key":
            self.key = content
        elif field == "destinationTopic":
            self.output_topic = str(content)
        elif field == "messageKey":
            self.message_key = str(content)
        elif field.startswith("properties."):
            # header values are strings; booleans render like Java's Boolean.toString
            self.properties[field[len("properties."):]] = content if isinstance(content, str) else (
                json.dumps(content) if isinstance(content, (dict, list)) else
                ("true" if content else "false") if isinstance(content, bool) else str(content))
        elif field.startswith("value."):
            name = field[len("value."):]
            if not isinstance(self.value, dict):
                if self.value is None or self.value == "":
                    self.value = {}
                else:
                    raise ValueError("Cannot set a value field without a schema on a non-map value")
            _set_path(self.value, name, content)
        elif field.startswith("key."):
            name = field[len("key."):]
            if not isinstance(self.key, dict):
                if self.key is None:
                    self.key = {}
                else:
                    raise ValueError("Cannot set a key field without a schema on a non-map key")
            _set_path(self.key, name, content)
        else:
            raise ValueError(f"Cannot set field {field}: it does not refer to any part of the message")

    def get_field(self, field: str) -> Any:
        from .el import eval_expression
        return eval_expression(field, self.el_context())


def _set_path(d: dict, name: str, content: Any) -> None:
    # like the reference, "value.a.b" sets the flat key "a.b" (no nesting)
    d[name] = content
