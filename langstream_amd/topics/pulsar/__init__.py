"""``pulsar`` streaming cluster over Pulsar's WebSocket + admin REST APIs.

Parity with the reference (``langstream-pulsar/PulsarStreamingClusterRuntime.java``,
``PulsarClusterRuntimeConfiguration.java``, ``langstream-pulsar-runtime/
PulsarTopicConnectionsRuntimeProvider.java``):
* configuration ``admin.serviceUrl`` (HTTP), ``service.serviceUrl``, ``default-tenant``
  (``public``), ``default-namespace`` (``default``), ``authentication.token``; topic
  ``name`` -> ``persistent://<tenant>/<namespace>/<name>`` unless already qualified;
* deploy: ``create-if-not-exists`` topics are created non-partitioned
  (``partitions: 0``) or partitioned; ``deletion-mode: delete`` topics are deleted;
* consumer: subscription ``langstream-agent-<agentId>`` (``subscriptionName`` overrides),
  **Failover** subscription type (one active consumer per partition: replica data
  parallelism), initial position Earliest, ``commit`` = per-message acknowledge;
* schemas (``schema.py``): deploy registers a topic's ``valueSchema`` (KeyValue SEPARATED
  with a ``keySchema``) through the admin API; producers encode with the topic's schema
  (configured, registered, or inferred from the first record's types and then
  registered, like the Java client); consumers and readers decode with the topic's
  registered schema (``AUTO_CONSUME``), KeyValue messages into key + value;
* producer: headers as message properties (text);
* reader (gateways): latest / earliest / absolute; the offset token is a JSON map
  ``{partition-topic: messageId}`` so a reader resumes each partition after the last
  message it returned (``PulsarTopicReader`` keeps the same map).
The broker side can be a real Pulsar (``webSocketServiceEnabled=true``) or the in-tree
``topics/pulsar/standalone.py``.
"""
from __future__ import annotations

import base64
import itertools
import json
import logging
import threading
import time
from concurrent.futures import Future
from datetime import datetime
from typing import Any, Dict, List, Optional
from urllib.parse import quote, urlsplit

import requests

from ...api.record import Header, Record
from ...api.topics import (TopicAdmin, TopicConnectionsRuntime, TopicConnectionsRuntimeRegistry, TopicConsumer,
                           TopicOffsetPosition, TopicProducer, TopicReader, TopicReadResult)
from ...utils.wsclient import WebSocket, WebSocketClosed
from ..kafka import serialize
from .schema import TopicSchema, infer

log = logging.getLogger(__name__)


class PulsarRecord(Record):
    __slots__ = ("message_id", "partition_topic")

    def __init__(self, topic: str, d: Dict[str, Any], schema: Optional[TopicSchema] = None):
        payload = base64.b64decode(d.get("payload") or "")
        key: Any = d.get("key")
        if schema is not None:
            key, value = schema.decode_message(key, payload)
        else:
            try:
                value = payload.decode()
            except UnicodeDecodeError:
                value = payload
        props = d.get("properties") or {}
        super().__init__(key, value, topic, _publish_ms(d.get("publishTime")),
                         [Header(k, v) for k, v in props.items()])
        self.message_id = d["messageId"]
        self.partition_topic = topic


def _publish_ms(s: Any) -> Optional[int]:
    if s is None:
        return None
    if isinstance(s, (int, float)):
        return int(s)
    try:
        return int(datetime.fromisoformat(str(s).replace("Z", "+00:00")).timestamp() * 1000)
    except ValueError:
        return None


class PulsarConfig:
    def __init__(self, streaming_cluster):
        cfg = (streaming_cluster.configuration if streaming_cluster is not None else {}) or {}
        admin = cfg.get("admin") or {}
        service = cfg.get("service") or {}
        self.admin_url = str(admin.get("serviceUrl") or cfg.get("webServiceUrl") or "http://localhost:8080").rstrip("/")
        ws = service.get("webSocketUrl") or cfg.get("webSocketUrl")
        if not ws:
            u = urlsplit(self.admin_url)
            ws = ("wss" if u.scheme == "https" else "ws") + "://" + u.netloc
        self.ws_url = str(ws).rstrip("/")
        self.tenant = cfg.get("default-tenant") or "public"
        self.namespace = cfg.get("default-namespace") or "default"
        auth = cfg.get("authentication") or {}
        tok = auth.get("token") or (auth.get("authParams") if auth.get("authPlugin", "").endswith("AuthenticationToken")
                                    else None)
        if isinstance(tok, str) and tok.startswith("token:"):
            tok = tok[len("token:"):]
        self.headers = {"Authorization": f"Bearer {tok}"} if tok else {}

    def full(self, name: str) -> str:
        if "://" in name:
            return name
        if name.count("/") == 2:
            return "persistent://" + name
        return f"persistent://{self.tenant}/{self.namespace}/{name}"

    @staticmethod
    def rest_path(full: str) -> str:
        domain, rest = full.split("://", 1)
        return f"{domain}/" + "/".join(quote(p, safe="") for p in rest.split("/"))

    def ws(self, kind: str, full: str, suffix: str = "", query: Optional[Dict[str, Any]] = None) -> WebSocket:
        url = f"{self.ws_url}/ws/v2/{kind}/{self.rest_path(full)}{suffix}"
        if query:
            url += "?" + "&".join(f"{k}={quote(str(v), safe='')}" for k, v in query.items())
        return WebSocket(url, headers=self.headers)

    # ---------------------------------------------------------------- admin
    def admin(self, method: str, path: str, **kw) -> requests.Response:
        headers = {**self.headers, **kw.pop("headers", {})}
        return requests.request(method, f"{self.admin_url}/admin/v2/{path}", headers=headers, timeout=30, **kw)

    def partitions(self, full: str) -> int:
        r = self.admin("GET", self.rest_path(full) + "/partitions")
        return int(r.json().get("partitions", 0)) if r.ok else 0

    # ---------------------------------------------------------------- schemas
    @staticmethod
    def base_topic(full: str) -> str:
        """The partitioned topic a ``-partition-N`` topic belongs to (schemas live there)."""
        import re as _re
        return _re.sub(r"-partition-\d+$", "", full)

    def schema_path(self, full: str) -> str:
        _, rest = self.base_topic(full).split("://", 1)
        return "schemas/" + "/".join(quote(p, safe="") for p in rest.split("/")) + "/schema"

    def get_schema(self, full: str) -> Optional[TopicSchema]:
        r = self.admin("GET", self.schema_path(full))
        if r.status_code == 404:
            return None
        if not r.ok:
            raise RuntimeError(f"reading the schema of {full}: {r.status_code} {r.text}")
        return TopicSchema.from_rest(r.json())

    def post_schema(self, full: str, ts: TopicSchema) -> None:
        r = self.admin("POST", self.schema_path(full), json=ts.rest_payload())
        if r.status_code not in (200, 204):
            raise RuntimeError(f"registering the schema of {full}: {r.status_code} {r.text}")

    def topic_exists(self, full: str) -> bool:
        if self.partitions(full) > 0:
            return True
        domain, rest = full.split("://", 1)
        t, ns, _ = rest.split("/", 2)
        r = self.admin("GET", f"{domain}/{t}/{ns}")
        return r.ok and full in r.json()


class PulsarConsumer(TopicConsumer):
    def __init__(self, cfg: PulsarConfig, topic: str, subscription: str, sub_type: str = "Failover",
                 max_records: int = 500, poll_s: float = 1.0):
        self.cfg, self.topic = cfg, cfg.full(topic)
        self.subscription, self.sub_type = subscription, sub_type
        self.max_records, self.poll_s = max_records, poll_s
        self.ws: Optional[WebSocket] = None
        self._out = 0
        self.schema = _SchemaCache(cfg, self.topic)

    def start(self) -> None:
        self.schema.get()
        self.ws = self.cfg.ws("consumer", self.topic, "/" + quote(self.subscription, safe=""),
                              {"subscriptionType": self.sub_type, "subscriptionInitialPosition": "Earliest",
                               "receiverQueueSize": 1000})

    def close(self) -> None:
        if self.ws is not None:
            self.ws.close()

    def read(self) -> List[Record]:
        out: List[Record] = []
        timeout = self.poll_s
        while len(out) < self.max_records:
            m = self.ws.recv(timeout=timeout)
            if m is None:
                break
            d = json.loads(m[1])
            if "messageId" not in d:
                if d.get("result", "ok") != "ok":
                    raise RuntimeError(f"pulsar consumer error: {d}")
                continue
            out.append(PulsarRecord(self.topic, d, self.schema.get()))
            timeout = 0.001
        self._out += len(out)
        return out

    def commit(self, records: List[Record]) -> None:
        for r in records:
            if isinstance(r, PulsarRecord):
                self.ws.send_text(json.dumps({"messageId": r.message_id}))

    def get_total_out(self) -> int:
        return self._out

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic, "subscription": self.subscription, "type": self.sub_type}


class _SchemaCache:
    """A topic's registered schema for readers (AUTO_CONSUME): fetched at start and, while
    the topic has none, at most once a second (a producer may register one later)."""

    def __init__(self, cfg: PulsarConfig, topic: str):
        self.cfg, self.topic = cfg, topic
        self.schema: Optional[TopicSchema] = None
        self._last = 0.0

    def get(self) -> Optional[TopicSchema]:
        if self.schema is None and time.monotonic() - self._last > 1.0:
            self._last = time.monotonic()
            try:
                self.schema = self.cfg.get_schema(self.topic)
            except (requests.RequestException, RuntimeError) as e:
                log.warning("cannot read the schema of %s: %s", self.topic, e)
        return self.schema


class PulsarProducer(TopicProducer):
    def __init__(self, cfg: PulsarConfig, topic: str, schema: Optional[TopicSchema] = None):
        self.cfg, self.topic = cfg, cfg.full(topic)
        self.schema = schema          # configured (topic keySchema / valueSchema)
        self._schema_lock = threading.Lock()
        self.ws: Optional[WebSocket] = None
        self._pending: Dict[str, Future] = {}
        self._lock = threading.Lock()
        self._ctx = itertools.count()
        self._in = 0
        self._reader: Optional[threading.Thread] = None
        self._started = False

    def start(self) -> None:
        if self._started:
            return
        if self.schema is None:
            self.schema = self.cfg.get_schema(self.topic)
        elif self.cfg.get_schema(self.topic) is None:
            self.cfg.post_schema(self.topic, self.schema)      # the Java client registers on create
        self.ws = self.cfg.ws("producer", self.topic)
        self._reader = threading.Thread(target=self._receipts, name=f"pulsar-producer-{self.topic}", daemon=True)
        self._reader.start()
        self._started = True

    def _receipts(self) -> None:
        while True:
            try:
                m = self.ws.recv(timeout=None)
            except (WebSocketClosed, OSError) as e:
                with self._lock:
                    pend, self._pending = self._pending, {}
                for f in pend.values():
                    if not f.done():
                        f.set_exception(ConnectionError(f"pulsar producer closed: {e}"))
                return
            if m is None:
                continue
            d = json.loads(m[1])
            with self._lock:
                f = self._pending.pop(str(d.get("context")), None)
            if f is None:
                continue
            if d.get("result") == "ok":
                self._in += 1
                f.set_result(d.get("messageId"))
            else:
                f.set_exception(RuntimeError(f"pulsar send failed: {d.get('errorMsg') or d}"))

    def close(self) -> None:
        if self.ws is not None:
            self.ws.close()

    def write(self, record: Record) -> Future:
        if not self._started:
            self.start()
        f: Future = Future()
        ctx = str(next(self._ctx))
        try:
            if self.schema is None:
                with self._schema_lock:
                    if self.schema is None:
                        # no configured / registered schema: infer one from this record's
                        # types and register it (PulsarTopicProducer.write, BASE_SCHEMAS)
                        inferred = infer(record.key(), record.value())
                        existing = self.cfg.get_schema(self.topic)
                        if existing is None:
                            self.cfg.post_schema(self.topic, inferred)
                        self.schema = existing or inferred
            key, payload = self.schema.encode_message(record.key(), record.value())
        except Exception as e:  # noqa: BLE001 - a value the schema cannot carry
            f.set_exception(e)
            return f
        msg: Dict[str, Any] = {"payload": base64.b64encode(payload).decode(),
                               "properties": {h.key: (serialize(h.value) or b"").decode(errors="replace")
                                              for h in record.headers() if h.value is not None},
                               "context": ctx}
        if key is not None:
            msg["key"] = key
        with self._lock:
            self._pending[ctx] = f
        try:
            self.ws.send_text(json.dumps(msg))
        except (OSError, WebSocketClosed) as e:
            with self._lock:
                self._pending.pop(ctx, None)
            f.set_exception(e)
        return f

    def get_total_in(self) -> int:
        return self._in

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic}


class PulsarReader(TopicReader):
    """One WebSocket reader per partition; offset = JSON {partition-topic: messageId}."""

    def __init__(self, cfg: PulsarConfig, topic: str, position: TopicOffsetPosition, poll_s: float = 0.5):
        self.cfg, self.topic, self.position, self.poll_s = cfg, cfg.full(topic), position, poll_s
        self.readers: Dict[str, WebSocket] = {}
        self.ids: Dict[str, str] = {}
        self.schema = _SchemaCache(cfg, self.topic)

    def start(self) -> None:
        self.schema.get()
        n = self.cfg.partitions(self.topic)
        names = [f"{self.topic}-partition-{i}" for i in range(n)] if n > 0 else [self.topic]
        if self.position.position == "absolute" and self.position.offset:
            self.ids = {k: v for k, v in json.loads(self.position.offset.decode()).items()}
        for name in names:
            start = self.ids.get(name) or ("earliest" if self.position.position == "earliest" else "latest")
            self.readers[name] = self.cfg.ws("reader", name, "", {"messageId": start})

    def close(self) -> None:
        for w in self.readers.values():
            w.close()

    def read(self) -> TopicReadResult:
        out: List[Record] = []
        per = max(0.01, self.poll_s / max(1, len(self.readers)))
        for name, w in self.readers.items():
            timeout = per
            while True:
                m = w.recv(timeout=timeout)
                if m is None:
                    break
                d = json.loads(m[1])
                if "messageId" not in d:
                    continue
                out.append(PulsarRecord(name, d, self.schema.get()))
                self.ids[name] = d["messageId"]
                w.send_text(json.dumps({"messageId": d["messageId"]}))
                timeout = 0.001
        offset = json.dumps(self.ids, sort_keys=True).encode() if out else None
        return TopicReadResult(out, offset)


class PulsarTopicConnectionsRuntime(TopicConnectionsRuntime):
    def init(self, streaming_cluster) -> None:
        self.sc = streaming_cluster
        self.cfg = PulsarConfig(streaming_cluster)

    def deploy(self, plan) -> None:
        for t in plan.topics.values():
            if t.creation_mode != "create-if-not-exists":
                continue
            full = self.cfg.full(t.name)
            if self.cfg.topic_exists(full):
                log.info("pulsar topic %s already exists", full)
                continue
            if (t.partitions or 0) <= 0:
                r = self.cfg.admin("PUT", self.cfg.rest_path(full))
            else:
                r = self.cfg.admin("PUT", self.cfg.rest_path(full) + "/partitions", data=str(int(t.partitions)),
                                   headers={"Content-Type": "application/json"})
            if r.status_code not in (200, 204, 409):
                raise RuntimeError(f"creating pulsar topic {full}: {r.status_code} {r.text}")
        for t in plan.topics.values():
            # schema deploy (PulsarTopicConnectionsRuntimeProvider.java:256-289): only when
            # the topic has no schema yet
            ts = TopicSchema.from_definitions(_sd(t.definition.key_schema if t.definition else None),
                                              _sd(t.definition.value_schema if t.definition else None))
            if ts is None:
                continue
            full = self.cfg.full(t.name)
            if self.cfg.get_schema(full) is None:
                log.info("deploying schema %s for pulsar topic %s", ts.rest_payload()["type"], full)
                self.cfg.post_schema(full, ts)
            else:
                log.info("pulsar topic %s already has a schema, skipping", full)

    def delete(self, plan) -> None:
        for t in plan.topics.values():
            if t.deletion_mode != "delete":
                continue
            full = self.cfg.full(t.name)
            suffix = "/partitions" if self.cfg.partitions(full) > 0 else ""
            r = self.cfg.admin("DELETE", self.cfg.rest_path(full) + suffix)
            if r.status_code not in (200, 204, 404):
                raise RuntimeError(f"deleting pulsar topic {full}: {r.status_code} {r.text}")

    def create_consumer(self, agent_id, streaming_cluster, configuration) -> TopicConsumer:
        sub = configuration.get("subscriptionName") or f"langstream-agent-{agent_id}"
        return PulsarConsumer(self.cfg, configuration["topic"], sub,
                              str(configuration.get("subscriptionType", "Failover")),
                              int(configuration.get("max.poll.records", 500)),
                              float(configuration.get("poll.timeout.ms", 1000)) / 1000.0)

    def create_producer(self, agent_id, streaming_cluster, configuration) -> TopicProducer:
        return PulsarProducer(self.cfg, configuration["topic"],
                              TopicSchema.from_definitions(configuration.get("keySchema"),
                                                           configuration.get("valueSchema")))

    def create_reader(self, streaming_cluster, configuration, initial_position) -> TopicReader:
        return PulsarReader(self.cfg, configuration["topic"], initial_position,
                            float(configuration.get("poll.timeout.ms", 500)) / 1000.0)

    def create_topic_admin(self, agent_id, streaming_cluster, configuration) -> TopicAdmin:
        return TopicAdmin()


def _sd(s) -> Optional[Dict[str, Any]]:
    return None if s is None else {"type": s.type, "schema": s.schema, "name": s.name}


TopicConnectionsRuntimeRegistry.register("pulsar", PulsarTopicConnectionsRuntime)
