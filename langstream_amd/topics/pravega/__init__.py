"""``pravega`` streaming cluster.

Parity with the reference (``langstream-pravega/PravegaStreamingClusterRuntime.java:33-66``,
``PravegaTopic.java:23-106``, ``langstream-pravega-runtime/.../PravegaClientUtils.java:31-89``,
``PravegaTopicConnectionsRuntimeProvider.java:65-507``):

* configuration ``client.controller-uri`` (default ``tcp://localhost:9090``) and
  ``client.scope`` (default ``langstream``);
* deploy: create the scope if missing, then every ``create-if-not-exists`` topic as a
  stream with ``ScalingPolicy.fixed(partitions)`` segments (``partitions <= 0`` -> 1);
  ``creation-mode: none`` is left alone, any other mode is an error;
* delete: streams created by the app (``create-if-not-exists``) with
  ``deletion-mode: delete`` are sealed and deleted;
* consumer: reader group ``reader-group`` (default ``langstream-agent-<agentId>``) over
  ``<scope>/<topic>``, starting at the stream head; reads wait up to 1 s
  (``readNextEvent(1000)``); each replica is one reader of the group, so the group's
  segments are shared among the replicas (data parallelism);
* producer: the event is the JSON ``RecordWrapper {key, value, headers, timestamp}``;
  a non-null key (``toString()`` for strings / numbers, JSON otherwise) is the routing
  key, so equal keys land in the same segment and keep their order;
* reader (gateways): per-segment offsets, so unlike the reference (which ignores the
  initial position, ``TODO: recover from "initialPosition"``) ``latest`` / ``earliest``
  / ``absolute`` all work; the offset token is JSON ``{segment: next offset}``.

Transport: the framed protocol of ``wire.py`` against ``standalone.py`` (``langstream
pravega-standalone``).  A real Pravega cluster speaks its own gRPC controller API and
segment-store WireCommands, for which no client exists offline: wire compatibility with
a live Pravega is not claimed (parity unpinned); the adapter semantics above are what
``tests/test_pravega.py`` pins.
"""
from __future__ import annotations

import base64
import itertools
import json
import logging
import queue
import socket
import threading
import time
import uuid
from concurrent.futures import Future
from typing import Any, Dict, List, Optional, Tuple

from ...api.record import Header, Record
from ...api.topics import (TopicAdmin, TopicConnectionsRuntime, TopicConnectionsRuntimeRegistry, TopicConsumer,
                           TopicOffsetPosition, TopicProducer, TopicReader, TopicReadResult)
from ...utils import fastjson
from . import wire

log = logging.getLogger(__name__)


class PravegaClient:
    """One TCP connection; synchronous request/reply (callers serialise on a lock)."""

    def __init__(self, controller_uri: str, timeout: float = 30.0):
        self.uri = controller_uri
        self.host, self.port = wire.parse_uri(controller_uri)
        self.timeout = timeout
        self._lock = threading.Lock()
        self._rid = itertools.count(1)
        self._sock: Optional[socket.socket] = None

    def _connect(self) -> socket.socket:
        s = socket.create_connection((self.host, self.port), timeout=self.timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._sock = s
        self._call_locked(wire.HELLO, {"version": wire.PROTOCOL_VERSION})
        return s

    def _call_locked(self, kind: int, meta: Dict[str, Any], items=None, timeout: Optional[float] = None):
        rid = next(self._rid)
        meta = dict(meta, rid=rid)
        s = self._sock
        s.settimeout(timeout if timeout is not None else self.timeout)
        s.sendall(wire.encode(kind, meta, items))
        _, reply, data = wire.read_frame(s)
        if reply.get("rid") != rid:
            raise ConnectionError(f"pravega reply out of order ({reply.get('rid')} != {rid})")
        if not reply.get("ok"):
            raise RuntimeError(f"pravega: {reply.get('error')}")
        return reply, data

    def call(self, kind: int, meta: Dict[str, Any], items=None, timeout: Optional[float] = None):
        with self._lock:
            if self._sock is None:
                self._connect()
            try:
                return self._call_locked(kind, meta, items, timeout)
            except (ConnectionError, OSError):
                self.close_socket()
                raise

    def close_socket(self) -> None:
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass
            self._sock = None

    # -- StreamManager ------------------------------------------------------------
    def create_scope(self, scope: str) -> bool:
        return self.call(wire.CREATE_SCOPE, {"scope": scope})[0]["created"]

    def scope_exists(self, scope: str) -> bool:
        return self.call(wire.SCOPE_EXISTS, {"scope": scope})[0]["exists"]

    def create_stream(self, scope: str, stream: str, segments: int) -> bool:
        return self.call(wire.CREATE_STREAM, {"scope": scope, "stream": stream, "segments": segments})[0]["created"]

    def stream_info(self, scope: str, stream: str) -> Dict[str, Any]:
        return self.call(wire.STREAM_INFO, {"scope": scope, "stream": stream})[0]

    def stream_exists(self, scope: str, stream: str) -> bool:
        return self.stream_info(scope, stream)["exists"]

    def seal_stream(self, scope: str, stream: str) -> None:
        self.call(wire.SEAL_STREAM, {"scope": scope, "stream": stream})

    def delete_stream(self, scope: str, stream: str) -> None:
        self.call(wire.DELETE_STREAM, {"scope": scope, "stream": stream})

    # -- ReaderGroupManager -------------------------------------------------------
    def create_reader_group(self, scope: str, group: str, stream: str, start: Any = "head") -> bool:
        return self.call(wire.CREATE_READER_GROUP,
                         {"scope": scope, "group": group, "stream": stream, "start": start})[0]["created"]

    def delete_reader_group(self, scope: str, group: str) -> None:
        self.call(wire.DELETE_READER_GROUP, {"scope": scope, "group": group})


def _jsonable(v: Any) -> Any:
    if isinstance(v, bytes):
        try:
            return v.decode()
        except UnicodeDecodeError:
            return base64.b64encode(v).decode()  # Jackson writes byte[] as base64
    return v


def serialise_key(k: Any) -> Optional[str]:
    """``serialiseKey``: strings and numbers as text, anything else as JSON."""
    if k is None:
        return None
    if isinstance(k, bytes):
        return _jsonable(k)
    if isinstance(k, (str, int, float, bool)):
        return str(k).lower() if isinstance(k, bool) else str(k)
    return fastjson.dumps(k)


def _as_sent(r: Record, v: Any, i: int) -> Any:
    """A map an agent parsed from JSON text leaves as that text (compact JSON), as the
    reference's MutableRecord hands it back (convertMapToStringOrBytes) before the wrapper
    is written: PravegaRunnerDockerTest reads '{"name":"some name"}' back, not a map."""
    ref = getattr(r, "_source_ref", None)
    if isinstance(v, (dict, list)) and isinstance(ref, dict) and "json_origin" in ref:
        origin = ref["json_origin"][i]
        if origin is str:
            return fastjson.dumps(v)
        if origin is bytes:
            return fastjson.dumps(v).encode()
    return v


def serialise_value(r: Record) -> bytes:
    """``serialiseValue``: the JSON ``RecordWrapper``."""
    headers = {h.key: _jsonable(h.value) for h in r.headers()}
    return fastjson.dumps({"key": _jsonable(_as_sent(r, r.key(), 0)), "value": _jsonable(_as_sent(r, r.value(), 1)),
                           "headers": headers, "timestamp": r.timestamp()}).encode()


class PravegaRecord(Record):
    __slots__ = ("segment", "offset")

    def __init__(self, topic: str, data: bytes, segment: int, offset: int):
        w = json.loads(data)
        super().__init__(w.get("key"), w.get("value"), topic, w.get("timestamp"),
                         [Header(k, v) for k, v in (w.get("headers") or {}).items()])
        self.segment, self.offset = segment, offset


class PravegaConfig:
    def __init__(self, streaming_cluster):
        conf = dict(getattr(streaming_cluster, "configuration", None) or {})
        client = dict(conf.get("client") or {})
        self.controller_uri = str(client.get("controller-uri", "tcp://localhost:9090"))
        self.scope = str(client.get("scope", "langstream"))

    def client(self) -> PravegaClient:
        return PravegaClient(self.controller_uri)


class PravegaConsumer(TopicConsumer):
    """One reader of a reader group; the group's segments are split among its readers."""

    def __init__(self, cfg: PravegaConfig, topic: str, group: str, reader_id: str,
                 max_records: int = 500, poll_ms: int = 1000):
        self.cfg, self.topic, self.group, self.reader_id = cfg, topic, group, reader_id
        self.max_records, self.poll_ms = max_records, poll_ms
        self.client: Optional[PravegaClient] = None
        self._out = 0

    def start(self) -> None:
        self.client = self.cfg.client()
        self.client.create_reader_group(self.cfg.scope, self.group, self.topic, "head")
        self.client.call(wire.READER_ONLINE, {"scope": self.cfg.scope, "group": self.group, "reader": self.reader_id})

    def close(self) -> None:
        if self.client is not None:
            try:
                self.client.call(wire.READER_OFFLINE,
                                 {"scope": self.cfg.scope, "group": self.group, "reader": self.reader_id})
            except (RuntimeError, ConnectionError, OSError) as e:
                log.info("pravega reader %s offline: %s", self.reader_id, e)
            self.client.close_socket()

    def read(self) -> List[Record]:
        reply, data = self.client.call(
            wire.READ_NEXT, {"scope": self.cfg.scope, "group": self.group, "reader": self.reader_id,
                             "timeout_ms": self.poll_ms, "max": self.max_records},
            timeout=self.poll_ms / 1000.0 + 30.0)
        out = [PravegaRecord(self.topic, d, seg, off) for (seg, off), d in zip(reply["events"], data)]
        self._out += len(out)
        return out

    def commit(self, records: List[Record]) -> None:
        # Reader positions advance as events are read (the reference's commit is a no-op too).
        pass

    def get_total_out(self) -> int:
        return self._out

    def get_info(self) -> Dict[str, Any]:
        return {"readerId": self.reader_id, "readerGroup": self.group}


class PravegaProducer(TopicProducer):
    """EventStreamWriter: write() queues, a writer thread ships batched appends in order."""

    def __init__(self, cfg: PravegaConfig, topic: str, max_batch: int = 512):
        self.cfg, self.topic, self.max_batch = cfg, topic, max_batch
        self.client: Optional[PravegaClient] = None
        self._q: "queue.Queue[Optional[Tuple[Optional[str], bytes, Future]]]" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._in = 0

    def start(self) -> None:
        if self._thread is not None:
            return
        self.client = self.cfg.client()
        self._thread = threading.Thread(target=self._run, name=f"pravega-writer-{self.topic}", daemon=True)
        self._thread.start()

    def _run(self) -> None:
        stop = False
        while not stop:
            item = self._q.get()
            if item is None:
                break
            batch = [item]
            while len(batch) < self.max_batch:
                try:
                    nxt = self._q.get_nowait()
                except queue.Empty:
                    break
                if nxt is None:
                    stop = True
                    break
                batch.append(nxt)
            try:
                reply, _ = self.client.call(wire.APPEND, {"scope": self.cfg.scope, "stream": self.topic,
                                                          "keys": [k for k, _, _ in batch]},
                                            [d for _, d, _ in batch])
                for (_, _, f), placed in zip(batch, reply["placed"]):
                    f.set_result(placed)
            except Exception as e:  # noqa: BLE001 - surfaced through the futures
                for _, _, f in batch:
                    if not f.done():
                        f.set_exception(e)

    def close(self) -> None:
        if self._thread is not None:
            self._q.put(None)
            self._thread.join(timeout=30)
            self._thread = None
        if self.client is not None:
            self.client.close_socket()

    def write(self, record: Record) -> Future:
        f: Future = Future()
        try:
            self._q.put((serialise_key(record.key()), serialise_value(record), f))
            self._in += 1
        except (TypeError, ValueError) as e:
            f.set_exception(e)
        return f

    def get_native_producer(self):
        return self.client

    def get_total_in(self) -> int:
        return self._in

    def get_info(self) -> Dict[str, Any]:
        return {"stream": self.topic}


class PravegaReader(TopicReader):
    """Position-addressed reader; offset token = JSON {segment: next offset}."""

    def __init__(self, cfg: PravegaConfig, topic: str, position: TopicOffsetPosition, poll_s: float = 0.5,
                 max_records: int = 500):
        self.cfg, self.topic, self.position = cfg, topic, position
        self.poll_s, self.max_records = poll_s, max_records
        self.client: Optional[PravegaClient] = None
        self.offsets: Dict[int, int] = {}

    def start(self) -> None:
        self.client = self.cfg.client()
        info = self.client.stream_info(self.cfg.scope, self.topic)
        if not info["exists"]:
            raise RuntimeError(f"pravega stream {self.cfg.scope}/{self.topic} does not exist")
        n = info["segments"]
        if self.position.position == "absolute" and self.position.offset:
            saved = json.loads(self.position.offset.decode())
            self.offsets = {i: int(saved.get(str(i), 0)) for i in range(n)}
        elif self.position.position == "earliest":
            self.offsets = {i: 0 for i in range(n)}
        else:
            self.offsets = {i: int(t) for i, t in enumerate(info["tails"])}

    def close(self) -> None:
        if self.client is not None:
            self.client.close_socket()

    def read(self) -> TopicReadResult:
        out: List[Record] = []
        deadline = time.monotonic() + self.poll_s
        while True:
            for seg, off in self.offsets.items():
                reply, data = self.client.call(wire.READ_SEGMENT, {
                    "scope": self.cfg.scope, "stream": self.topic, "segment": seg, "offset": off,
                    "max": self.max_records})
                for i, d in enumerate(data):
                    out.append(PravegaRecord(self.topic, d, seg, off + i))
                self.offsets[seg] = off + len(data)
            if out or time.monotonic() >= deadline:
                break
            time.sleep(0.02)
        offset = json.dumps({str(k): v for k, v in self.offsets.items()}, sort_keys=True).encode() if out else None
        return TopicReadResult(out, offset)


class PravegaTopicAdmin(TopicAdmin):
    pass


class PravegaTopicConnectionsRuntime(TopicConnectionsRuntime):
    def init(self, streaming_cluster) -> None:
        self.sc = streaming_cluster
        self.cfg = PravegaConfig(streaming_cluster)

    def deploy(self, plan) -> None:
        c = self.cfg.client()
        try:
            if not c.scope_exists(self.cfg.scope):
                log.info("creating pravega scope %s", self.cfg.scope)
                c.create_scope(self.cfg.scope)
            for t in plan.topics.values():
                mode = t.creation_mode or "none"
                if mode == "create-if-not-exists":
                    if c.create_stream(self.cfg.scope, t.name, max(1, int(t.partitions or 0))):
                        log.info("created pravega stream %s/%s", self.cfg.scope, t.name)
                elif mode != "none":
                    raise ValueError(f"Unknown create mode {mode}")
        finally:
            c.close_socket()

    def delete(self, plan) -> None:
        c = self.cfg.client()
        try:
            for t in plan.topics.values():
                if t.creation_mode != "create-if-not-exists" or t.deletion_mode != "delete":
                    continue
                if not c.stream_exists(self.cfg.scope, t.name):
                    continue
                try:
                    c.seal_stream(self.cfg.scope, t.name)
                    c.delete_stream(self.cfg.scope, t.name)
                except RuntimeError as e:
                    log.info("pravega stream %s not deleted: %s", t.name, e)
        finally:
            c.close_socket()

    def create_consumer(self, agent_id, streaming_cluster, configuration) -> TopicConsumer:
        group = configuration.get("reader-group") or f"langstream-agent-{agent_id}"
        reader = f"{agent_id or 'reader'}-{uuid.uuid4().hex[:8]}"
        return PravegaConsumer(self.cfg, configuration["topic"], group, reader,
                               int(configuration.get("max.poll.records", 500)),
                               int(configuration.get("poll.timeout.ms", 1000)))

    def create_producer(self, agent_id, streaming_cluster, configuration) -> TopicProducer:
        return PravegaProducer(self.cfg, configuration["topic"])

    def create_reader(self, streaming_cluster, configuration, initial_position) -> TopicReader:
        return PravegaReader(self.cfg, configuration["topic"], initial_position,
                             float(configuration.get("poll.timeout.ms", 500)) / 1000.0)

    def create_topic_admin(self, agent_id, streaming_cluster, configuration) -> TopicAdmin:
        return PravegaTopicAdmin()


TopicConnectionsRuntimeRegistry.register("pravega", PravegaTopicConnectionsRuntime)
