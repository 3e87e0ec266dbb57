"""``memory`` streaming cluster: topics on the native in-process partitioned log
(``native/memlog.cpp``).

Semantics mirror the Kafka adapter of the reference (KAFKA/KafkaStreamingClusterRuntime.java:41-88,
KRT/KafkaConsumerWrapper.java, KafkaProducerWrapper.java, KafkaReaderWrapper.java):
* consumer group ``langstream-agent-<agentId>`` shared by every replica of an agent
  (replica data-parallelism over partitions), at-least-once with out-of-order acks and
  a contiguous-prefix committed offset;
* producers serialise map/list values to JSON (like the Kafka JSON serializer) and
  partition by key hash (round-robin without a key);
* readers (gateways) start at latest / earliest / an absolute per-partition offset
  and return a resumable offset token.
One log instance per ``configuration.name`` (default ``default``) per process.
"""
from __future__ import annotations

import itertools
import atexit
import logging
import threading
import time
import uuid
import zlib
from concurrent.futures import Future
from typing import Any, Dict, List, Optional

from ..api.record import Header, Record
from ..api.topics import (TopicAdmin, TopicConnectionsRuntime, TopicConnectionsRuntimeRegistry, TopicConsumer,
                          TopicOffsetPosition, TopicProducer, TopicReader, TopicReadResult, decode_offsets,
                          encode_offsets)
from ..native import lib
from ..utils import fastjson

log = logging.getLogger(__name__)

_logs: Dict[str, Any] = {}
_logs_lock = threading.Lock()


def _close_gate() -> None:
    """atexit: let readers blocked in the native log leave it before finalization."""
    native = lib()
    native.memlog_close_gate()
    deadline = time.monotonic() + 2.0
    while native.memlog_waiters() > 0 and time.monotonic() < deadline:
        time.sleep(0.005)


def memlog(name: str = "default"):
    with _logs_lock:
        m = _logs.get(name)
        if m is None:
            if not _logs:
                atexit.register(_close_gate)
            m = lib().MemLog()
            _logs[name] = m
        return m


def reset_memlogs() -> None:
    with _logs_lock:
        _logs.clear()


def _key_hash(key: Any) -> int:
    if key is None:
        return -1
    b = key if isinstance(key, bytes) else str(key).encode()
    return zlib.crc32(b)


def serialize_value(v: Any) -> Any:
    if isinstance(v, (dict, list)):
        return fastjson.dumps(v)
    return v


class MemRecord(Record):
    __slots__ = ("partition", "offset", "topic")

    def __init__(self, topic: str, partition: int, offset: int, payload: tuple):
        key, value, headers, ts = payload
        super().__init__(key, value, topic, ts, headers)
        self.topic = topic
        self.partition = partition
        self.offset = offset


class MemoryConsumer(TopicConsumer):
    def __init__(self, log_, topic: str, group: str, max_records: int = 500, poll_ms: float = 200.0):
        self.log = log_
        self.topic = topic
        self.group = group
        self.member = f"{group}-{uuid.uuid4().hex[:8]}"
        self.max_records = max_records
        self.poll_ms = poll_ms
        self._out = 0
        self._started = False

    def start(self) -> None:
        if not self.log.has_topic(self.topic):
            self.log.create_topic(self.topic, 1, 0)
        self.log.join(self.topic, self.group, self.member)
        self._started = True

    def close(self) -> None:
        if self._started:
            self.log.leave(self.topic, self.group, self.member)
            self._started = False

    def read(self) -> List[Record]:
        out = []
        for p, off, payload in self.log.poll(self.topic, self.group, self.member, self.max_records, self.poll_ms):
            out.append(MemRecord(self.topic, p, off, payload))
        self._out += len(out)
        return out

    def commit(self, records: List[Record]) -> None:
        offs = [(r.partition, r.offset) for r in records if isinstance(r, MemRecord)]
        if offs:
            self.log.ack(self.topic, self.group, offs)

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic, "group": self.group, "member": self.member,
                "assignment": self.log.assignment(self.topic, self.group, self.member),
                "committed": self.log.committed(self.topic, self.group), "lag": self.log.lag(self.topic, self.group)}

    def get_total_out(self) -> int:
        return self._out


class MemoryProducer(TopicProducer):
    _rr = itertools.count()

    def __init__(self, log_, topic: str):
        self.log = log_
        self.topic = topic
        self._in = 0

    def start(self) -> None:
        if not self.log.has_topic(self.topic):
            self.log.create_topic(self.topic, 1, 0)

    def write(self, record: Record) -> Future:
        f: Future = Future()
        try:
            payload = (record.key(), serialize_value(record.value()),
                       tuple(Header(h.key, serialize_value(h.value)) for h in record.headers()),
                       record.timestamp() or int(time.time() * 1000))
            kh = _key_hash(record.key())
            part = -1 if kh >= 0 else next(self._rr)
            self.log.append(self.topic, payload, max(kh, 0), part)
            self._in += 1
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def get_total_in(self) -> int:
        return self._in

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic}


class MemoryReader(TopicReader):
    def __init__(self, log_, topic: str, position: TopicOffsetPosition, poll_ms: float = 200.0):
        self.log = log_
        self.topic = topic
        self.position = position
        self.poll_ms = poll_ms
        self.positions: List[int] = []

    def start(self) -> None:
        if not self.log.has_topic(self.topic):
            self.log.create_topic(self.topic, 1, 0)
        if self.position.position == "earliest":
            self.positions = list(self.log.begin_offsets(self.topic))
        elif self.position.position == "latest":
            self.positions = list(self.log.end_offsets(self.topic))
        else:
            d = decode_offsets(self.position.offset)
            n = self.log.partitions(self.topic)
            self.positions = [d.get(p, 0) for p in range(n)]

    def read(self) -> TopicReadResult:
        recs, self.positions = self.log.read_from(self.topic, self.positions, 500, self.poll_ms)
        out = [MemRecord(self.topic, p, off, payload) for p, off, payload in recs]
        return TopicReadResult(out, encode_offsets(dict(enumerate(self.positions))))


class MemoryTopicConnectionsRuntime(TopicConnectionsRuntime):
    def init(self, streaming_cluster) -> None:
        cfg = (streaming_cluster.configuration if streaming_cluster is not None else {}) or {}
        self.log = memlog(str(cfg.get("name", "default")))
        self.retention = int(cfg.get("retention-messages", 0))

    def deploy(self, plan) -> None:
        for t in plan.topics.values():
            if t.creation_mode == "create-if-not-exists" and not self.log.has_topic(t.name):
                self.log.create_topic(t.name, max(1, t.partitions), self.retention)

    def delete(self, plan) -> None:
        for t in plan.topics.values():
            if t.deletion_mode == "delete":
                self.log.delete_topic(t.name)

    def _topic(self, cfg: Dict[str, Any]) -> str:
        t = cfg.get("topic")
        if not t:
            raise ValueError("topic is required")
        return t

    def create_consumer(self, agent_id, streaming_cluster, configuration) -> TopicConsumer:
        group = configuration.get("group.id") or f"langstream-agent-{agent_id}"
        return MemoryConsumer(self.log, self._topic(configuration), group,
                              int(configuration.get("max.poll.records", 500)),
                              float(configuration.get("poll.timeout.ms", 200)))

    def create_producer(self, agent_id, streaming_cluster, configuration) -> TopicProducer:
        return MemoryProducer(self.log, self._topic(configuration))

    def create_reader(self, streaming_cluster, configuration, initial_position) -> TopicReader:
        return MemoryReader(self.log, self._topic(configuration), initial_position,
                            float(configuration.get("poll.timeout.ms", 200)))

    def create_topic_admin(self, agent_id, streaming_cluster, configuration) -> TopicAdmin:
        return TopicAdmin()


class NoopTopicConnectionsRuntime(TopicConnectionsRuntime):
    """``noop`` streaming type: planning only (CORE/noop/*)."""

    def create_consumer(self, agent_id, streaming_cluster, configuration):
        raise ValueError("noop streaming cluster cannot create consumers")

    def create_producer(self, agent_id, streaming_cluster, configuration):
        raise ValueError("noop streaming cluster cannot create producers")

    def create_reader(self, streaming_cluster, configuration, initial_position):
        raise ValueError("noop streaming cluster cannot create readers")


TopicConnectionsRuntimeRegistry.register("memory", MemoryTopicConnectionsRuntime)
TopicConnectionsRuntimeRegistry.register("noop", NoopTopicConnectionsRuntime)
