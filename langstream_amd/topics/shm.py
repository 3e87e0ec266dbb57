"""``shm`` streaming cluster: topics in a cross-process shared-memory log
(``native/shmlog.cpp``) -- the single-node broker that lets one process per GPU run
replicas of the same agent as members of one consumer group.

The reference scales agents only by replica data-parallelism: StatefulSet replicas
that share the Kafka consumer group ``langstream-agent-<agentId>``
(KAFKA/KafkaStreamingClusterRuntime.java:73-75, DEPL/agents/AgentResourcesFactory.java:
525-540).  On one MI355X node the replicas are processes (one per GPU, ``bench.py
--gpus N`` / torchrun), and this adapter gives them Kafka's semantics without a TCP
broker: partitions range-assigned over the live members of a group (re-assigned on
join / leave / process death), at-least-once redelivery from the committed offset,
out-of-order acks with a contiguous committed prefix, and group-less readers at
earliest / latest / absolute offsets for gateways.

Records cross the process boundary as msgpack ``(key, value, headers, timestamp)``;
map / list values are JSON-encoded first, as the Kafka JSON serializer does
(KRT/KafkaProducerWrapper.java:58-270).

Configuration (``instance.yaml`` ``streamingCluster.configuration``):
  name             log name; processes using the same name share topics (default
                   ``default``; ``$LANGSTREAM_SHM_NAME`` overrides, so a launcher can
                   give every job its own log)
  path             explicit file path (default ``/dev/shm/langstream-<name>``, or the
                   temp dir when /dev/shm is too small)
  size-mb          arena size (default 2048; sparse: pages are committed on use)
  block-kb         block size = max record size (default 4096)
  retention-messages  per-partition cap (default 0: bounded by the arena, oldest
                   fully-committed blocks recycled first)
"""
from __future__ import annotations

import atexit
import itertools
import logging
import os
import tempfile
import threading
import time
import uuid
from concurrent.futures import Future
from typing import Any, Dict, List, Optional

import msgpack

from ..api.record import Header, Record
from ..api.topics import (TopicAdmin, TopicConnectionsRuntime, TopicConnectionsRuntimeRegistry, TopicConsumer,
                          TopicOffsetPosition, TopicProducer, TopicReader, TopicReadResult, decode_offsets,
                          encode_offsets)
from ..native import lib
from .memory import _key_hash, serialize_value

log = logging.getLogger(__name__)

_logs: Dict[str, Any] = {}
_lock = threading.Lock()
_gate_registered = False


def _close_gate() -> None:
    """atexit: wake readers parked in the native log before interpreter finalization."""
    native = lib()
    native.shmlog_close_gate()
    deadline = time.monotonic() + 2.0
    while native.shmlog_waiters() > 0 and time.monotonic() < deadline:
        time.sleep(0.005)


def default_path(name: str, size: int) -> str:
    base = "/dev/shm"
    try:
        st = os.statvfs(base)
        if st.f_bavail * st.f_frsize < size:
            base = tempfile.gettempdir()
    except OSError:
        base = tempfile.gettempdir()
    return os.path.join(base, f"langstream-{name}")


def shmlog(name: str = "default", path: Optional[str] = None, size_mb: int = 2048, block_kb: int = 4096):
    """Open (creating on first use) the shared log ``name`` in this process."""
    global _gate_registered
    size = int(size_mb) << 20
    path = path or default_path(name, size)
    with _lock:
        m = _logs.get(path)
        if m is None:
            if not _gate_registered:
                atexit.register(_close_gate)
                _gate_registered = True
            m = lib().ShmLog(path, size, int(block_kb) << 10)
            _logs[path] = m
        return m


def unlink_shmlog(name: str = "default", path: Optional[str] = None, size_mb: int = 2048) -> None:
    """Remove the backing file (processes that mapped it keep their mapping)."""
    path = path or default_path(name, int(size_mb) << 20)
    with _lock:
        _logs.pop(path, None)
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass


def _pack(record: Record) -> bytes:
    hs = [(h.key, serialize_value(h.value)) for h in record.headers()]
    return msgpack.packb((record.key(), serialize_value(record.value()), hs,
                          record.timestamp() or int(time.time() * 1000)), use_bin_type=True)


class ShmRecord(Record):
    __slots__ = ("partition", "offset", "topic")

    def __init__(self, topic: str, partition: int, offset: int, data: bytes):
        key, value, headers, ts = msgpack.unpackb(data, raw=False, use_list=False)
        super().__init__(key, value, topic, ts, tuple(Header(k, v) for k, v in headers))
        self.topic = topic
        self.partition = partition
        self.offset = offset


class ShmConsumer(TopicConsumer):
    def __init__(self, log_, topic: str, group: str, max_records: int = 500, poll_ms: float = 200.0):
        self.log = log_
        self.topic = topic
        self.group = group
        self.member = f"{os.getpid()}-{uuid.uuid4().hex[:12]}"
        self.max_records = max_records
        self.poll_ms = poll_ms
        self._c = None
        self._out = 0

    def start(self) -> None:
        if not self.log.has_topic(self.topic):
            self.log.create_topic(self.topic, 1, 0)
        self._c = lib().ShmConsumer(self.log, self.topic, self.group, self.member)
        self._c.start()

    def close(self) -> None:
        if self._c is not None:
            self._c.close()
            self._c = None

    def read(self) -> List[Record]:
        c = self._c
        if c is None:
            return []
        out = [ShmRecord(self.topic, p, off, data) for p, off, data in c.poll(self.max_records, self.poll_ms)]
        self._out += len(out)
        return out

    def commit(self, records: List[Record]) -> None:
        offs = [(r.partition, r.offset) for r in records if isinstance(r, ShmRecord)]
        if offs and self._c is not None:
            self._c.ack(offs)

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic, "group": self.group, "member": self.member,
                "assignment": self._c.assignment() if self._c else [],
                "committed": self.log.committed(self.topic, self.group), "lag": self.log.lag(self.topic, self.group)}

    def get_total_out(self) -> int:
        return self._out


class ShmProducer(TopicProducer):
    _rr = itertools.count()

    def __init__(self, log_, topic: str, timeout_ms: float = 30000.0):
        self.log = log_
        self.topic = topic
        self.timeout_ms = timeout_ms
        self._in = 0

    def start(self) -> None:
        if not self.log.has_topic(self.topic):
            self.log.create_topic(self.topic, 1, 0)

    def write(self, record: Record) -> Future:
        f: Future = Future()
        try:
            kh = _key_hash(record.key())
            part = -1 if kh >= 0 else next(self._rr)
            self.log.append(self.topic, _pack(record), max(kh, 0), part, self.timeout_ms)
            self._in += 1
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def get_total_in(self) -> int:
        return self._in

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic}


class ShmReader(TopicReader):
    def __init__(self, log_, topic: str, position: TopicOffsetPosition, poll_ms: float = 200.0):
        self.log = log_
        self.topic = topic
        self.position = position
        self.poll_ms = poll_ms
        self._r = None

    def start(self) -> None:
        if not self.log.has_topic(self.topic):
            self.log.create_topic(self.topic, 1, 0)
        if self.position.position == "earliest":
            pos = list(self.log.begin_offsets(self.topic))
        elif self.position.position == "latest":
            pos = list(self.log.end_offsets(self.topic))
        else:
            d = decode_offsets(self.position.offset)
            pos = [d.get(p, 0) for p in range(self.log.partitions(self.topic))]
        self._r = lib().ShmReader(self.log, self.topic, pos)

    def read(self) -> TopicReadResult:
        recs = self._r.read(500, self.poll_ms)
        out = [ShmRecord(self.topic, p, off, data) for p, off, data in recs]
        return TopicReadResult(out, encode_offsets(dict(enumerate(self._r.positions()))))


class ShmTopicConnectionsRuntime(TopicConnectionsRuntime):
    def init(self, streaming_cluster) -> None:
        cfg = (streaming_cluster.configuration if streaming_cluster is not None else {}) or {}
        name = os.environ.get("LANGSTREAM_SHM_NAME") or str(cfg.get("name", "default"))
        self.log = shmlog(name, cfg.get("path"), int(cfg.get("size-mb", 2048)), int(cfg.get("block-kb", 4096)))
        self.retention = int(cfg.get("retention-messages", 0))

    def deploy(self, plan) -> None:
        for t in plan.topics.values():
            if t.creation_mode == "create-if-not-exists" and not self.log.has_topic(t.name):
                self.log.create_topic(t.name, max(1, t.partitions), self.retention)

    def delete(self, plan) -> None:
        for t in plan.topics.values():
            if t.deletion_mode == "delete":
                self.log.delete_topic(t.name)

    @staticmethod
    def _topic(cfg: Dict[str, Any]) -> str:
        t = cfg.get("topic")
        if not t:
            raise ValueError("topic is required")
        return t

    def create_consumer(self, agent_id, streaming_cluster, configuration) -> TopicConsumer:
        group = configuration.get("group.id") or f"langstream-agent-{agent_id}"
        return ShmConsumer(self.log, self._topic(configuration), group,
                           int(configuration.get("max.poll.records", 500)),
                           float(configuration.get("poll.timeout.ms", 200)))

    def create_producer(self, agent_id, streaming_cluster, configuration) -> TopicProducer:
        return ShmProducer(self.log, self._topic(configuration))

    def create_reader(self, streaming_cluster, configuration, initial_position) -> TopicReader:
        return ShmReader(self.log, self._topic(configuration), initial_position,
                         float(configuration.get("poll.timeout.ms", 200)))

    def create_topic_admin(self, agent_id, streaming_cluster, configuration) -> TopicAdmin:
        return TopicAdmin()


TopicConnectionsRuntimeRegistry.register("shm", ShmTopicConnectionsRuntime)
