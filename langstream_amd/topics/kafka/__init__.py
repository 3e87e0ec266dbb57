"""Kafka streaming runtime on the in-tree protocol client.

Parity:
* planner/runtime config (``KafkaStreamingClusterRuntime.java:41-88``,
  ``KafkaTopic.java:62-138``): topics get ``partitions`` (default 1) and the
  ``replication-factor`` option (default 1); consumers use
  ``group.id = langstream-agent-<agentId>`` (shared by every replica -> consumer-group
  data parallelism) and ``auto.offset.reset = earliest``; ``consumer.*`` / ``producer.*``
  / ``admin`` configuration pass through; ``bootstrap.servers`` from the streaming
  cluster's ``admin`` block (or top-level).
* consumer (``KafkaConsumerWrapper.java``): poll -> records; out-of-order commit
  tracking advancing only the contiguous prefix per partition; a failed commit is
  raised by the next read().
* producer / consumer serde (``KafkaProducerWrapper.java:57-270``, ``KafkaTopic.java:90-126``,
  ``serde.py``): topic ``keySchema`` / ``valueSchema`` force String / ByteArray / Avro
  (Confluent wire format, schemas registered in the schema registry); without a schema
  the Java type of each key / value / header picks the Kafka binary serializer
  (Boolean 1 B, Short / Integer / Long 2 / 4 / 8 B, Float / Double IEEE-754, UUID, JSON
  for maps and lists, Avro for AvroRecord values); consumers use StringDeserializer
  (bytes when not UTF-8) unless the schema says bytes / avro.
* schema registry (``KafkaTopicConnectionsRuntime.java:232-325``): on deploy, Avro key /
  value schemas of ``create-if-not-exists`` topics are registered under
  ``<topic>-key`` / ``<topic>-value`` at ``admin.schema.registry.url``.
* reader (``KafkaReaderWrapper.java``): assign-all, latest / earliest / absolute
  (``{partition: offset}`` JSON, base64 in the gateway API).
* admin (``KafkaTopicConnectionsRuntime.java:166-291``): create-if-not-exists topics
  on deploy, delete topics with deletion-mode ``delete``.
* security (``security.py``): TLS and SASL/PLAIN from the Java property names of the
  ``admin`` map (consumer / producer maps may override) -- the reference's
  ``examples/instances/astra.yaml`` shape; compressed record batches (gzip / snappy /
  lz4) decode on fetch, and ``producer.compression.type`` compresses produced batches.
"""
from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import Future
from typing import Any, Dict, List, Optional, Tuple

from ...api.record import Header, Record
from ...api.topics import (BatchWriteError, TopicAdmin, TopicConnectionsRuntime, TopicConnectionsRuntimeRegistry, TopicConsumer,
                           TopicOffsetPosition, TopicProducer, TopicReader, TopicReadResult, decode_offsets,
                           encode_offsets)
from . import codecs, serde
from ...utils import fastjson
from .client import GroupConsumer, KafkaClient, PartitionReader, Producer
from .security import SecurityConfig

log = logging.getLogger(__name__)


def serialize(v: Any) -> Optional[bytes]:
    """Reflection serialisation (no topic schema): serde.serialize_typed without Avro."""
    return serde.serialize_typed(v)


def deserialize(b: Optional[bytes]) -> Any:
    """StringDeserializer (bytes when the payload is not UTF-8)."""
    if b is None:
        return None
    try:
        return b.decode()
    except UnicodeDecodeError:
        return b


_STRING = serde.ValueDeserializer(serde.STRING_DESER, None)


class KafkaRecord(Record):
    __slots__ = ("topic", "partition", "offset")

    def __init__(self, topic: str, partition: int, offset: int, ts: int, key, value, headers,
                 kdes=None, vdes=None):
        super().__init__((kdes or deserialize)(key), (vdes or deserialize)(value), topic, ts,
                         [Header(k, deserialize(v)) for k, v in headers])
        self.topic, self.partition, self.offset = topic, partition, offset


def _serdes(configuration: Dict[str, Any], registry_cfgs, topic: str, producer: bool):
    """(key, value) serializers or deserializers for a consumer / producer configuration
    (the KafkaTopic configuration: key/value (de)serializer class + the topic schemas)."""
    ks, vs = configuration.get("keySchema"), configuration.get("valueSchema")
    registry = None
    if (ks and ks.get("type") == "avro") or (vs and vs.get("type") == "avro") or producer:
        registry = serde.SchemaRegistryClient.from_config(*registry_cfgs)
    if producer:
        kcls = configuration.get("key.serializer") or serde.serializer_for_schema(ks)
        vcls = configuration.get("value.serializer") or serde.serializer_for_schema(vs)
        auto = str(configuration.get("auto.register.schemas", "true")).lower() != "false"
        return (serde.ValueSerializer(kcls, serde.AvroSerializer(registry, topic, True, serde.topic_schema(ks), auto)),
                serde.ValueSerializer(vcls, serde.AvroSerializer(registry, topic, False, serde.topic_schema(vs), auto)))
    kcls = configuration.get("key.deserializer") or serde.deserializer_for_schema(ks)
    vcls = configuration.get("value.deserializer") or serde.deserializer_for_schema(vs)
    return serde.ValueDeserializer(kcls, registry), serde.ValueDeserializer(vcls, registry)


def _bootstrap(streaming_cluster) -> str:
    cfg = (streaming_cluster.configuration if streaming_cluster is not None else {}) or {}
    admin = cfg.get("admin") or {}
    bs = admin.get("bootstrap.servers") or cfg.get("bootstrap.servers") or cfg.get("bootstrapServers")
    if not bs:
        raise ValueError("kafka streaming cluster needs admin.bootstrap.servers")
    return str(bs)


class KafkaConsumer(TopicConsumer):
    def __init__(self, bootstrap: str, topic: str, group: str, reset: str, max_records: int, poll_ms: int,
                 security: Optional[SecurityConfig] = None, deserializers=None):
        self.client = KafkaClient(bootstrap, client_id=f"consumer-{group}", security=security)
        self.c = GroupConsumer(self.client, topic, group, reset, max_poll_records=max_records)
        self.topic, self.group, self.poll_ms = topic, group, poll_ms
        self.kdes, self.vdes = deserializers or (None, None)
        self._out = 0

    def start(self) -> None:
        self.c.start()

    def close(self) -> None:
        self.c.close()
        self.client.close()

    def read(self) -> List[Record]:
        recs = self.c.poll(self.poll_ms)
        kd, vd = self.kdes, self.vdes
        out = [KafkaRecord(self.topic, p, off, ts, k, v, hs, kd, vd) for p, off, ts, k, v, hs in recs]
        self._out += len(out)
        return out

    def commit(self, records: List[Record]) -> None:
        self.c.commit([(r.partition, r.offset) for r in records if isinstance(r, KafkaRecord)])

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic, "group": self.group, "member": self.c.member_id,
                "assignment": self.c.assigned, "committed": self.c.committed()}

    def get_total_out(self) -> int:
        return self._out


class _Group:
    """The future behind ``n`` queued records (one record for ``write``).  A failed
    ``write_many`` group fails with a ``BatchWriteError`` naming the records whose produce
    request failed: records of the batch acknowledged in another request are not
    retried, skipped or dead-lettered."""
    __slots__ = ("fut", "n", "left", "errs")

    def __init__(self, fut: Future, n: int, batch: bool = False):
        self.fut, self.n, self.left, self.errs = fut, (n if batch else 0), n, None

    def one_done(self, err, idx: int) -> None:
        # only the sender thread calls this: no lock needed
        if err is not None:
            if self.errs is None:
                self.errs = {}
            self.errs[idx] = err
        self.left -= 1
        if self.left == 0:
            if not self.errs:
                self.fut.set_result(None)
            elif self.n == 0:
                self.fut.set_exception(next(iter(self.errs.values())))
            else:
                self.fut.set_exception(BatchWriteError([self.errs.get(i) for i in range(self.n)]))


class KafkaProducer(TopicProducer):
    """Asynchronous, batching producer (the Kafka client's accumulator + sender thread,
    linger 0): ``write`` queues the record and returns a future; one sender thread drains
    everything queued so far into one produce request per partition (acks=all) and
    resolves the futures when the broker acknowledges.  Order per partition is the write
    order.  Writing one synchronous request per record capped an agent at one broker
    round trip per record (BASELINE config 2: ~500 records/s)."""

    MAX_BATCH_RECORDS = 1000
    MAX_BATCH_BYTES = 900 * 1024   # under the broker's default message.max.bytes (1 MiB)

    def __init__(self, bootstrap: str, topic: str, security: Optional[SecurityConfig] = None, codec: int = 0,
                 serializers=None):
        self.client = KafkaClient(bootstrap, client_id=f"producer-{topic}", security=security)
        self.kser, self.vser = serializers or (serialize, serialize)
        self.p = Producer(self.client, topic, codec=codec)
        self.topic = topic
        self._in = 0
        self._cv = threading.Condition()
        self._q: List[Tuple[tuple, "_Group", int, int]] = []   # (item, group, bytes, index in group)
        self._closed = False
        self._thread: Optional[threading.Thread] = None
        self._last: Optional[Future] = None

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()
        if self._thread is not None:
            self._thread.join(30)
        self.client.close()

    def _item(self, record: Record):
        hs = [(h.key, serialize(h.value)) for h in record.headers()]
        item = (self.kser(record.key()), self.vser(record.value()), hs, int(record.timestamp() or time.time() * 1000))
        size = len(item[0] or b"") + len(item[1] or b"") + sum(len(k) + len(v or b"") for k, v in hs) + 32
        return item, size

    def _enqueue(self, entries, f: Future) -> Future:
        with self._cv:
            if self._closed:
                f.set_exception(RuntimeError(f"producer for {self.topic} is closed"))
                return f
            self._q.extend(entries)
            self._last = f
            if self._thread is None:
                self._thread = threading.Thread(target=self._sender, name=f"kafka-producer-{self.topic}",
                                                daemon=True)
                self._thread.start()
            self._cv.notify()
        return f

    def write(self, record: Record) -> Future:
        f: Future = Future()
        try:
            item, size = self._item(record)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
            return f
        return self._enqueue([(item, _Group(f, 1), size, 0)], f)

    def write_many(self, records: List[Record]) -> Future:
        """Queue the records as one unit (same order, same batching into produce requests
        as ``write``) behind ONE future: resolved when the last of them is acknowledged,
        failed with a ``BatchWriteError`` (which records failed) if any produce request
        carrying them failed.  Per-record futures and their
        callbacks were a third of an embeddings agent's per-record host time."""
        f: Future = Future()
        if not records:
            f.set_result(None)
            return f
        try:
            items = [self._item(r) for r in records]
        except Exception as e:  # noqa: BLE001  (nothing queued: all or none)
            f.set_exception(e)
            return f
        g = _Group(f, len(items), batch=True)
        return self._enqueue([(it, g, size, i) for i, (it, size) in enumerate(items)], f)

    def _sender(self) -> None:
        while True:
            with self._cv:
                while not self._q and not self._closed:
                    self._cv.wait()
                if not self._q:
                    return
                n, nbytes = 0, 0
                while n < len(self._q) and n < self.MAX_BATCH_RECORDS and (n == 0 or nbytes + self._q[n][2] <= self.MAX_BATCH_BYTES):
                    nbytes += self._q[n][2]
                    n += 1
                batch, self._q = self._q[:n], self._q[n:]
            try:
                self.p.send_many([it for it, _, _, _ in batch])
                self._in += len(batch)
                err = None
            except Exception as e:  # noqa: BLE001
                err = e
            for _, g, _, i in batch:
                g.one_done(err, i)

    def flush(self, timeout: float = 30.0) -> None:
        """Wait until every record written so far is acknowledged (one sender thread
        resolves futures in write order, so the last one covers them all)."""
        with self._cv:
            last = self._last
        if last is not None:
            last.result(timeout)

    def get_total_in(self) -> int:
        return self._in

    def get_info(self) -> Dict[str, Any]:
        return {"topic": self.topic}


class KafkaReader(TopicReader):
    def __init__(self, bootstrap: str, topic: str, position: TopicOffsetPosition, poll_ms: int = 500,
                 security: Optional[SecurityConfig] = None, deserializers=None):
        self.client = KafkaClient(bootstrap, client_id=f"reader-{topic}", security=security)
        self.topic, self.position, self.poll_ms = topic, position, poll_ms
        self.kdes, self.vdes = deserializers or (None, None)
        self.r: Optional[PartitionReader] = None

    def start(self) -> None:
        if self.position.position == "absolute":
            self.r = PartitionReader(self.client, self.topic, offsets=decode_offsets(self.position.offset))
        else:
            self.r = PartitionReader(self.client, self.topic, start=self.position.position)

    def close(self) -> None:
        self.client.close()

    def read(self) -> TopicReadResult:
        recs = self.r.read(self.poll_ms)
        kd, vd = self.kdes, self.vdes
        out = [KafkaRecord(self.topic, p, off, ts, k, v, hs, kd, vd) for p, off, ts, k, v, hs in recs]
        return TopicReadResult(out, encode_offsets(dict(self.r.positions)))


class KafkaTopicConnectionsRuntime(TopicConnectionsRuntime):
    def init(self, streaming_cluster) -> None:
        self.sc = streaming_cluster
        self.bootstrap = _bootstrap(streaming_cluster)
        cfg = (streaming_cluster.configuration if streaming_cluster is not None else {}) or {}
        self.admin_cfg = cfg.get("admin") or {}
        self.consumer_cfg = cfg.get("consumer") or {}
        self.producer_cfg = cfg.get("producer") or {}
        self.security = SecurityConfig.from_config(self.admin_cfg)
        self.consumer_security = SecurityConfig.from_config(self.admin_cfg, self.consumer_cfg)
        self.producer_security = SecurityConfig.from_config(self.admin_cfg, self.producer_cfg)

    def deploy(self, plan) -> None:
        client = KafkaClient(self.bootstrap, client_id="langstream-admin", security=self.security)
        try:
            for t in plan.topics.values():
                if t.creation_mode == "create-if-not-exists":
                    rf = int((t.options or {}).get("replication-factor", 1))
                    client.create_topic(t.name, max(1, t.partitions), rf, t.config or {})
                    self._enforce_schema(t)
        finally:
            client.close()

    def _enforce_schema(self, t) -> None:
        """Register the topic's Avro key / value schemas (TopicNameStrategy subjects),
        KafkaTopicConnectionsRuntime.java:232-281; a missing registry url is an error
        only when a topic actually declares an Avro schema."""
        d = getattr(t, "definition", None)
        pairs = [(True, getattr(d, "key_schema", None)), (False, getattr(d, "value_schema", None))]
        pairs = [(k, s) for k, s in pairs if s is not None and s.type == "avro" and s.schema]
        if not pairs:
            return
        reg = serde.SchemaRegistryClient.from_config(self.admin_cfg)
        if reg is None:
            raise ValueError("Missing 'schema.registry.url' property in streaming cluster configuration admin section")
        for is_key, s in pairs:
            reg.register(serde.subject_name(t.name, is_key), s.schema)

    def delete(self, plan) -> None:
        client = KafkaClient(self.bootstrap, client_id="langstream-admin", security=self.security)
        try:
            for t in plan.topics.values():
                if t.deletion_mode == "delete":
                    client.delete_topic(t.name)
        finally:
            client.close()

    def create_consumer(self, agent_id, streaming_cluster, configuration) -> TopicConsumer:
        group = configuration.get("group.id") or f"langstream-agent-{agent_id}"
        return KafkaConsumer(self.bootstrap, configuration["topic"], group,
                             str(configuration.get("auto.offset.reset", "earliest")),
                             int(configuration.get("max.poll.records", 500)),
                             int(configuration.get("poll.timeout.ms", 500)), self.consumer_security,
                             _serdes(configuration, (self.admin_cfg, self.consumer_cfg), configuration["topic"], False))

    def create_producer(self, agent_id, streaming_cluster, configuration) -> TopicProducer:
        ctype = configuration.get("compression.type", self.producer_cfg.get("compression.type"))
        return KafkaProducer(self.bootstrap, configuration["topic"], self.producer_security, codecs.codec_of(ctype),
                             _serdes(configuration, (self.admin_cfg, self.producer_cfg), configuration["topic"], True))

    def create_reader(self, streaming_cluster, configuration, initial_position) -> TopicReader:
        return KafkaReader(self.bootstrap, configuration["topic"], initial_position,
                           int(configuration.get("poll.timeout.ms", 500)), self.consumer_security,
                           _serdes(configuration, (self.admin_cfg, self.consumer_cfg), configuration["topic"], False))

    def create_topic_admin(self, agent_id, streaming_cluster, configuration) -> TopicAdmin:
        return TopicAdmin()


TopicConnectionsRuntimeRegistry.register("kafka", KafkaTopicConnectionsRuntime)
