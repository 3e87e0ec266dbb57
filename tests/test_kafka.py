"""Kafka protocol, client and the in-tree single-node broker; a pipeline running on the
``kafka`` streaming type.

Mirrors the reference's Kafka runtime tests (KafkaConsumerTest out-of-order commits,
KafkaClusterRuntimeDockerTest topic creation, consumer-group DP) against the in-tree
broker instead of a Kafka container."""
import json
import threading
import time
import uuid

import pytest

from langstream_amd.topics.kafka import protocol as P
from langstream_amd.topics.kafka.broker import KafkaBroker
from langstream_amd.topics.kafka.client import GroupConsumer, KafkaClient, PartitionReader, Producer, range_assign


@pytest.fixture(scope="module")
def broker():
    b = KafkaBroker(default_partitions=1).start()
    yield b
    b.stop()


def test_varint_crc_murmur():
    for v in (0, 1, -1, 63, -64, 300, -300, 1 << 40, -(1 << 40)):
        enc = P.zigzag_varint(v)
        assert P.read_varint(enc, 0) == (v, len(enc))
    assert P.crc32c(b"123456789") == 0xE3069283          # CRC-32C check value
    assert P.murmur2(b"21") == -973932308                 # Kafka Utils.murmur2 test vector
    assert P.partition_for_key(b"key", 3) in range(3)


def test_batch_roundtrip():
    recs = [(b"k1", b"v1", [("h", b"x")], 1000), (None, b"v2", [], 1005), (b"k3", None, [("a", None)], 1010)]
    data = P.encode_batch(42, recs)
    out = list(P.decode_batches(data, verify_crc=True))
    assert [(o, ts, k, v, h) for o, ts, k, v, h in out] == [
        (42, 1000, b"k1", b"v1", [("h", b"x")]), (43, 1005, None, b"v2", []), (44, 1010, b"k3", None, [("a", None)])]
    assert list(P.decode_batches(data[:-3])) == []  # truncated batch ignored


def test_range_assignor():
    a = range_assign({"m1": ["t"], "m2": ["t"], "m3": ["t"]}, {"t": 7})
    assert a == {"m1": {"t": [0, 1, 2]}, "m2": {"t": [3, 4]}, "m3": {"t": [5, 6]}}


def test_produce_fetch_offsets(broker):
    c = KafkaClient(broker.bootstrap)
    t = "t-" + uuid.uuid4().hex[:6]
    assert c.create_topic(t, 3)
    assert not c.create_topic(t, 3)  # already exists
    p = Producer(c, t)
    for i in range(30):
        p.send(f"k{i % 5}".encode(), f"v{i}".encode(), [("i", str(i).encode())], 1000 + i)
    ends = c.list_offsets(t, -1)
    assert sum(ends.values()) == 30
    r = PartitionReader(c, t, start="earliest")
    got = r.read(100)
    assert len(got) == 30
    # keyed records: one key -> one partition
    parts = {}
    for part, off, ts, k, v, hs in got:
        parts.setdefault(k, set()).add(part)
    assert all(len(s) == 1 for s in parts.values())
    assert r.read(50) == []
    c.delete_topic(t)
    c.close()


def test_consumer_group_rebalance_and_ooo_commit(broker):
    t = "g-" + uuid.uuid4().hex[:6]
    admin = KafkaClient(broker.bootstrap)
    admin.create_topic(t, 4)
    prod = Producer(admin, t)
    for i in range(40):
        prod.send(None, f"m{i}".encode(), [], int(time.time() * 1000))
    group = "grp-" + uuid.uuid4().hex[:6]
    c1 = GroupConsumer(KafkaClient(broker.bootstrap), t, group, session_timeout_ms=3000)
    c1.start()
    assert c1.assigned == [0, 1, 2, 3]
    first = []
    while len(first) < 40:
        first += c1.poll(200)
    # out-of-order commit: ack offset 1 then 0 on partition 0 -> committed offset moves to 2 only after both
    p0 = sorted(r[1] for r in first if r[0] == 0)
    c1.commit([(0, p0[1])])
    assert c1.committed()[0] == 0
    c1.commit([(0, p0[0])])
    assert c1.committed()[0] == 2
    # second member joins -> rebalance splits the partitions
    c2 = GroupConsumer(KafkaClient(broker.bootstrap), t, group, session_timeout_ms=3000)
    th = threading.Thread(target=c2.start)
    th.start()
    deadline = time.time() + 15
    while time.time() < deadline and (c1._need_rejoin is False or not c2.assigned):
        c1.poll(100)
        if c2.assigned and sorted(c1.assigned + c2.assigned) == [0, 1, 2, 3] and not c1._need_rejoin:
            break
    th.join(15)
    assert sorted(c1.assigned + c2.assigned) == [0, 1, 2, 3]
    assert c1.assigned and c2.assigned
    # committed offsets survive the rebalance: partition 0's owner resumed from offset 2
    owner = c1 if 0 in c1.assigned else c2
    assert owner.committed()[0] == 2
    c1.close()
    c2.close()


def test_pipeline_on_kafka_runtime(broker):
    from langstream_amd.runtime.local import LocalApplicationRunner
    tin, tout = "in-" + uuid.uuid4().hex[:6], "out-" + uuid.uuid4().hex[:6]
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
    partitions: 2
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: c
    type: compute
    input: {tin}
    output: {tout}
    resources:
      parallelism: 2
    configuration:
      fields:
        - name: "value.n2"
          expression: "value.n * 2"
"""
    instance = f"""
instance:
  streamingCluster:
    type: kafka
    configuration:
      admin:
        bootstrap.servers: "{broker.bootstrap}"
"""
    app = LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, instance=instance).start(wait=20)
    try:
        for i in range(10):
            app.produce(tin, json.dumps({"n": i}), key=f"k{i}")
        out = app.consume(tout, 10, timeout=30)
        vals = sorted(json.loads(r.value())["n2"] for r in out)
        assert vals == [2 * i for i in range(10)]
    finally:
        app.stop(10)


def test_pipeline_replicas_as_pod_processes(tmp_path):
    """resources.parallelism: 2 with replica_processes: two agent-pod processes
    (runtime/pod.py) join one consumer group on a broker in its own process."""
    from langstream_amd.runtime.local import LocalApplicationRunner
    from langstream_amd.topics.kafka.broker import BrokerProcess
    b = BrokerProcess(partitions=2)
    tin, tout = "in-" + uuid.uuid4().hex[:6], "out-" + uuid.uuid4().hex[:6]
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
    partitions: 4
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: c
    id: twice
    type: compute
    input: {tin}
    output: {tout}
    resources:
      parallelism: 2
    configuration:
      fields:
        - name: "value.n2"
          expression: "value.n * 2"
"""
    instance = f"""
instance:
  streamingCluster:
    type: kafka
    configuration:
      admin:
        bootstrap.servers: "{b.bootstrap}"
"""
    app = LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, instance=instance, state_dir=str(tmp_path),
                                           replica_processes=True).start(wait=120)
    try:
        assert len(app.processes) == 2 and not app.runners
        assert all(p.proc.poll() is None for p in app.processes)
        for i in range(40):
            app.produce(tin, json.dumps({"n": i}), key=f"k{i}")
        out = app.consume(tout, 40, timeout=60)
        vals = sorted(json.loads(r.value())["n2"] for r in out)
        assert vals == [2 * i for i in range(40)]
        assert not app.errors
    finally:
        app.stop(20)
        b.stop()
    assert all(p.proc.returncode == 0 for p in app.processes)


def test_producer_write_many_one_future(broker):
    """``KafkaProducer.write_many``: one future for a group of records spanning several
    produce requests (> MAX_BATCH_RECORDS); order kept per partition; interleaves with
    single writes; a serialisation error queues nothing."""
    from langstream_amd.api.record import SimpleRecord
    from langstream_amd.topics.kafka import KafkaProducer
    c = KafkaClient(broker.bootstrap)
    t = "wm-" + uuid.uuid4().hex[:6]
    c.create_topic(t, 1)
    prod = KafkaProducer(broker.bootstrap, t)
    n = KafkaProducer.MAX_BATCH_RECORDS * 2 + 345
    single = prod.write(SimpleRecord.of("s0", "first"))
    f = prod.write_many([SimpleRecord.of(f"k{i}", json.dumps({"i": i, "pad": "x" * 300})) for i in range(n)])
    last = prod.write(SimpleRecord.of("s1", "last"))
    f.result(60)
    single.result(60)
    last.result(60)

    class Bad:
        def __init__(self):
            pass
    bad = prod.write_many([SimpleRecord.of("ok", "x"), SimpleRecord.of("bad", Bad())])
    with pytest.raises(Exception):
        bad.result(10)
    assert prod.write_many([]).result(1) is None
    prod.flush()
    got = []
    r = PartitionReader(c, t, start="earliest")
    while len(got) < n + 2:
        recs = r.read(500)
        assert recs
        got.extend(recs)
    vals = [v.decode() for _, _, _, _, v, _ in got]
    assert vals[0] == "first" and vals[-1] == "last" and len(got) == n + 2
    assert [json.loads(v)["i"] for v in vals[1:-1]] == list(range(n))
    prod.close()
    c.delete_topic(t)
    c.close()


def test_producer_write_many_reports_per_record_errors(broker):
    """the middle produce request of a write_many fails -> BatchWriteError
    whose errors name exactly that request's records; the others were delivered."""
    from langstream_amd.api.record import SimpleRecord
    from langstream_amd.api.topics import BatchWriteError
    from langstream_amd.topics.kafka import KafkaProducer
    c = KafkaClient(broker.bootstrap)
    t = "wmerr-" + uuid.uuid4().hex[:6]
    c.create_topic(t, 1)
    prod = KafkaProducer(broker.bootstrap, t)
    prod.MAX_BATCH_RECORDS = 2
    real = prod.p.send_many
    calls = {"n": 0}

    def flaky(items):
        calls["n"] += 1
        if calls["n"] == 2:
            raise ConnectionError("produce request failed")
        return real(items)
    prod.p.send_many = flaky
    with prod._cv:      # queue the whole group before the sender wakes
        f = prod.write_many([SimpleRecord.of(f"k{i}", f"v{i}") for i in range(6)])
    with pytest.raises(BatchWriteError) as ei:
        f.result(30)
    errs = ei.value.errors
    assert [e is not None for e in errs] == [False, False, True, True, False, False]
    one = prod.write(SimpleRecord.of("x", "y"))
    one.result(30)
    got = PartitionReader(c, t, start="earliest").read(100)
    assert [v.decode() for _, _, _, _, v, _ in got] == ["v0", "v1", "v4", "v5", "y"]
    prod.close()
    c.delete_topic(t)
