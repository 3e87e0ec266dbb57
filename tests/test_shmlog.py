"""Cross-process shared-memory topic log (``shm`` streaming type): consumer-group
semantics across OS processes (the single-node broker behind multi-GPU replica DP).

Parity: the Kafka consumer-group behaviour the reference's replicas rely on
(KAFKA/KafkaStreamingClusterRuntime.java:73-75, KRT/KafkaConsumerWrapper.java:70-277):
disjoint partition ownership, at-least-once redelivery from the committed offset after
a rebalance, contiguous-prefix commits with out-of-order acks."""
import multiprocessing as mp
import os
import time
import uuid

import pytest

from langstream_amd.api.model import StreamingCluster
from langstream_amd.api.record import Header, SimpleRecord
from langstream_amd.api.topics import TopicConnectionsRuntimeRegistry, TopicOffsetPosition
from langstream_amd.native import lib
from langstream_amd.topics.shm import ShmTopicConnectionsRuntime, shmlog, unlink_shmlog


@pytest.fixture
def logname():
    name = f"t-{uuid.uuid4().hex[:10]}"
    yield name
    unlink_shmlog(name, size_mb=64)


def _rt(name):
    rt = ShmTopicConnectionsRuntime()
    rt.init(StreamingCluster("shm", {"name": name, "size-mb": 64, "block-kb": 64}))
    return rt


def test_roundtrip_types_headers_and_reader_positions(logname):
    rt = _rt(logname)
    rt.log.create_topic("t", 3, 0)
    p = rt.create_producer("a", None, {"topic": "t"})
    p.start()
    vals = [{"a": 1, "b": [1, 2]}, "text", b"\x00\x01", 42, 3.5, None, True]
    for i, v in enumerate(vals):
        p.write(SimpleRecord.of(f"k{i}", v, [Header("h", "x"), Header("n", 7)])).result(5)
    rd = rt.create_reader(None, {"topic": "t"}, TopicOffsetPosition.EARLIEST)
    rd.start()
    got, tok = [], None
    deadline = time.time() + 5
    while len(got) < len(vals) and time.time() < deadline:
        res = rd.read()
        got += res.records
        tok = res.offset
    by_key = {r.key(): r for r in got}
    assert by_key["k0"].value() == '{"a":1,"b":[1,2]}'  # maps are JSON-encoded as on Kafka (compact)
    assert by_key["k2"].value() == b"\x00\x01" and by_key["k3"].value() == 42 and by_key["k5"].value() is None
    assert by_key["k1"].header_value("n") == 7
    # resume from the returned absolute position: only new records
    p.write(SimpleRecord.of("late", "v")).result(5)
    rd2 = rt.create_reader(None, {"topic": "t"}, TopicOffsetPosition.absolute(tok))
    rd2.start()
    assert [r.key() for r in rd2.read().records] == ["late"]
    latest = rt.create_reader(None, {"topic": "t"}, TopicOffsetPosition.LATEST)
    latest.start()
    assert latest.read().records == []


def test_group_out_of_order_ack_and_redelivery(logname):
    rt = _rt(logname)
    rt.log.create_topic("in", 1, 0)
    p = rt.create_producer("a", None, {"topic": "in"})
    for i in range(5):
        p.write(SimpleRecord.of(None, i)).result(5)
    c = rt.create_consumer("ag", None, {"topic": "in"})
    c.start()
    recs = c.read()
    assert [r.value() for r in recs] == [0, 1, 2, 3, 4]
    c.commit([recs[0], recs[2], recs[3]])           # 1 outstanding -> committed = 1
    assert rt.log.committed("in", "langstream-agent-ag") == [1]
    c.close()
    c2 = rt.create_consumer("ag", None, {"topic": "in"})
    c2.start()
    assert [r.value() for r in c2.read()] == [1, 2, 3, 4]   # at-least-once from committed


def test_blocks_recycle_only_after_commit(logname):
    rt = _rt(logname)          # 64 MiB arena of 64 KiB blocks
    rt.log.create_topic("big", 1, 0)
    c = rt.create_consumer("ag", None, {"topic": "big", "max.poll.records": 100000})
    c.start()
    prod = rt.create_producer("a", None, {"topic": "big"})
    blob = "x" * 30000
    n = 0
    for _ in range(6):       # 6 x 1500 x 30 KB = 270 MB through a 64 MB arena
        for _ in range(1500):
            prod.write(SimpleRecord.of(None, blob)).result(5)
            n += 1
        got = c.read()
        while got:
            c.commit(got)
            got = c.read()
    assert rt.log.committed("big", "langstream-agent-ag") == [n]
    # committed blocks were recycled (eviction is lazy: only when the arena is full)
    assert rt.log.begin_offsets("big")[0] > 0


def _member(name, q, go, n_expected):
    from langstream_amd.topics.shm import ShmTopicConnectionsRuntime
    rt = ShmTopicConnectionsRuntime()
    rt.init(StreamingCluster("shm", {"name": name, "size-mb": 64, "block-kb": 64}))
    c = rt.create_consumer("ag", None, {"topic": "work", "poll.timeout.ms": 50})
    c.start()
    go.wait(30)
    seen = []
    idle = 0
    while idle < 20:
        recs = c.read()
        if not recs:
            idle += 1
            continue
        idle = 0
        seen += [(r.partition, r.value()) for r in recs]
        c.commit(recs)
    q.put((os.getpid(), seen))
    c.close()


def test_consumer_group_across_processes_disjoint_partitions(logname):
    rt = _rt(logname)
    rt.log.create_topic("work", 4, 0)
    ctx = mp.get_context("spawn")
    q, go = ctx.Queue(), ctx.Event()
    procs = [ctx.Process(target=_member, args=(logname, q, go, 200)) for _ in range(2)]
    for pr in procs:
        pr.start()
    deadline = time.time() + 60
    while time.time() < deadline and rt.log.group_members("work", "langstream-agent-ag") < 2:
        time.sleep(0.1)
    prod = rt.create_producer("a", None, {"topic": "work"})
    for i in range(200):
        prod.write(SimpleRecord.of(f"k{i}", i)).result(5)
    go.set()
    outs = [q.get(timeout=60) for _ in procs]
    for pr in procs:
        pr.join(30)
    a, b = outs[0][1], outs[1][1]
    assert sorted(v for _, v in a + b) == list(range(200))     # exactly once, nothing lost
    pa, pb = {p for p, _ in a}, {p for p, _ in b}
    assert pa and pb and not (pa & pb)                           # disjoint partitions
    assert rt.log.committed("work", "langstream-agent-ag") == rt.log.end_offsets("work")


def _dying_member(name, ready):
    from langstream_amd.topics.shm import ShmTopicConnectionsRuntime
    rt = ShmTopicConnectionsRuntime()
    rt.init(StreamingCluster("shm", {"name": name, "size-mb": 64, "block-kb": 64}))
    c = rt.create_consumer("ag", None, {"topic": "work"})
    c.start()
    c.read()          # take records, never ack, then die without leaving the group
    ready.set()
    time.sleep(0.5)
    os._exit(0)


def test_dead_member_partitions_are_reassigned_and_redelivered(logname):
    rt = _rt(logname)
    rt.log.create_topic("work", 2, 0)
    prod = rt.create_producer("a", None, {"topic": "work"})
    for i in range(10):
        prod.write(SimpleRecord.of(f"k{i}", i)).result(5)
    ctx = mp.get_context("spawn")
    ready = ctx.Event()
    pr = ctx.Process(target=_dying_member, args=(logname, ready))
    pr.start()
    assert ready.wait(60)
    me = rt.create_consumer("ag", None, {"topic": "work", "poll.timeout.ms": 50})
    me.start()
    pr.join(30)
    got = []
    deadline = time.time() + 10
    while len(got) < 10 and time.time() < deadline:
        got += me.read()      # the dead member is reaped -> all partitions are ours
    assert sorted(r.value() for r in got) == list(range(10))
    assert rt.log.group_members("work", "langstream-agent-ag") == 1


def test_registry_type_shm(logname):
    rt = TopicConnectionsRuntimeRegistry.get(StreamingCluster("shm", {"name": logname, "size-mb": 64}))
    assert isinstance(rt, ShmTopicConnectionsRuntime)


def test_retention_overtaking_an_unacked_consumer_does_not_freeze_commits(logname):
    """with retention-messages, head blocks are dropped even when a group has
    not committed them.  The lagging member must move its committed offset (and the
    group's published one) up to the first stored offset, or the contiguous-prefix
    commit freezes below offsets that can never be acked again."""
    rt = _rt(logname)
    rt.log.create_topic("r", 1, 200)                  # keep ~200 messages
    c = rt.create_consumer("ag", None, {"topic": "r", "max.poll.records": 5})
    c.start()
    prod = rt.create_producer("a", None, {"topic": "r"})
    blob = "y" * 2000
    for i in range(10):
        prod.write(SimpleRecord.of(None, f"{i}:" + blob)).result(5)
    first = c.read()                                  # delivered, never acked
    assert first
    for i in range(10, 3000):                          # retention drops the head past them
        prod.write(SimpleRecord.of(None, f"{i}:" + blob)).result(5)
    base = rt.log.begin_offsets("r")[0]
    assert base > 10
    seen = 0
    for _ in range(2000):
        recs = c.read()
        if not recs:
            break
        c.commit(recs)
        seen += len(recs)
    committed = rt.log.committed("r", "langstream-agent-ag")[0]
    assert committed == rt.log.end_offsets("r")[0] == 3000
    assert rt.log.lag("r", "langstream-agent-ag") in (0, [0], {0: 0}) or sum(
        rt.log.lag("r", "langstream-agent-ag")) == 0
    # a fresh member of the group starts at the committed end, not at stale offsets
    c.close()
    c2 = rt.create_consumer("ag", None, {"topic": "r"})
    c2.start()
    assert c2.read() == []
