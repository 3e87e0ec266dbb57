"""Pravega streaming runtime against the in-tree single-node server; a pipeline running
on the ``pravega`` type.

Mirrors the reference's ``PravegaClusterRuntimeDockerTest.testMapPravegaTopic``
(langstream-pravega-runtime/src/test/java/ai/langstream/pravega/PravegaClusterRuntimeDockerTest.java:36-91:
streams created on deploy, only ``deletion-mode: delete`` streams removed on delete)
without a Pravega container; wire compatibility with a live Pravega is unpinned."""
import json
import time
import uuid

import pytest

from langstream_amd.api.record import Header, SimpleRecord
from langstream_amd.api.topics import TopicOffsetPosition
from langstream_amd.topics.pravega import (PravegaClient, PravegaConfig, PravegaConsumer, PravegaProducer,
                                           PravegaReader, PravegaTopicConnectionsRuntime, wire)
from langstream_amd.topics.pravega.standalone import PravegaStandalone


class _SC:
    def __init__(self, uri, scope="langstream"):
        self.type = "pravega"
        self.configuration = {"client": {"controller-uri": uri, "scope": scope}}


@pytest.fixture(scope="module")
def server():
    s = PravegaStandalone().start()
    yield s
    s.stop()


def _read(c, n, timeout=10):
    out = []
    deadline = time.time() + timeout
    while len(out) < n and time.time() < deadline:
        out += c.read()
    return out


def test_key_routing_is_stable():
    assert wire.segment_for_key("a", 1) == 0
    segs = {wire.segment_for_key(f"k{i}", 4) for i in range(200)}
    assert segs == {0, 1, 2, 3}
    assert all(wire.segment_for_key("same", 4) == wire.segment_for_key("same", 4) for _ in range(3))
    assert wire.parse_uri("tcp://h:1234") == ("h", 1234)


def test_deploy_and_delete_streams(server):
    from langstream_amd.core.deployer import ApplicationDeployer
    from langstream_amd.core.parser import build_application_instance
    module = """
module: "module-1"
id: "pipeline-1"
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
  - name: "input-topic-2-partitions"
    creation-mode: create-if-not-exists
    deletion-mode: none
    partitions: 2
  - name: "input-topic-delete"
    creation-mode: create-if-not-exists
    deletion-mode: delete
"""
    instance = f"""
instance:
  streamingCluster:
    type: "pravega"
    configuration:
      client:
        controller-uri: "{server.controller_uri}"
        scope: "langstream"
  computeCluster:
    type: "none"
"""
    app = build_application_instance({"module.yaml": module}, instance).application
    dep = ApplicationDeployer()
    plan = dep.create_implementation("app", app)
    dep.setup("tenant", plan)
    c = PravegaClient(server.controller_uri)
    for name in ("input-topic", "input-topic-2-partitions", "input-topic-delete"):
        assert c.stream_exists("langstream", name)
    assert c.stream_info("langstream", "input-topic-2-partitions")["segments"] == 2
    assert c.stream_info("langstream", "input-topic")["segments"] == 1
    dep.delete("tenant", plan)
    dep.cleanup("tenant", plan)
    assert not c.stream_exists("langstream", "input-topic-delete")
    assert c.stream_exists("langstream", "input-topic-2-partitions")
    assert c.stream_exists("langstream", "input-topic")


def test_seal_and_delete_rules(server):
    c = PravegaClient(server.controller_uri)
    c.create_scope("s1")
    c.create_stream("s1", "t", 1)
    with pytest.raises(RuntimeError, match="sealed before deletion"):
        c.delete_stream("s1", "t")
    c.seal_stream("s1", "t")
    cfg = PravegaConfig(_SC(server.controller_uri, "s1"))
    p = PravegaProducer(cfg, "t")
    p.start()
    with pytest.raises(RuntimeError, match="sealed"):
        p.write(SimpleRecord.of(value="x")).result(10)
    p.close()
    c.delete_stream("s1", "t")
    assert not c.stream_exists("s1", "t")


def test_reader_group_shares_segments_and_keeps_key_order(server):
    scope, topic = "langstream", "rg-" + uuid.uuid4().hex[:6]
    c = PravegaClient(server.controller_uri)
    c.create_scope(scope)
    c.create_stream(scope, topic, 4)
    cfg = PravegaConfig(_SC(server.controller_uri))
    p = PravegaProducer(cfg, topic)
    p.start()
    futs = [p.write(SimpleRecord.of(key=f"k{i % 8}", value={"n": i}, headers=[Header("h", "v")]))
            for i in range(400)]
    placed = [f.result(10) for f in futs]
    assert len({seg for seg, _ in placed}) > 1
    r1 = PravegaConsumer(cfg, topic, "g1", "r1", poll_ms=200)
    r2 = PravegaConsumer(cfg, topic, "g1", "r2", poll_ms=200)
    r1.start()
    r2.start()
    got = _read(r1, 1, timeout=2)
    got += _read(r2, 1, timeout=2)
    deadline = time.time() + 10
    while len(got) < 400 and time.time() < deadline:
        got += r1.read() + r2.read()
    assert len(got) == 400
    assert {r.get_header("h").value for r in got} == {"v"}
    # each key lives in one segment, and within a segment events keep their order
    by_key = {}
    for r in sorted(got, key=lambda r: (r.segment, r.offset)):
        v = json.loads(r.value()) if isinstance(r.value(), str) else r.value()
        by_key.setdefault(r.key(), []).append(v["n"])
    for k, ns in by_key.items():
        assert ns == sorted(ns), k
    # both readers owned segments of the group
    assert {r.segment for r in r1.read()} == set() and r1.get_info()["readerGroup"] == "g1"
    # a reader going offline hands its segments over, positioned after its last read event
    p.write(SimpleRecord.of(key="k1", value={"n": 1000})).result(10)
    p.write(SimpleRecord.of(key="k2", value={"n": 1001})).result(10)
    r2.close()
    late = _read(r1, 2, timeout=5)
    assert sorted(json.loads(x.value())["n"] if isinstance(x.value(), str) else x.value()["n"] for x in late) \
        == [1000, 1001]
    r1.close()
    p.close()


def test_reader_positions(server):
    scope, topic = "langstream", "pos-" + uuid.uuid4().hex[:6]
    c = PravegaClient(server.controller_uri)
    c.create_scope(scope)
    c.create_stream(scope, topic, 2)
    cfg = PravegaConfig(_SC(server.controller_uri))
    p = PravegaProducer(cfg, topic)
    p.start()
    for i in range(6):
        p.write(SimpleRecord.of(key=f"k{i}", value=f"v{i}")).result(10)
    latest = PravegaReader(cfg, topic, TopicOffsetPosition("latest"), poll_s=0.2)
    latest.start()
    assert latest.read().records == []
    earliest = PravegaReader(cfg, topic, TopicOffsetPosition("earliest"), poll_s=0.2)
    earliest.start()
    res = earliest.read()
    assert sorted(r.value() for r in res.records) == [f"v{i}" for i in range(6)]
    for i in range(6, 9):
        p.write(SimpleRecord.of(key=f"k{i}", value=f"v{i}")).result(10)
    assert sorted(r.value() for r in latest.read().records) == ["v6", "v7", "v8"]
    resumed = PravegaReader(cfg, topic, TopicOffsetPosition.absolute(res.offset), poll_s=0.2)
    resumed.start()
    assert sorted(r.value() for r in resumed.read().records) == ["v6", "v7", "v8"]
    for r in (latest, earliest, resumed):
        r.close()
    p.close()


def test_pipeline_on_pravega_runtime(server):
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
    type: pravega
    configuration:
      client:
        controller-uri: "{server.controller_uri}"
"""
    app = LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, instance=instance).start(wait=20)
    try:
        c = PravegaClient(server.controller_uri)
        assert c.stream_info("langstream", tin)["segments"] == 2
        for i in range(10):
            app.produce(tin, json.dumps({"n": i}), key=f"k{i}")
        out = app.consume(tout, 10, timeout=30)
        # RecordWrapper JSON: a structured value comes back as a map, as with Jackson
        vals = sorted((r.value() if isinstance(r.value(), dict) else json.loads(r.value()))["n2"] for r in out)
        assert vals == [2 * i for i in range(10)]
    finally:
        app.stop(10)


def test_runtime_registered():
    from langstream_amd.api.topics import TopicConnectionsRuntimeRegistry
    import langstream_amd.topics  # noqa: F401
    rt = TopicConnectionsRuntimeRegistry.get(_SC("tcp://127.0.0.1:1"))
    assert isinstance(rt, PravegaTopicConnectionsRuntime)
