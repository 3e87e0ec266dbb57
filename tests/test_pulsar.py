"""Pulsar streaming runtime (WebSocket + admin REST client) against the in-tree
Pulsar-compatible standalone broker; a pipeline running on the ``pulsar`` type.

Mirrors the reference's PulsarClusterRuntimeDockerTest (topic creation on deploy,
Failover subscriptions, per-message acknowledge) without a Pulsar container."""
import json
import time
import uuid

import pytest

from langstream_amd.api.record import SimpleRecord
from langstream_amd.api.topics import TopicOffsetPosition
from langstream_amd.topics.pulsar import PulsarConfig, PulsarConsumer, PulsarProducer, PulsarReader
from langstream_amd.topics.pulsar.standalone import PulsarStandalone
from langstream_amd.utils.wsclient import WebSocket


class _SC:
    def __init__(self, url):
        self.type = "pulsar"
        self.configuration = {"admin": {"serviceUrl": url}, "service": {"serviceUrl": url.replace("http", "pulsar")},
                              "default-tenant": "public", "default-namespace": "default"}


@pytest.fixture(scope="module")
def broker():
    b = PulsarStandalone().start()
    yield b
    b.stop()


def _read(c, n, timeout=10):
    out = []
    deadline = time.time() + timeout
    while len(out) < n and time.time() < deadline:
        out += c.read()
    return out


def test_wsclient_roundtrip_large_frames(broker):
    cfg = PulsarConfig(_SC(broker.web_url))
    t = cfg.full("ws-" + uuid.uuid4().hex[:6])
    p = PulsarProducer(cfg, t)
    p.start()
    big = "x" * 200_000  # 64-bit length frames
    p.write(SimpleRecord.of("k", big)).result(10)
    c = PulsarConsumer(cfg, t, "s1")
    c.start()
    got = _read(c, 1)
    assert got[0].value() == big and got[0].key() == "k"
    c.close()
    p.close()
    with pytest.raises(ConnectionError):
        WebSocket(broker.web_url.replace("http", "ws") + "/nope")


def test_admin_create_list_delete(broker):
    cfg = PulsarConfig(_SC(broker.web_url))
    name = cfg.full("adm-" + uuid.uuid4().hex[:6])
    assert not cfg.topic_exists(name)
    assert cfg.admin("PUT", cfg.rest_path(name) + "/partitions", data="3").status_code == 204
    assert cfg.admin("PUT", cfg.rest_path(name) + "/partitions", data="3").status_code == 409
    assert cfg.partitions(name) == 3 and cfg.topic_exists(name)
    lst = cfg.admin("GET", "persistent/public/default").json()
    assert f"{name}-partition-2" in lst
    assert cfg.admin("DELETE", cfg.rest_path(name) + "/partitions").status_code == 204
    assert not cfg.topic_exists(name)


def test_failover_ack_and_redelivery(broker):
    cfg = PulsarConfig(_SC(broker.web_url))
    t = cfg.full("fo-" + uuid.uuid4().hex[:6])
    cfg.admin("PUT", cfg.rest_path(t) + "/partitions", data="2")
    p = PulsarProducer(cfg, t)
    for i in range(20):
        p.write(SimpleRecord.of(f"k{i % 4}", json.dumps({"i": i}), [])).result(10)
    c1 = PulsarConsumer(cfg, t, "grp")
    c1.start()
    first = _read(c1, 20)
    assert sorted(json.loads(r.value())["i"] for r in first) == list(range(20))
    # ack half, drop the connection: the other half is redelivered to the next consumer
    c1.commit(first[:10])
    time.sleep(0.3)
    c1.close()
    c2 = PulsarConsumer(cfg, t, "grp")
    c2.start()
    again = _read(c2, 10)
    assert sorted(r.value() for r in again) == sorted(r.value() for r in first[10:])
    # two live consumers on a 2-partition topic: each partition has one active consumer
    c3 = PulsarConsumer(cfg, t, "grp")
    c3.start()
    c2.commit(again)
    for i in range(20, 40):
        p.write(SimpleRecord.of(f"k{i % 4}", json.dumps({"i": i}), [])).result(10)
    got2, got3 = [], []
    deadline = time.time() + 10
    while len(got2) + len(got3) < 20 and time.time() < deadline:
        got2 += c2.read()
        got3 += c3.read()
    assert sorted(json.loads(r.value())["i"] for r in got2 + got3) == list(range(20, 40))
    parts2 = {r.message_id for r in got2}
    parts3 = {r.message_id for r in got3}
    assert not parts2 & parts3
    for c in (c2, c3):
        c.close()
    p.close()


def test_reader_positions(broker):
    cfg = PulsarConfig(_SC(broker.web_url))
    t = cfg.full("rd-" + uuid.uuid4().hex[:6])
    p = PulsarProducer(cfg, t)
    for i in range(5):
        p.write(SimpleRecord.of(None, f"v{i}")).result(10)
    r = PulsarReader(cfg, t, TopicOffsetPosition.EARLIEST)
    r.start()
    got, off = [], None
    deadline = time.time() + 10
    while len(got) < 3 and time.time() < deadline:
        res = r.read()
        got += res.records
        off = res.offset or off
    r.close()
    # resume after the last record the first reader returned
    r2 = PulsarReader(cfg, t, TopicOffsetPosition.absolute(off))
    r2.start()
    rest = []
    deadline = time.time() + 10
    while len(got) + len(rest) < 5 and time.time() < deadline:
        rest += r2.read().records
    assert [x.value() for x in got + rest] == [f"v{i}" for i in range(5)]
    latest = PulsarReader(cfg, t, TopicOffsetPosition.LATEST)
    latest.start()
    assert latest.read().records == []
    p.write(SimpleRecord.of(None, "new")).result(10)
    deadline = time.time() + 10
    fresh = []
    while not fresh and time.time() < deadline:
        fresh = latest.read().records
    assert [x.value() for x in fresh] == ["new"]
    for x in (r2, latest, p):
        x.close()


def test_pipeline_on_pulsar_runtime(broker):
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
    type: pulsar
    configuration:
      admin:
        serviceUrl: "{broker.web_url}"
      service:
        serviceUrl: "{broker.service_url}"
"""
    app = LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, instance=instance).start(wait=20)
    try:
        cfg = PulsarConfig(_SC(broker.web_url))
        assert cfg.partitions(cfg.full(tin)) == 2 and cfg.topic_exists(cfg.full(tout))
        for i in range(10):
            app.produce(tin, json.dumps({"n": i}), key=f"k{i}")
        out = app.consume(tout, 10, timeout=30)
        vals = sorted(json.loads(r.value())["n2"] for r in out)
        assert vals == [2 * i for i in range(10)]
    finally:
        app.stop(10)
