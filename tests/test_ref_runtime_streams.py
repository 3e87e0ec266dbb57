"""Ported reference runtime scenarios, part 5: the runner on the Pulsar and Pravega
streaming types (``langstream-runtime/langstream-runtime-impl/src/test/java/ai/langstream/
pulsar/PulsarRunnerDockerTest.java`` and ``pravega/PravegaRunnerDockerTest.java``), here
against the in-tree Pulsar-compatible and Pravega stand-ins instead of containers (so
wire parity with live brokers stays unpinned: no Pulsar / Pravega client ships offline).
"""
from __future__ import annotations

import json
import uuid

import pytest

from ref_runtime_harness import Run, header, uniq
from langstream_amd.topics.pravega.standalone import PravegaStandalone
from langstream_amd.topics.pulsar.standalone import PulsarStandalone


@pytest.fixture(scope="module")
def pulsar():
    b = PulsarStandalone().start()
    yield b
    b.stop()


@pytest.fixture(scope="module")
def pravega():
    s = PravegaStandalone().start()
    yield s
    s.stop()


def _module(tin, tout, body, out_extra=""):
    return {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
  - name: "{tout}"
    creation-mode: create-if-not-exists
{out_extra}pipeline:
{body.format(tin=tin, tout=tout)}"""}


DROP = ('  - name: "drop-description"\n    id: "step1"\n    type: "drop-fields"\n    input: "{tin}"\n'
        '    output: "{tout}"\n    configuration:\n      fields:\n        - "description"\n')
FAILING = ('  - name: "some agent"\n    id: "step1"\n    type: "mock-failing-processor"\n    input: "{tin}"\n'
           '    output: "{tout}"\n    errors:\n        on-failure: dead-letter\n    configuration:\n'
           '      fail-on-content: "fail-me"\n')
DOC = '{"name": "some name", "description": "some description"}'


def _ps(b, tenant="public", ns="default"):
    return "pulsar", (b.web_url, b.service_url, tenant, ns)


def _raw(b, topic):
    t = b.topics[topic]
    return [m for p in t.parts for m in p.log]


# ---------------------------------------------------------------- PulsarRunnerDockerTest
def test_pulsar_simple(pulsar):
    """PulsarRunnerDockerTest.simpleTest: drop-fields on Pulsar topics; the message
    property travels with the record."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run(*_ps(pulsar), _module(tin, tout, DROP)) as r:
        r.produce(tin, DOC, headers={"header-key": "header-value"})
        recs = r.wait_for(tout, ['{"name":"some name"}'])
        assert header(recs[0], "header-key") == "header-value"


def test_pulsar_different_tenant(pulsar):
    """PulsarRunnerDockerTest.simpleTestDifferentTenant: default-tenant / default-namespace
    of the instance place the topics under persistent://mytenant/mynamespace/."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run(*_ps(pulsar, "mytenant", "mynamespace"), _module(tin, tout, DROP)) as r:
        assert f"persistent://mytenant/mynamespace/{tin}" in pulsar.topics
        r.produce(tin, DOC, headers={"header-key": "header-value"})
        recs = r.wait_for(tout, ['{"name":"some name"}'])
        assert header(recs[0], "header-key") == "header-value"
        assert len(_raw(pulsar, f"persistent://mytenant/mynamespace/{tout}")) == 1


def test_pulsar_topic_schema(pulsar):
    """PulsarRunnerDockerTest.testTopicSchema: a ``bytes`` output topic gets the compact
    JSON text as raw bytes."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _module(tin, tout, DROP, out_extra='    schema:\n      type: "bytes"\n')
    with Run(*_ps(pulsar), files) as r:
        r.produce(tin, DOC)
        r.wait_for(tout, ['{"name":"some name"}'])
        raw = _raw(pulsar, f"persistent://public/default/{tout}")
        assert [m.payload for m in raw] == [b'{"name":"some name"}']


def test_pulsar_key_value_schema(pulsar):
    """PulsarRunnerDockerTest.testKeyValueSchema: string key / string value topics
    (KeyValue SEPARATED): identity keeps both."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    kv = '    schema:\n      type: "string"\n    keySchema:\n      type: "string"\n'
    files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
{kv}  - name: "{tout}"
    creation-mode: create-if-not-exists
{kv}pipeline:
  - id: "step1"
    type: "identity"
    input: "{tin}"
    output: "{tout}"
"""}
    with Run(*_ps(pulsar), files) as r:
        r.produce(tin, "value", key="key")
        recs = r.wait_for(tout, ["value"])
        assert recs[0].key() in ("key", b"key")
        raw = _raw(pulsar, f"persistent://public/default/{tout}")
        assert [(m.key, m.payload) for m in raw] == [("key", b"value")]


def test_pulsar_dead_letter(pulsar):
    """PulsarRunnerDockerTest.testDeadLetter: failing records go to <input>-deadletter."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run(*_ps(pulsar), _module(tin, tout, FAILING)) as r:
        for i in range(10):
            r.produce(tin, f"fail-me-{i}")
            r.produce(tin, f"keep-me-{i}")
        r.wait_for(tin + "-deadletter", [f"fail-me-{i}" for i in range(10)])
        r.wait_for(tout, [f"keep-me-{i}" for i in range(10)])


# ---------------------------------------------------------------- PravegaRunnerDockerTest
def test_pravega_run_agent(pravega):
    """PravegaRunnerDockerTest.testRunAgent: drop-fields on Pravega streams in scope
    ``langstream``."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run("pravega", pravega.controller_uri, _module(tin, tout, DROP)) as r:
        r.produce(tin, DOC)
        recs = r.wait_for(tout, ['{"name":"some name"}'])
        assert recs


def test_pravega_dead_letter(pravega):
    """PravegaRunnerDockerTest.testDeadLetter (agent ``step2`` as there: reader groups are
    named after the agent and outlive an application on the same controller)."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run("pravega", pravega.controller_uri, _module(tin, tout, FAILING.replace('"step1"', '"step2"'))) as r:
        for i in range(10):
            r.produce(tin, f"fail-me-{i}")
            r.produce(tin, f"keep-me-{i}")
        r.wait_for(tin + "-deadletter", [f"fail-me-{i}" for i in range(10)])
        r.wait_for(tout, [f"keep-me-{i}" for i in range(10)])
