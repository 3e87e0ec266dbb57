"""Ported reference runtime scenarios, part 4: HTTP / LangServe / JDBC / web-crawler
agents, Kafka Connect sink and source adapters, topic-name placeholders, and the
runtime's unit-level runner pieces (record tracker, agent and asset-manager loading).

Each test cites the Java method it mirrors under
``langstream-runtime/langstream-runtime-impl/src/test/java/ai/langstream/``; topic-level
cases run on the memory streaming cluster and on the in-tree Kafka broker.  The
reference's WireMock stubs are ``ref_runtime_harness.FakeHTTP``; its HerdDB container is
the in-tree HerdDB service (``agents/vector/herddb.py``); its Java Kafka Connect
``DummySinkConnector``/``DummySourceConnector`` are the same connectors written against
this runtime's Python connector API (``agents/kafka_connect.py``).
"""
from __future__ import annotations

import json
import os
import threading
import time
import uuid
from typing import List

import pytest

from ref_runtime_harness import FakeHTTP, Run, as_json, uniq
from langstream_amd.agents.kafka_connect import Connector, ConnectRecord, SinkTask, SourceTask
from langstream_amd.api.agent import AgentSource, SourceRecordAndResult
from langstream_amd.api.record import SimpleRecord
from langstream_amd.runtime.errors import PermanentFailureException
from langstream_amd.topics.kafka.broker import KafkaBroker


@pytest.fixture(scope="module")
def kafka():
    b = KafkaBroker(default_partitions=1).start()
    yield b
    b.stop()


@pytest.fixture(params=["memory", "kafka"])
def streaming(request, kafka):
    return request.param, (kafka.bootstrap if request.param == "kafka" else None)


@pytest.fixture(scope="module")
def wiremock():
    w = FakeHTTP()
    yield w
    w.close()


def _topics(*names):
    return "topics:\n" + "".join(f"  - name: \"{n}\"\n    creation-mode: create-if-not-exists\n"
                                 f"    deletion-mode: delete\n" for n in names)


# ---------------------------------------------------------------- kafka/HttpRequestAgentRunnerIT.java
MODEL_JSON = ('{"id": "my-model",\n "created": "2021-08-31T12:00:00Z",\n "model": "gpt-35-turbo",\n'
              ' "object": "text-generation",\n "choices": [{"text": "It is a car."}]}\n')
SECRETS = "secrets:\n- id: s1\n  data:\n    token: my-token!\n"


def _http_app(w, tin, tout, extra=""):
    return {"module.yaml": _topics(tin, tout) + f"""pipeline:
  - name: "http-request"
    type: "http-request"
    input: {tin}
    output: {tout}
    id: step1
    configuration:
        output-field: value.api
        url: {w.url}/api/models
        query-string:
            name: "{{{{{{ value.id }}}}}}"
{extra}"""}


def _http_run(streaming, files, want):
    tin = next(k for k in files["module.yaml"].split('"') if k.startswith("input-topic"))
    tout = next(k for k in files["module.yaml"].split('"') if k.startswith("output-topic"))
    with Run(*streaming, files, secrets=SECRETS) as r:
        r.produce(tin, '{"id":"my-model","classification":"good"}')
        r.wait_for(tout, [want])


def test_http_get_json(streaming, wiremock):
    """HttpRequestAgentRunnerIT.testGetJson: the JSON response lands in value.api."""
    wiremock.stub("GET", "/api/models?name=my-model", text=MODEL_JSON)
    tin, tout = uniq("input-topic"), uniq("output-topic")
    _http_run(streaming, _http_app(wiremock, tin, tout),
              '{"id":"my-model","classification":"good","api":{"id":"my-model","created":"2021-08-31T12:00:00Z",'
              '"model":"gpt-35-turbo","object":"text-generation","choices":[{"text":"It is a car."}]}}')


def test_http_get_raw_text(streaming):
    """HttpRequestAgentRunnerIT.testGetRawText: a non-JSON body is stored as a string."""
    w = FakeHTTP()
    try:
        w.stub("GET", "/api/models?name=my-model", text="some-string", ctype="text/plain")
        tin, tout = uniq("input-topic"), uniq("output-topic")
        _http_run(streaming, _http_app(w, tin, tout), '{"id":"my-model","classification":"good","api":"some-string"}')
    finally:
        w.close()


def test_http_post_with_body(streaming):
    """HttpRequestAgentRunnerIT.testPostWithBody: templated body, headers with a secret;
    the stub only answers when body and both headers match exactly."""
    w = FakeHTTP()
    try:
        w.stub("POST", "/api/models?name=my-model", body='{"id": "my-model"}', text=MODEL_JSON,
               headers={"Content-Type": "application/json", "Authorization": "Bearer my-token!"})
        tin, tout = uniq("input-topic"), uniq("output-topic")
        extra = """        method: POST
        body: '{"id": "{{{ value.id }}}"}'
        headers:
          Content-Type: application/json
          Authorization: Bearer {{{ secrets.s1.token }}}
"""
        _http_run(streaming, _http_app(w, tin, tout, extra),
                  '{"id":"my-model","classification":"good","api":{"id":"my-model","created":"2021-08-31T12:00:00Z",'
                  '"model":"gpt-35-turbo","object":"text-generation","choices":[{"text":"It is a car."}]}}')
    finally:
        w.close()


# ---------------------------------------------------------------- kafka/LangServeInvokeAgentRunnerIT.java
LANGSERVE_TOKENS = ["", "Why", " don", "'t", " cats", " play", " poker", " in", " the", " wild", "?\n\n", "Too",
                    " many", " che", "et", "ah", "s", "!", ""]


def test_langserve_stream_output(streaming):
    """LangServeInvokeAgentRunnerIT.testStreamOuput: the SSE stream of /chain/stream is
    re-chunked 1, 2, 4, 8... up to min-chunks-per-message onto the streaming topic and the
    whole answer goes to value.answer."""
    sse = "".join("event: data\ndata: " + json.dumps({"content": t, "additional_kwargs": {}, "type": "AIMessageChunk",
                                                     "example": False}) + "\n\n" for t in LANGSERVE_TOKENS)
    sse += "event: end"
    w = FakeHTTP()
    try:
        w.stub("POST", "/chain/stream", body='{"input":{"topic":"cats"}}', text=sse, ctype="text/event-stream")
        tin, tout, tstream = uniq("input-topic"), uniq("output-topic"), uniq("streaming-answers-topic")
        files = {"module.yaml": _topics(tin, tout, tstream) + f"""pipeline:
  - type: "langserve-invoke"
    input: {tin}
    output: {tout}
    id: step1
    configuration:
        output-field: value.answer
        stream-to-topic: {tstream}
        stream-response-field: value
        min-chunks-per-message: 10
        debug: false
        method: POST
        allow-redirects: true
        handle-cookies: false
        url: {w.url}/chain/stream
        headers:
           Authorisation: "Bearer {{{{secrets.langserve.token}}}}"
        fields:
           - name: topic
             expression: "value.topic"
"""}
        secrets = 'secrets:\n  - id: langserve\n    data:\n      token: "my-token"\n'
        with Run(*streaming, files, secrets=secrets) as r:
            r.produce(tin, '{"topic":"cats"}')
            r.wait_for(tout, ['{"answer":"Why don\'t cats play poker in the wild?\\n\\nToo many cheetahs!",'
                              '"topic":"cats"}'])
            r.wait_for(tstream, ["Why", " don't", " cats play poker in", " the wild?\n\nToo many cheetah", "s!"])
        assert w.requests[-1][3].get("Authorisation") == "Bearer my-token"
    finally:
        w.close()


# ---------------------------------------------------------------- kafka/JdbcDatabaseIT.java
@pytest.fixture()
def herddb():
    from langstream_amd.agents.vector import herddb as h
    srv = h.HerdDBServer().start()
    yield f"jdbc:herddb:server:localhost:{srv.port}"
    srv.stop()


def test_jdbc_simple_queries(streaming, herddb):
    """JdbcDatabaseIT.testSimpleQueries: an auto_increment table; ``execute`` with
    generated-keys returns {count: 1, generatedKeys: {key: n}}, then ``query`` reads the row
    back by that key."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"configuration.yaml": f"""
configuration:
  resources:
    - type: "datasource"
      name: "JdbcDatasource"
      configuration:
        service: "jdbc"
        driverClass: "herddb.jdbc.Driver"
        url: "{herddb}"
        user: "sa"
        password: "hdb"
""", "module.yaml": f"""
assets:
  - name: "documents-table"
    asset-type: "jdbc-table"
    creation-mode: create-if-not-exists
    config:
      table-name: "documents"
      datasource: "JdbcDatasource"
      create-statements:
        - |
          CREATE TABLE documents (
          pkfield integer auto_increment primary key,
          text string)
""" + _topics(tin, tout) + f"""pipeline:
  - name: "Write"
    type: "query"
    input: {tin}
    id: step1
    configuration:
      mode: "execute"
      datasource: "JdbcDatasource"
      output-field: "value.command_results"
      generated-keys:
        - "pkfield"
      query: |
            INSERT INTO DOCUMENTS (text) values(?)
      fields:
        - "value.text"
  - name: "Read"
    type: "query"
    output: {tout}
    configuration:
      mode: "query"
      datasource: "JdbcDatasource"
      output-field: "value.query_results"
      query: |
            SELECT * FROM DOCUMENTS where pkfield = ?
      fields:
        - "fn:toInt(value.command_results.generatedKeys.key)"
"""}
    with Run(*streaming, files) as r:
        for i in range(10):
            r.produce(tin, json.dumps({"text": f"doc{i}.pdf"}, separators=(",", ":")))
        recs, _ = r.read_all(tout, 10, 30)
        assert len(recs) == 10
        for i, rec in enumerate(recs):
            v = as_json(rec.value())
            assert v["text"] == f"doc{i}.pdf"
            assert v["command_results"] == {"count": 1, "generatedKeys": {"key": i + 1}}
            assert v["query_results"] == [{"pkfield": i + 1, "text": f"doc{i}.pdf"}]


# ---------------------------------------------------------------- kafka/PlaceholderEndToEndTest.java
def test_schema_with_variable_topic_names(kafka):
    """PlaceholderEndToEndTest.testUseSchemaWithKafkaAndVariableTopicNames: topic names
    from ``${globals.*}``; an Avro record goes through identity into the output topic,
    whose schema is registered from the record."""
    from langstream_amd.api.avro import wire_decode, wire_encode
    from langstream_amd.topics.kafka.client import KafkaClient, PartitionReader, Producer
    from langstream_amd.topics.kafka.schema_registry import SchemaRegistryClient, SchemaRegistryServer
    schema = {"type": "record", "name": "Pojo", "namespace": "mynamespace",
              "fields": [{"name": "name", "type": "string"}]}
    reg = SchemaRegistryServer()
    try:
        tin, tout = uniq("my-input-topic"), uniq("my-output-topic")
        files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "${{globals.input-topic}}"
    creation-mode: create-if-not-exists
    schema:
      type: avro
      schema: '{json.dumps(schema)}'
  - name: "${{globals.output-topic}}"
    creation-mode: create-if-not-exists
    schema:
      type: avro
pipeline:
  - name: "identity"
    id: "step1"
    type: "identity"
    input: "${{globals.input-topic}}"
    output: "${{globals.output-topic}}"
"""}
        glb = {"input-topic": tin, "output-topic": tout, "stream-response-topic": uniq("my-stream-topic")}
        with Run("kafka", kafka.bootstrap, files, globals_=glb, extra_admin={"schema.registry.url": reg.url}) as r:
            assert sorted(r.plan.topics) == sorted([tin, tout])
            sr = SchemaRegistryClient(reg.url)
            sid = sr.register(f"{tin}-value", schema)
            c = KafkaClient(kafka.bootstrap)
            Producer(c, tin).send_many([(None, wire_encode(sid, schema, {"name": "foo"}), [], int(time.time() * 1000))])
            got, rd = [], PartitionReader(c, tout, start="earliest")
            deadline = time.time() + 20
            while not got and time.time() < deadline:
                got = rd.read(10)
            assert got, "no output record"
            value = got[0][4]
            out_id = int.from_bytes(value[1:5], "big")
            assert wire_decode(value, lambda i: sr.get_by_id(i).to_json() if i == out_id else None) == {"name": "foo"}
            c.close()
    finally:
        reg.close()


# ---------------------------------------------------------------- kafka/WebCrawlerSourceIT.java
def test_webcrawler_source(streaming, tmp_path):
    """WebCrawlerSourceIT.test: three linked pages crawled from the seed; each record is
    the page re-serialised from its parsed tree; the crawler's status file is on disk."""
    w = FakeHTTP()
    try:
        w.stub("GET", "/index.html", text='<a href="secondPage.html">link</a>\n', ctype="text/html")
        w.stub("GET", "/secondPage.html", text='  <a href="thirdPage.html">link</a>\n  <a href="index.html">link to '
                                               'home</a>\n', ctype="text/html")
        w.stub("GET", "/thirdPage.html", text="  Hello!\n", ctype="text/html")
        app_id = "app-" + uuid.uuid4().hex[:4]
        tout = uniq("output-topic")
        files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "${{globals.output-topic}}"
    creation-mode: create-if-not-exists
pipeline:
  - type: "webcrawler-source"
    id: "step1"
    output: "${{globals.output-topic}}"
    configuration:
        seed-urls: ["{w.url}/index.html"]
        allow-non-html-contents: true
        allowed-domains: ["{w.url}"]
        state-storage: disk
"""}
        state = str(tmp_path / "state")
        with Run(*streaming, files, globals_={"output-topic": tout}, app_id=app_id, state_dir=state) as r:
            r.wait_for(tout, [
                '<html>\n <head></head>\n <body>\n  <a href="secondPage.html">link</a>\n </body>\n</html>',
                '<html>\n <head></head>\n <body>\n  <a href="thirdPage.html">link</a> <a href="index.html">link to '
                'home</a>\n </body>\n</html>',
                '<html>\n <head></head>\n <body>\n  Hello!\n </body>\n</html>'], timeout=30)
        name = f"{app_id}-step1.webcrawler.status.json"
        found = [os.path.join(d, name) for d, _, fs in os.walk(os.path.join(state, "step1")) if name in fs]
        assert found, f"{name} not under {state}/step1"
    finally:
        w.close()


# ---------------------------------------------------------------- kafka/KafkaConnectSinkRunnerIT.java
class DummySink(SinkTask):
    received: List[ConnectRecord] = []

    def put(self, records):
        DummySink.received.extend(records)


class DummySinkConnector(Connector):
    def task_class(self):
        return DummySink

    def task_configs(self, max_tasks):
        return [{}]


def _sink_app(tin, on_failure):
    return {"module.yaml": f"""
module: "module-2"
id: "pipeline-2"
errors:
  on-failure: "{on_failure}"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
pipeline:
  - name: "sink2"
    id: "step2"
    type: "sink"
    input: "{tin}"
    configuration:
      adapterConfig:
        __test_inject_conversion_error: "1"
        lingerTimeMs: 50
      connector.class: {__name__}:DummySinkConnector
      file: /tmp/test.sink.txt
"""}


GOOD = '{"name": "some name", "description": "some description"}'


def _until(cond, timeout=20.0):
    deadline = time.time() + timeout
    while not cond():
        assert time.time() < deadline, "condition not reached"
        time.sleep(0.02)


def test_kafka_connect_sink_fail_on_error(streaming):
    """KafkaConnectSinkRunnerIT.testRunKafkaConnectSinkFailOnErr: the injected conversion
    error stops the agent with that cause; the task receives nothing."""
    DummySink.received = []
    tin = uniq("input-topic2")
    with Run(*streaming, _sink_app(tin, "fail")) as r:
        r.produce(tin, "err")
        r.produce(tin, GOOD)
        err = r.wait_failure()
        cause = err.__cause__ if isinstance(err, PermanentFailureException) and err.__cause__ else err
        assert "Injected record conversion error" in str(cause)
        time.sleep(0.5)
        assert DummySink.received == []


@pytest.mark.parametrize("on_failure", ["skip", "dead-letter"])
def test_kafka_connect_sink_skip_or_dlq_on_error(streaming, on_failure):
    """KafkaConnectSinkRunnerIT.testRunKafkaConnectSinkSkipOnErr /
    testRunKafkaConnectSinkDlqOnErr: the bad record is skipped (or dead-lettered) and
    the good one reaches the task."""
    DummySink.received = []
    tin = uniq("input-topic3")
    with Run(*streaming, _sink_app(tin, on_failure)) as r:
        r.produce(tin, "err")
        r.produce(tin, GOOD)
        _until(lambda: len(DummySink.received) == 1)
        assert DummySink.received[0].value in (GOOD, GOOD.encode())
        if on_failure == "dead-letter":
            r.wait_for(tin + "-deadletter", ["err"])
        assert not r.app.errors


# ---------------------------------------------------------------- kafka/KafkaConnectSourceRunnerIT.java
class DummySource(SourceTask):
    def start(self, props):
        self.messages = [f"message-{i}" for i in range(int(props["num-messages"]))]

    def poll(self):
        if not self.messages:
            time.sleep(0.05)
            return []
        return [ConnectRecord(None, 0, None, None, self.messages.pop(0), {}, int(time.time() * 1000))]


class DummySourceConnector(Connector):
    def start(self, props):
        self.props = dict(props)

    def task_class(self):
        return DummySource

    def task_configs(self, max_tasks):
        return [self.props]       # the whole connector configuration goes to the task


def test_kafka_connect_source(streaming):
    """KafkaConnectSourceRunnerIT.testRunKafkaConnectSource: 5 messages from the task's
    poll() in order."""
    tout, toff = uniq("output-topic"), uniq("offset-topic")
    files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tout}"
    creation-mode: create-if-not-exists
  - name: "{toff}"
    creation-mode: create-if-not-exists
    partitions: 1
    options:
      replication-factor: 1
    config:
      cleanup.policy: compact
pipeline:
  - name: "source1"
    id: "step1"
    type: "source"
    output: "{tout}"
    configuration:
      connector.class: {__name__}:DummySourceConnector
      num-messages: 5
      offset.storage.topic: "{toff}"
"""}
    with Run(*streaming, files) as r:
        r.wait_for(tout, [f"message-{i}" for i in range(5)])


# ---------------------------------------------------------------- runtime/agent/AgentRecordTrackerTest.java
class _MySource(AgentSource):
    def __init__(self):
        super().__init__()
        self.committed = []

    def commit(self, records):
        self.committed.extend(records)

    def read(self):
        return []


def _tracker():
    from langstream_amd.runtime.tracker import SourceRecordTracker
    src = _MySource()
    return src, SourceRecordTracker(src)


def _no_leaks(t):
    assert not t._remaining and not t._sink_to_source and not t._ordered


def test_tracker():
    """AgentRecordTrackerTest.testTracker"""
    src, t = _tracker()
    source, sink = SimpleRecord.of("key", "sourceValue"), SimpleRecord.of("key", "sinkValue")
    t.track([SourceRecordAndResult(source, [sink], None)])
    t.commit([sink])
    assert src.committed == [source]
    _no_leaks(t)


def test_tracker_chunking():
    """AgentRecordTrackerTest.testChunking: the source commits after BOTH sink records."""
    src, t = _tracker()
    source = SimpleRecord.of("key", "sourceValue")
    s1, s2 = SimpleRecord.of("key", "sinkValue"), SimpleRecord.of("key", "sinkValue2")
    t.track([SourceRecordAndResult(source, [s1, s2], None)])
    t.commit([s1])
    assert src.committed == []
    t.commit([s2])
    assert src.committed == [source]
    _no_leaks(t)


def test_tracker_skipped_record():
    """AgentRecordTrackerTest.testSkippedRecord: a source with no results commits at the
    next commit pass."""
    src, t = _tracker()
    source, sink = SimpleRecord.of("key", "sourceValue"), SimpleRecord.of("key", "sinkValue")
    t.track([SourceRecordAndResult(source, [], None)])
    t.commit([sink])
    assert src.committed == [source]
    _no_leaks(t)


# ---------------------------------------------------------------- runtime/LoadAgentCodeTest.java
class _NullRecord:
    def key(self):
        return None

    def value(self):
        return None

    def origin(self):
        return None

    def timestamp(self):
        return None

    def headers(self):
        return []


def _load(agent_type):
    from langstream_amd.api.agent import AgentContext
    from langstream_amd.runtime.registry import create_agent
    a = create_agent(agent_type)
    a.set_metadata("x", agent_type, 0)
    a.init({})
    a.set_context(AgentContext(agent_id="x", global_agent_id="app-x"))
    a.start()
    return a


def test_load_noop():
    """LoadAgentCodeTest.testLoadNoop: one result, with no records."""
    a, res = _load("noop"), []
    a.process([_NullRecord()], res.append)
    assert len(res) == 1 and res[0].result_records == []


def test_load_identity():
    """LoadAgentCodeTest.testLoadIdentity: the same record object comes back, as result
    and as source."""
    a, rec = _load("identity"), _NullRecord()
    for _ in range(3):
        res = []
        a.process([rec], res.append)
        assert len(res) == 1 and res[0].result_records[0] is rec and res[0].source_record is rec


# ---------------------------------------------------------------- runtime/LoadAssertManagerCodeTest.java
class MockDatabaseResourceAssetManager:
    deployed: List[object] = []

    def __init__(self, asset):
        self.asset = asset

    def asset_exists(self):
        return any(a.id == self.asset.id for a in MockDatabaseResourceAssetManager.deployed)

    def deploy_asset(self):
        ds = (self.asset.config or {}).get("datasource")
        assert ds and ds.get("configuration", {}).get("url") == "bar"
        MockDatabaseResourceAssetManager.deployed.append(self.asset)

    def delete_asset_if_exists(self):
        if self.asset in MockDatabaseResourceAssetManager.deployed:
            MockDatabaseResourceAssetManager.deployed.remove(self.asset)
            return True
        return False


def test_load_mock_asset():
    """LoadAssertManagerCodeTest.testLoadMockAsset: a registered asset type loads through
    the registry; not there before deploy, there after."""
    from langstream_amd.agents.assets import AssetManagerRegistry
    from langstream_amd.api.model import AssetDefinition
    AssetManagerRegistry.register("mock-database-resource", MockDatabaseResourceAssetManager)
    asset = AssetDefinition(id="a1", name="a1", asset_type="mock-database-resource",
                            config={"datasource": {"configuration": {"url": "bar"}}})
    m = AssetManagerRegistry.create(asset)
    assert not m.asset_exists()
    m.deploy_asset()
    assert m.asset_exists()
    assert m.delete_asset_if_exists() and not m.asset_exists()
