"""Ported reference runtime scenarios, part 3: flow control, GenAI toolkit, re-rank, FLARE,
text processing and Avro schemas, on the memory streaming cluster and the in-tree Kafka
broker.  The reference's HerdDB container (``herddb/herddb:0.28.0``) is the in-tree
database service of ``langstream run --start-database`` (agents/vector/herddb.py),
addressed by the same ``jdbc:herddb:server:localhost:<port>`` URL.

* kafka/FlowControlRunnerIT (6): testDispatch, testDispatchNoDefaultDestination,
  testDispatchDefaultToAnotherAgent, testTimerSource, testTriggerEventProcessor
* kafka/GenIAgentsRunnerIT (2): testRunAITools, testRunAIToolsComposite
* kafka/RerankAgentRunnerIT.testSimpleRerank
* kafka/FlareControllerAgentRunnerIT.testSimpleFlare
* kafka/TextProcessingAgentsRunnerIT: testFullLanguageProcessingPipeline, testSplitThenJson
* kafka/KafkaSchemaTest.testUseSchemaWithKafka
"""
from __future__ import annotations

import json
import time
import uuid

import pytest

from ref_runtime_harness import FakeHTTP, Run, as_json, header, uniq
from langstream_amd.topics.kafka.broker import KafkaBroker


@pytest.fixture(scope="module")
def kafka():
    b = KafkaBroker(default_partitions=1).start()
    yield b
    b.stop()


@pytest.fixture(params=["memory", "kafka"])
def streaming(request, kafka):
    return request.param, (kafka.bootstrap if request.param == "kafka" else None)


def _topics(*names):
    return "topics:\n" + "".join(f"  - name: \"{n}\"\n    creation-mode: create-if-not-exists\n" for n in names)


# ---------------------------------------------------------------- FlowControlRunnerIT
def test_dispatch(streaming):
    """FlowControlRunnerIT.testDispatch: routes by header, default to the output topic."""
    tin, t1, t2, tdef = uniq("input-topic"), uniq("topic1"), uniq("topic2"), uniq("default-topic")
    files = {"module.yaml": _topics(tin, t1, t2, tdef) + f"""pipeline:
  - name: "Dispatch"
    type: "dispatch"
    input: {tin}
    output: {tdef}
    id: step1
    configuration:
      routes:
         - when: properties.language == "en"
           destination: {t1}
         - when: properties.language == "fr"
           destination: {t2}
         - when: properties.language == "none"
           action: drop
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, "for-default", headers={"language": "it"})
        r.produce(tin, "for-topic1", headers={"language": "en"})
        r.produce(tin, "for-topic2", headers={"language": "fr"})
        r.produce(tin, "dropped", headers={"language": "none"})
        r.wait_for(tdef, ["for-default"])
        r.wait_for(t1, ["for-topic1"])
        r.wait_for(t2, ["for-topic2"])


def test_dispatch_no_default_destination(streaming):
    """FlowControlRunnerIT.testDispatchNoDefaultDestination: without an output the
    dispatcher behaves like a sink for unrouted records (and they are committed)."""
    tin, t1, t2 = uniq("input-topic-no-default"), uniq("topic1-no-default"), uniq("topic2-no-default")
    files = {"module.yaml": _topics(tin, t1, t2) + f"""pipeline:
  - name: "Dispatch"
    type: "dispatch"
    input: {tin}
    id: step1
    configuration:
      routes:
         - when: properties.language == "en"
           destination: {t1}
         - when: properties.language == "fr"
           destination: {t2}
         - when: properties.language == "none"
           action: drop
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, "for-default", headers={"language": "it"})
        r.produce(tin, "for-topic1", headers={"language": "en"})
        r.produce(tin, "for-topic2", headers={"language": "fr"})
        r.wait_for(t1, ["for-topic1"])
        r.wait_for(t2, ["for-topic2"])
        runner = r.app.runners[0]
        deadline = time.time() + 10
        while runner.tracker.pending() and time.time() < deadline:
            time.sleep(0.02)
        assert runner.tracker.pending() == 0          # executeAgentRunners: fully committed


def test_dispatch_default_to_another_agent(streaming):
    """FlowControlRunnerIT.testDispatchDefaultToAnotherAgent: the default route is the next
    agent of the fused chain (compute), routed records skip it."""
    tin, t1, t2, tdef = (uniq("input-topic-to-agent"), uniq("topic1-to-agent"), uniq("topic2-to-agent"),
                         uniq("default-topic-to-agent"))
    files = {"module.yaml": _topics(tin, t1, t2, tdef) + f"""pipeline:
  - name: "Dispatch"
    type: "dispatch"
    input: {tin}
    id: step1
    configuration:
      routes:
         - when: properties.language == "en"
           destination: {t1}
           action: dispatch
         - when: properties.language == "fr"
           destination: {t2}
         - when: properties.language == "none"
           action: drop
  - name: "Compute"
    type: "compute"
    output: {tdef}
    id: step1
    configuration:
      fields:
         - name: "value"
           expression: "'modified'"
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, "for-default", headers={"language": "it"})
        r.produce(tin, "for-topic1", headers={"language": "en"})
        r.produce(tin, "for-topic2", headers={"language": "fr"})
        r.wait_for(tdef, ["modified"])
        r.wait_for(t1, ["for-topic1"])
        r.wait_for(t2, ["for-topic2"])


def test_timer_source(streaming):
    """FlowControlRunnerIT.testTimerSource: a record per period with the computed key
    (a UUID in a JSON key), value and header."""
    tout = uniq("timer-source-output-topic")
    files = {"module.yaml": _topics(tout) + f"""pipeline:
  - name: "Timer"
    type: "timer-source"
    id: step1
    output: {tout}
    configuration:
      period-seconds: 1
      fields:
         - name: "key.id"
           expression: "fn:uuid()"
         - name: "value.stringpayload"
           expression: "'constant-payload'"
         - name: "value.intpayload"
           expression: "42"
         - name: "properties.foo"
           expression: "'bar'"
"""}
    with Run(*streaming, files) as r:
        recs, _ = r.read_all(tout, 2, 15)
        assert len(recs) >= 2
        assert as_json(recs[0].value()) == {"intpayload": 42, "stringpayload": "constant-payload"}
        key = as_json(recs[0].key())
        uuid.UUID(key["id"])
        assert header(recs[0], "foo") == "bar"


def test_trigger_event_processor(streaming):
    """FlowControlRunnerIT.testTriggerEventProcessor: every chunk continues; the last chunk
    also goes to the side topic."""
    tin, side, tout = uniq("input-topic-splitter"), uniq("side-topic"), uniq("output-topic-chunks")
    files = {"module.yaml": _topics(tin, side, tout) + f"""pipeline:
  - name: "Chunk some text"
    id: step1
    type: "text-splitter"
    input: {tin}
    configuration:
      chunk_size: 5
      chunk_overlap: 0
  - name: "Trigger event on last chunk"
    type: "trigger-event"
    output: {tout}
    configuration:
      destination: {side}
      when: fn:toInt(properties.text_num_chunks) == (fn:toInt(properties.chunk_id) + 1)
      fields:
         - name: "properties.foo"
           expression: "'bar'"
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, "some very long text. end")
        r.wait_for(tout, ["some very long", "text. end"])
        side_recs = r.wait_for(side, ["text. end"])
        assert header(side_recs[0], "foo") == "bar"


# ---------------------------------------------------------------- GenIAgentsRunnerIT
def test_run_ai_tools(streaming):
    """GenIAgentsRunnerIT.testRunAITools: drop-fields keeps the headers."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"module.yaml": 'module: "module-1"\nid: "pipeline-1"\n' + _topics(tin, tout) + f"""pipeline:
  - name: "drop-description"
    id: "step1"
    type: "drop-fields"
    input: "{tin}"
    output: "{tout}"
    configuration:
      fields:
        - "description"
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, '{"name": "some name", "description": "some description"}',
                  headers={"header-key": "header-value"})
        recs, _ = r.read_all(tout, 1, 20)
        assert [as_json(x.value()) for x in recs] == [{"name": "some name"}]
        assert header(recs[0], "header-key") == "header-value"


def test_run_ai_tools_composite(streaming):
    """GenIAgentsRunnerIT.testRunAIToolsComposite: one fused pod whose /info lists the topic
    source, drop-fields, drop and the topic sink with their counters.  (The reference
    asserts the counters without sending a record; here one record goes through first.)"""
    tin, tout = uniq("input-topic1"), uniq("output-topic2")
    files = {"module.yaml": 'module: "module-1"\nid: "pipeline-1"\n' + _topics(tin, tout) + f"""pipeline:
  - name: "drop-description"
    id: "step1"
    type: "drop-fields"
    input: "{tin}"
    configuration:
      fields:
        - "description"
  - name: "drop"
    id: "step2"
    type: "drop"
    output: "{tout}"
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, '{"name": "n", "description": "d"}')
        runner = r.app.runners[0]
        deadline = time.time() + 10
        while runner.records_in < 1 and time.time() < deadline:
            time.sleep(0.02)
        time.sleep(0.2)
        info = runner.agent_info()
        types = [p["agent-type"] for p in info]
        assert types == ["topic-source", "drop-fields", "drop", "topic-sink"]
        by = {p["agent-type"]: p for p in info}
        assert by["topic-source"]["metrics"]["total-out"] >= 1
        assert by["drop-fields"]["metrics"]["total-in"] == 1 and by["drop-fields"]["metrics"]["total-out"] == 1
        assert by["drop"]["metrics"]["total-in"] == 1 and by["drop"]["metrics"]["total-out"] == 0
        assert all(p["metrics"]["started-at"] != 0 for p in info)
        r.wait_for(tout, [], timeout=0.3)        # dropped


# ---------------------------------------------------------------- RerankAgentRunnerIT / FLARE
@pytest.fixture()
def herddb():
    from langstream_amd.agents.vector import herddb as h
    srv = h.HerdDBServer().start()
    yield f"jdbc:herddb:server:localhost:{srv.port}"
    srv.stop()


def _datasource(url, extra=""):
    return f"""
configuration:
  resources:
    - type: "datasource"
      name: "JdbcDatasource"
      configuration:
        service: "jdbc"
        driverClass: "herddb.jdbc.Driver"
        url: "{url}"
        user: "sa"
        password: "hdb"
{extra}"""


def _writer(url, tin):
    return {"configuration.yaml": _datasource(url), "module.yaml": f"""
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
          filename TEXT,
          chunk_id int,
          num_tokens int,
          lang TEXT,
          text TEXT,
          embeddings_vector FLOATA,
          PRIMARY KEY (filename, chunk_id));
{_topics(tin)}pipeline:
  - name: "Write"
    type: "vector-db-sink"
    input: {tin}
    id: step1
    configuration:
      datasource: "JdbcDatasource"
      table-name: "documents"
      fields:
        - name: "filename"
          expression: "value.filename"
          primary-key: true
        - name: "chunk_id"
          expression: "value.chunk_id"
          primary-key: true
        - name: "embeddings_vector"
          expression: "fn:toListOfFloat(value.embeddings_vector)"
        - name: "lang"
          expression: "value.language"
        - name: "text"
          expression: "value.text"
        - name: "num_tokens"
          expression: "value.chunk_num_tokens"
"""}


def _write_docs(streaming, url):
    tin = uniq("sink-topic")
    with Run(*streaming, _writer(url, tin)) as r:
        for i in range(10):
            r.produce(tin, json.dumps({"filename": f"doc{i}.pdf", "chunk_id": 1, "embeddings_vector": [i, 2, 3, 4, 5],
                                       "language": "en", "text": f"text{i}", "chunk_num_tokens": 10}))
        runner = r.app.runners[0]
        deadline = time.time() + 20
        while (runner.records_in < 10 or runner.tracker.pending()) and time.time() < deadline:
            time.sleep(0.05)
        assert runner.records_in == 10 and runner.tracker.pending() == 0


def test_simple_rerank(streaming, herddb):
    """RerankAgentRunnerIT.testSimpleRerank: 10 vectors written through vector-db-sink, the
    question's top-20 by cosine from the database, MMR (lambda 0.5, k1 1.5, b 0.7) keeps 8
    in the reference's exact order."""
    _write_docs(streaming, herddb)
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"configuration.yaml": _datasource(herddb), "module.yaml": _topics(tin, tout) + f"""pipeline:
   - name: "convert-to-structure"
     id: "step1"
     type: "document-to-json"
     input: "{tin}"
     configuration:
       text-field: "question"
   - name: "mock-compute-embeddings"
     type: "compute"
     configuration:
       fields:
          - name: "value.question_embeddings"
            expression: "fn:toListOfFloat([1,2,3,4,5])"
   - name: "lookup-related-documents"
     type: "query-vector-db"
     configuration:
       datasource: "JdbcDatasource"
       query: "SELECT text,embeddings_vector FROM documents ORDER BY cosine_similarity(embeddings_vector, CAST(? as FLOAT ARRAY)) DESC LIMIT 20"
       fields:
         - "value.question_embeddings"
       output-field: "value.related_documents"
   - name: "re-rank documents with MMR"
     type: "re-rank"
     output: {tout}
     configuration:
       max: 8
       field: "value.related_documents"
       query-text: "value.question"
       query-embeddings: "value.question_embeddings"
       output-field: "value.related_documents"
       text-field: "record.text"
       embeddings-field: "record.embeddings_vector"
       algorithm: "MMR"
       lambda: 0.5
       k1: 1.5
       b: 0.7
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, "this is a question")
        recs, _ = r.read_all(tout, 1, 20)
        v = as_json(recs[0].value())
        docs = v["related_documents"]
        assert [d["text"] for d in docs] == ["text1", "text9", "text0", "text8", "text7", "text2", "text6", "text3"]
        for d in docs:
            i = float(d["text"][4:])
            assert [float(x) for x in d["embeddings_vector"]] == [i, 2.0, 3.0, 4.0, 5.0]
        assert v["question"] == "this is a question"
        assert [float(x) for x in v["question_embeddings"]] == [1.0, 2.0, 3.0, 4.0, 5.0]


def test_simple_flare(streaming, herddb):
    """FlareControllerAgentRunnerIT.testSimpleFlare: embeddings + vector lookup over a
    loop-over list, a text completion with logprobs, the flare controller looping low
    confidence spans back to flare-loop-input-topic (max-iterations), then the answer."""
    from test_ref_runtime_genai import TEXT_SSE
    _write_docs(streaming, herddb)
    w = FakeHTTP()
    try:
        w.stub("POST", "/openai/deployments/text-embeddings-ada/embeddings?api-version=2023-08-01-preview",
               json_body={"data": [{"embedding": [1.0, 5.4, 8.7, 7, 9], "index": 0, "object": "embedding"}],
                          "model": "text-embedding-ada-002", "object": "list",
                          "usage": {"prompt_tokens": 5, "total_tokens": 5}})
        w.stub("POST", "/openai/deployments/gp-3.5-turbo-instruct/completions?api-version=2023-08-01-preview",
               text=TEXT_SSE)
        extra = f"""    - type: "open-ai-configuration"
      name: "OpenAI Azure configuration"
      configuration:
        url: "{w.url}"
        access-key: "sdòflkjsòlfkj"
        provider: "azure"
"""
        tin, tloop, tout = uniq("input-topic"), uniq("flare-loop-input-topic"), uniq("output-topic")
        files = {"configuration.yaml": _datasource(herddb, extra), "module.yaml": _topics(tin, tloop, tout) + f"""pipeline:
  - name: "init-structure"
    id: "kickstart-chat"
    type: "document-to-json"
    input: "{tin}"
    configuration:
      text-field: "text"
  - name: "kickstart-document-retrieval"
    type: "compute"
    output: "{tloop}"
    configuration:
      fields:
        - name: "value.documents_to_retrieve"
          expression: "fn:listAdd(fn:emptyList(), value.text)"
        - name: "value.related_documents"
          expression: "fn:emptyList()"
  - name: "convert-docs-to-struct"
    id: "flare-loop"
    type: "compute"
    input: "{tloop}"
    configuration:
      fields:
        - name: "value.documents_to_retrieve"
          expression: "fn:listToListOfStructs(value.documents_to_retrieve, 'text')"
        - name: "value.related_documents"
          expression: "fn:emptyList()"
  - name: "compute-embeddings"
    type: "compute-ai-embeddings"
    configuration:
      loop-over: "value.documents_to_retrieve"
      model: "text-embeddings-ada"
      embeddings-field: "record.embeddings"
      text: "{{{{ record.text }}}}"
      flush-interval: 0
  - name: "lookup-related-documents"
    type: "query-vector-db"
    configuration:
      datasource: "JdbcDatasource"
      loop-over: "value.documents_to_retrieve"
      query: |
              SELECT text,embeddings_vector
              FROM documents
              ORDER BY cosine_similarity(embeddings_vector, CAST(? as FLOAT ARRAY)) DESC LIMIT 5
      fields:
        - "record.embeddings"
      output-field: "value.retrieved_documents"
  - name: "add-documents-to-list"
    type: "compute"
    configuration:
        fields:
          - name: "value.related_documents"
            expression: "fn:addAll(value.related_documents, value.retrieved_documents)"
          - name: "value.retrieved_documents"
            expression: "fn:emptyList()"
          - name: "value.documents_to_retrieve"
            expression: "fn:emptyList()"
  - name: "query-the-LLM"
    type: "ai-text-completions"
    configuration:
      model: "gp-3.5-turbo-instruct"
      completion-field: "value.result"
      logprobs: 5
      logprobs-field: "value.tokens"
      max-tokens: 100
      prompt:
          - |
              There is a list of documents that you must use to perform your task.
              Do not provide information that is not related to the provided documents.

              {{{{# value.related_documents}}}}
              {{{{text}}}}
              {{{{/ value.related_documents}}}}

              This is the task:
              {{{{ value.text }}}}

  - name: "ensure-quality-of-result"
    type: "flare-controller"
    configuration:
        tokens-field: "value.tokens.tokens"
        logprobs-field: "value.tokens.logprobs"
        loop-topic: "{tloop}"
        retrieve-documents-field: "value.documents_to_retrieve"
  - name: "cleanup-response"
    type: "compute"
    output: "{tout}"
    configuration:
      fields:
        - name: "value"
          expression: "value.result"
"""}
        with Run(*streaming, files) as r:
            assert sorted(n.id for n in r.plan.agents.values()) == ["flare-loop", "kickstart-chat"]
            r.produce(tin, "this is a question")
            r.wait_for(tout, ["I am an AI language model and I do not have personal experiences or the"], timeout=60)
            completions = [q for q in w.requests if "completions" in q[1]]
            # " language model and" / " the" stay low-confidence on every pass: the record
            # loops max-iterations + 1 = 11 times, then passes (12 completions in all)
            assert len(completions) == 12
            prompt = json.loads(completions[-1][2])["prompt"][0]
            assert "text" in prompt and "this is a question" in prompt
    finally:
        w.close()


# ---------------------------------------------------------------- TextProcessingAgentsRunnerIT
def test_full_language_processing_pipeline(streaming):
    """TextProcessingAgentsRunnerIT.testFullLanguageProcessingPipeline: the Italian text is
    filtered out, the English one split at 50 chars (keep_separator) and normalised."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"module.yaml": 'module: "module-1"\nid: "pipeline-1"\n' + _topics(tin, tout) + f"""pipeline:
  - name: "Extract text"
    type: "text-extractor"
    input: "{tin}"
  - name: "Detect language"
    type: "language-detector"
    configuration:
       allowedLanguages: ["en"]
       property: "language"
  - name: "Split into chunks"
    type: "text-splitter"
    configuration:
      chunk_size: 50
      chunk_overlap: 0
      keep_separator: true
      length_function: "length"
  - name: "Normalise text"
    type: "text-normaliser"
    output: "{tout}"
    configuration:
        make-lowercase: true
        trim-spaces: true
"""}
    with Run(*streaming, files) as r:
        assert [n.id for n in r.plan.agents.values()] == ["module-1-pipeline-1-text-extractor-1"]
        r.produce(tin, "Questo testo è scritto in Italiano.")
        r.produce(tin, "This text is written in English, but it is very long,\nso you may want to split it into chunks.")
        r.wait_for(tout, ["this text is written in english, but it is very", "long,",
                          "so you may want to split it into chunks."])


@pytest.mark.parametrize("intermediate", [False, True])
def test_split_then_json(streaming, intermediate):
    """TextProcessingAgentsRunnerIT.testSplitThenJson: the chunk headers copied into the JSON
    (copy-properties), fused or across an intermediate topic."""
    tin, tout, tmid = uniq("input-topic"), uniq("output-topic"), uniq("intermediate-topic")
    split = ("  - name: \"Split into chunks\"\n    id: step1\n    type: \"text-splitter\"\n    input: %s\n%s"
             "    configuration:\n      chunk_size: 50\n      chunk_overlap: 0\n      keep_separator: true\n"
             "      length_function: \"length\"\n") % (tin, f"    output: {tmid}\n" if intermediate else "")
    to_json = ("  - name: \"Convert chunks to JSON\"\n    type: \"document-to-json\"\n%s    output: %s\n"
               "    configuration:\n        text-field: text\n        copy-properties: true\n") % (
        f"    id: step2\n    input: {tmid}\n" if intermediate else "", tout)
    files = {"module.yaml": 'module: "module-1"\nid: "pipeline-1"\n' + _topics(tin, tout, *([tmid] if intermediate else []))
             + "pipeline:\n" + split + to_json}
    with Run(*streaming, files) as r:
        assert sorted(n.id for n in r.plan.agents.values()) == (["step1", "step2"] if intermediate else ["step1"])
        r.produce(tin, "This text is written in English, but it is very long,\nso you may want to split it into chunks.")
        recs, _ = r.read_all(tout, 3, 20)
        assert [as_json(x.value()) for x in recs] == [
            {"chunk_text_length": "47", "text": "This text is written in English, but it is very", "text_num_chunks": "3",
             "chunk_id": "0", "chunk_num_tokens": "47"},
            {"chunk_text_length": "5", "text": "long,", "text_num_chunks": "3", "chunk_id": "1",
             "chunk_num_tokens": "5"},
            {"chunk_text_length": "40", "text": "so you may want to split it into chunks.", "text_num_chunks": "3",
             "chunk_id": "2", "chunk_num_tokens": "40"}]


# ---------------------------------------------------------------- KafkaSchemaTest
def test_use_schema_with_kafka(kafka):
    """KafkaSchemaTest.testUseSchemaWithKafka: an Avro record (Confluent wire format, schema
    registry) through identity keeps its schema; the output decodes to the same record."""
    from langstream_amd.api.avro import AvroSchema, wire_decode, wire_encode
    from langstream_amd.topics.kafka.client import KafkaClient, PartitionReader, Producer
    from langstream_amd.topics.kafka.schema_registry import SchemaRegistryClient, SchemaRegistryServer
    schema = {"type": "record", "name": "Pojo", "namespace": "mynamespace",
              "fields": [{"name": "name", "type": "string"}]}
    reg = SchemaRegistryServer()
    try:
        tin, tout = uniq("input-topic"), uniq("output-topic")
        files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
    schema:
      type: avro
      schema: '{json.dumps(schema)}'
  - name: "{tout}"
    creation-mode: create-if-not-exists
    schema:
      type: avro
      schema: |
           {json.dumps(schema)}
pipeline:
  - name: "identity"
    id: "step1"
    type: "identity"
    input: "{tin}"
    output: "{tout}"
"""}
        with Run("kafka", kafka.bootstrap, files, extra_admin={"schema.registry.url": reg.url}):
            sr = SchemaRegistryClient(reg.url)
            sid = sr.register(f"{tin}-value", schema)
            c = KafkaClient(kafka.bootstrap)
            Producer(c, tin).send_many([(None, wire_encode(sid, schema, {"name": "foo"}), [], int(time.time() * 1000))])
            got = []
            rd = PartitionReader(c, tout, start="earliest")
            deadline = time.time() + 20
            while not got and time.time() < deadline:
                got = rd.read(10)
            assert got, "no output record"
            value = got[0][4]
            out_id = int.from_bytes(value[1:5], "big")
            assert value[0] == 0 and sr.get_by_id(out_id) == AvroSchema(schema)
            assert wire_decode(value, lambda i: schema if i == out_id else None) == {"name": "foo"}
            c.close()
    finally:
        reg.close()
