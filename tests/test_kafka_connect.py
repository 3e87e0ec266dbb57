"""Kafka Connect adapters (agent types ``source`` / ``sink``, KRT/kafkaconnect/*): the
Kafka-bundled FileStream connectors run as Python connectors; the sink handles its own
commits (records are committed only after the task's pre_commit acknowledged them)."""
import time

import pytest

from langstream_amd.runtime.local import LocalApplicationRunner
from langstream_amd.topics.memory import reset_memlogs

APP = """
topics:
  - name: "connect-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "file-source"
    id: "src"
    type: "source"
    output: "connect-topic"
    configuration:
      connector.class: org.apache.kafka.connect.file.FileStreamSourceConnector
      file: "{inp}"
      batch.size: 10
  - name: "file-sink"
    id: "snk"
    type: "sink"
    input: "connect-topic"
    configuration:
      connector.class: org.apache.kafka.connect.file.FileStreamSinkConnector
      file: "{out}"
      adapterConfig:
        batchSize: 7
        lingerTimeMs: 50
"""


@pytest.fixture(autouse=True)
def _fresh():
    reset_memlogs()
    yield
    reset_memlogs()


def test_file_source_to_file_sink(tmp_path):
    inp, out = tmp_path / "in.txt", tmp_path / "out.txt"
    inp.write_text("".join(f"line {i}\n" for i in range(25)))
    r = LocalApplicationRunner.from_yaml({"pipeline.yaml": APP.format(inp=inp, out=out)}, application_id="kc")
    r.start()
    try:
        deadline = time.time() + 20
        while time.time() < deadline:
            if out.exists() and len(out.read_text().splitlines()) >= 25:
                break
            if r.errors:
                raise r.errors[0]
            time.sleep(0.05)
        assert out.read_text().splitlines() == [f"line {i}" for i in range(25)]
        # the sink committed through the consumer once pre_commit acknowledged the batches
        log = r.topic_runtime.log
        deadline = time.time() + 5
        while time.time() < deadline and log.committed("connect-topic", "langstream-agent-snk") != [25]:
            time.sleep(0.05)
        assert log.committed("connect-topic", "langstream-agent-snk") == [25]
        info = r.agent_info()
        assert any(s.get("info", {}).get("connector.class", "").endswith("FileStreamSinkConnector")
                   for v in info.values() for s in v)
    finally:
        r.stop()


def test_unknown_java_connector_fails_clearly(tmp_path):
    from langstream_amd.agents.kafka_connect import load_connector
    with pytest.raises(ValueError, match="Java connectors cannot run"):
        load_connector("com.datastax.oss.kafka.sink.CassandraSinkConnector")
