"""Kafka Connect adapters (agent types ``source`` / ``sink``, KRT/kafkaconnect/*): the
Kafka-bundled FileStream connectors run as Python connectors; the sink handles its own
commits (records are committed only after the task's pre_commit acknowledged them)."""
import os
import time

import pytest

from langstream_amd.runtime.local import LocalApplicationRunner
from langstream_amd.topics.memory import reset_memlogs

REF_EX = "/root/reference/examples/applications"

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
        load_connector("io.confluent.connect.jdbc.JdbcSinkConnector")


def test_reference_kafka_connect_example_writes_to_cassandra(tmp_path):
    """The reference's examples/applications/kafka-connect app, unchanged (its
    pipeline.yaml + configuration.yaml + secrets shape), on the in-tree broker-less memory
    log, writing through the built-in CassandraSinkConnector to the fake CQL server of
    test_cassandra.py via a secure-connect bundle that points at it."""
    import io
    import json as _json
    import shutil
    import zipfile
    from tests.test_cassandra import FakeCassandra
    from langstream_amd.api.record import SimpleRecord
    from langstream_amd.runtime.local import LocalApplicationRunner
    if not os.path.isdir(os.path.join(REF_EX, "kafka-connect")):
        pytest.skip("reference checkout not present")
    cass = FakeCassandra(user="token", password="AstraCS:xyz")
    try:
        cass._run("CREATE KEYSPACE IF NOT EXISTS vsearch WITH replication = {'class': 'SimpleStrategy'}", [], [None])
        cass._run("CREATE TABLE IF NOT EXISTS vsearch.products (id int, name text, description text, "
                  "PRIMARY KEY (id))", [], [None])
        bundle = tmp_path / "secure-connect-db.zip"
        with zipfile.ZipFile(bundle, "w") as z:
            z.writestr("config.json", _json.dumps({"host": "127.0.0.1", "cql_port": cass.port, "keyspace": "vsearch"}))
        app = tmp_path / "app"
        shutil.copytree(os.path.join(REF_EX, "kafka-connect"), app)
        secrets = ("secrets:\n  - id: cassandra\n    data:\n      username: token\n      password: AstraCS:xyz\n"
                   f"      secure-connect-bundle: {bundle}\n")
        instance = "instance:\n  streamingCluster:\n    type: memory\n  computeCluster:\n    type: none\n"
        (tmp_path / "instance.yaml").write_text(instance)
        (tmp_path / "secrets.yaml").write_text(secrets)
        r = LocalApplicationRunner.from_directory(str(app), str(tmp_path / "instance.yaml"),
                                                  str(tmp_path / "secrets.yaml"))
        node = next(iter(r.plan.agents.values()))
        node.configuration.setdefault("adapterConfig", {})["lingerTimeMs"] = 50
        r.start()
        try:
            prod = r.topic_runtime.create_producer("test", None, {"topic": "input-topic"})
            prod.start()
            for i in range(5):
                prod.write(SimpleRecord.of(None, _json.dumps({"id": i, "name": f"n{i}", "description": f"d{i}"}))) \
                    .result(5)
            deadline = time.time() + 20
            rows = {}
            while time.time() < deadline and len(rows) < 5:
                rows = cass.keyspaces["vsearch"]["products"]["rows"]
                time.sleep(0.05)
            assert sorted(v["id"] for v in rows.values()) == list(range(5))
            assert rows[(3,)] == {"id": 3, "description": "d3", "name": "n3"}
            assert not r.errors
        finally:
            r.stop()
    finally:
        cass.close()
