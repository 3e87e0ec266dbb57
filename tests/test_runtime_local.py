"""End-to-end runtime on CPU: parse -> plan -> deploy memory topics -> AgentRunner
threads, with the GenAI host steps, python agents and the error policies.

Mirrors the reference's in-process runner tests (AbstractApplicationRunner
subclasses such as ErrorHandlingTest, PythonAgentsIT-style processors, ComputeStepTest)."""
import json
import os
import textwrap
import uuid

import pytest

from langstream_amd.runtime.local import LocalApplicationRunner
from langstream_amd.topics.memory import reset_memlogs


@pytest.fixture(autouse=True)
def _fresh_topics():
    reset_memlogs()
    yield
    reset_memlogs()


def _t():
    return "t" + uuid.uuid4().hex[:8]


def _values(records):
    out = []
    for r in records:
        v = r.value()
        if isinstance(v, (bytes, str)):
            try:
                v = json.loads(v)
            except ValueError:
                pass
        out.append(v)
    return out


def test_compute_and_drop_fields_pipeline():
    tin, tout = _t(), _t()
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: drop
    type: drop-fields
    input: {tin}
    configuration:
      fields: ["secret"]
  - name: compute
    type: compute
    output: {tout}
    configuration:
      fields:
        - name: "value.total"
          expression: "value.a + value.b"
        - name: "value.shout"
          expression: "fn:uppercase(value.name)"
        - name: "properties.kind"
          expression: "'sum'"
"""
    with LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}) as app:
        app.produce(tin, json.dumps({"a": 2, "b": 3, "name": "bob", "secret": "x"}))
        recs = app.consume(tout, 1, timeout=20)
    assert len(recs) == 1
    v = _values(recs)[0]
    assert v == {"a": 2, "b": 3, "name": "bob", "total": 5, "shout": "BOB"}
    assert recs[0].header_value("kind") == "sum"


def _user_code(tmp_path, body: str) -> str:
    d = tmp_path / "python"
    d.mkdir(parents=True, exist_ok=True)
    mod = "userproc_" + uuid.uuid4().hex[:6]
    (d / f"{mod}.py").write_text(textwrap.dedent(body))
    return mod


FAILING = """
from langstream import SimpleRecord

class Proc:
    def process(self, record):
        if record.value() == "bad":
            raise ValueError("bad record")
        return [SimpleRecord(record.value() + "!")]
"""


@pytest.mark.parametrize("policy", ["skip", "dead-letter"])
def test_error_policies(tmp_path, policy):
    tin, tout = _t(), _t()
    mod = _user_code(tmp_path, FAILING)
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: proc
    type: python-processor
    input: {tin}
    output: {tout}
    errors:
      on-failure: {policy}
      retries: 1
    configuration:
      className: {mod}.Proc
"""
    with LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, code_directory=str(tmp_path)) as app:
        for v in ("a", "bad", "b"):
            app.produce(tin, v)
        out = app.consume(tout, 2, timeout=20)
        assert sorted(_values(out)) == ["a!", "b!"]
        if policy == "dead-letter":
            dl = app.consume(tin + "-deadletter", 1, timeout=20)
            assert _values(dl) == ["bad"]
            assert dl[0].header_value("error-msg") is not None or dl[0].header_value("cause-msg") is not None


def test_fail_policy_stops_agent(tmp_path):
    tin, tout = _t(), _t()
    mod = _user_code(tmp_path, FAILING)
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: proc
    type: python-processor
    input: {tin}
    output: {tout}
    errors:
      on-failure: fail
      retries: 0
    configuration:
      className: {mod}.Proc
"""
    app = LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}, code_directory=str(tmp_path)).start()
    try:
        app.produce(tin, "bad")
        with pytest.raises(Exception):
            app.consume(tout, 1, timeout=10)
    finally:
        app.stop(5)


def test_text_splitter_and_document_to_json():
    tin, tout = _t(), _t()
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: split
    type: text-splitter
    input: {tin}
    configuration:
      chunk_size: 40
      chunk_overlap: 0
      length_function: length
  - name: tojson
    type: document-to-json
    output: {tout}
    configuration:
      text-field: text
"""
    text = "The quick brown fox jumps over the lazy dog. " * 4
    with LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}) as app:
        app.produce(tin, text)
        recs = app.consume(tout, 4, timeout=20)
    vals = _values(recs)
    assert len(vals) >= 4
    assert all(isinstance(v, dict) and "text" in v for v in vals)
    assert all(len(v["text"]) <= 40 for v in vals)
    assert recs[0].header_value("chunk_id") is not None
