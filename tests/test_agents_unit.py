"""Agent-level unit tests (CPU): the expression language, mustache templates, the GenAI
host steps, text processing, flow control, re-rank, FLARE, chunk coalescing, ordered
batching and ordered commits.

Mirrors the reference's per-agent unit suites: JstlEvaluatorTest /
JstlFunctionsTest, the TransformFunction step tests (ComputeStepTest, DropFieldsTest,
FlattenStepTest, CastStepTest, MergeKeyValueStepTest, UnwrapKeyValueStepTest),
TextSplitterAgentTest, DispatchAgentTest, ReRankAgentTest, FlareControllerAgentTest,
OrderedAsyncBatchExecutorTest and SourceRecordTrackerTest."""
import json
import threading
import time

import numpy as np
import pytest

from langstream_amd.agents.genai.el import eval_expression, eval_predicate
from langstream_amd.agents.genai.mustache import render
from langstream_amd.agents.genai.mutable import MutableRecord
from langstream_amd.agents.genai.services import ChunkCoalescer
from langstream_amd.api.record import Header, SimpleRecord, SourceRecordAndResult
from langstream_amd.api.util import OrderedAsyncBatchExecutor
from langstream_amd.runtime.registry import create_agent
from langstream_amd.runtime.tracker import SourceRecordTracker


def _ctx(value, key=None, props=None):
    rec = SimpleRecord.of(key, json.dumps(value) if isinstance(value, (dict, list)) else value,
                          [Header(k, v) for k, v in (props or {}).items()])
    return MutableRecord.from_record(rec).el_context()


def _run(agent_type, config, records, timeout=10):
    a = create_agent(agent_type)
    a.init(config)
    a.start()
    out, done = [], threading.Event()

    def sink(r):
        out.append(r)
        if len(out) >= len(records):
            done.set()

    a.process(records, sink)
    assert done.wait(timeout), f"{agent_type}: {len(out)}/{len(records)} results"
    a.close()
    return out


def _j(v):
    return json.loads(v) if isinstance(v, (str, bytes)) else v


def _vals(result):
    assert result.error is None, result.error
    out = []
    for r in result.result_records:
        v = r.value()
        try:
            v = json.loads(v) if isinstance(v, str) else v
        except ValueError:
            pass
        out.append(v)
    return out


# ------------------------------------------------------------------ expression language
@pytest.mark.parametrize("expr,expected", [
    ("value.a + value.b", 5),
    ("value.a * 2 - 1", 3),
    ("value.b / 2", 1.5),
    ("value.b % 2", 1),
    ("value.a < value.b && value.b <= 3", True),
    ("value.a == 2 ? 'two' : 'other'", "two"),
    ("not empty value.s and value.s eq 'hi'", True),
    ("empty value.missing", True),
    ("fn:concat(value.s, '-', key)", "hi-k"),
    ("fn:uppercase(value.s)", "HI"),
    ("fn:split('a,b,c', ',')", ["a", "b", "c"]),
    ("fn:toInt('42') + 1", 43),
    ("fn:toDouble('2.5')", 2.5),
    ("fn:length(value.l)", 3),
    ("fn:coalesce(value.missing, 'dflt')", "dflt"),
    ("fn:replace('a-b-c', '-', '+')", "a+b+c"),
    ("fn:contains(value.s, 'h')", True),
    ("fn:fromJson('{\"x\": 1}').x", 1),
    ("fn:toJson(value.l)", "[1, 2, 3]"),
    ("fn:listAdd(fn:listOf(1, 2), 3)", [1, 2, 3]),
    ("fn:mapPut(fn:mapOf('a', 1), 'b', 2)", {"a": 1, "b": 2}),
    ("fn:mapRemove(fn:mapOf('a', 1, 'b', 2), 'a')", {"b": 2}),
    ("fn:toListOfFloat(value.l)", [1.0, 2.0, 3.0]),
    ("fn:trim('  x ')", "x"),
    ("properties.p1", "v1"),
])
def test_el_expressions(expr, expected):
    ctx = _ctx({"a": 2, "b": 3, "s": "hi", "l": [1, 2, 3]}, key="k", props={"p1": "v1"})
    got = eval_expression(expr, ctx)
    if isinstance(expected, str) and expected.startswith("["):
        assert json.loads(got) == json.loads(expected)
    else:
        assert got == expected


def test_el_filter_and_timestamps():
    ctx = _ctx({"docs": [{"s": 0.9, "t": "a"}, {"s": 0.1, "t": "b"}]})
    assert eval_expression("fn:filter(value.docs, 'record.s > 0.5')", ctx) == [{"s": 0.9, "t": "a"}]
    assert eval_expression("fn:timestampAdd(1000, 2, 'seconds')", ctx) == 3000
    assert eval_predicate("value.docs[0].s > 0.5", ctx) is True
    assert eval_predicate(None, ctx) is True
    u1, u2 = eval_expression("fn:uuid()", ctx), eval_expression("fn:uuid()", ctx)
    assert u1 != u2 and len(u1) == 36


# ------------------------------------------------------------------ mustache
def test_mustache_sections_and_escaping():
    ctx = {"value": {"q": "a<b", "docs": [{"text": "one"}, {"text": "two"}], "empty": []}}
    assert render("{{ value.q }}", ctx) == "a&lt;b"
    assert render("{{{ value.q }}}", ctx) == "a<b"
    assert render("{{# value.docs}}[{{ text}}]{{/ value.docs}}", ctx) == "[one][two]"
    assert render("{{^ value.empty}}none{{/ value.empty}}", ctx) == "none"
    assert render("x{{ value.missing }}y", ctx) == "xy"


# ------------------------------------------------------------------ GenAI host steps
def _step(step, records):
    return _run("ai-tools", {"steps": [step]}, records)


def test_compute_step_types_and_destinations():
    r = SimpleRecord.of("k", json.dumps({"n": "7", "f": 1.5}))
    res = _step({"type": "compute", "fields": [
        {"name": "value.n_int", "expression": "fn:toInt(value.n)", "type": "INT32"},
        {"name": "value.s", "expression": "value.f", "type": "STRING"},
        {"name": "properties.flag", "expression": "true", "type": "BOOLEAN"},
        {"name": "key", "expression": "fn:concat('new-', key)"}]}, [r])[0]
    out = res.result_records[0]
    v = json.loads(out.value()) if isinstance(out.value(), str) else out.value()
    assert v["n_int"] == 7 and v["s"] == "1.5"
    assert out.key() == "new-k"
    assert {h.key: h.value for h in out.headers()}["flag"] == "true"


def test_drop_fields_flatten_merge_unwrap():
    r = SimpleRecord.of(json.dumps({"id": 1}), json.dumps({"a": {"b": 1, "c": {"d": 2}}, "x": 1, "y": 2}))
    assert _vals(_step({"type": "drop-fields", "fields": ["x", "y"]}, [r])[0]) == [{"a": {"b": 1, "c": {"d": 2}}}]
    flat = _vals(_step({"type": "flatten"}, [r])[0])[0]
    assert flat == {"a_b": 1, "a_c_d": 2, "x": 1, "y": 2}
    flat2 = _vals(_step({"type": "flatten", "delimiter": "."}, [r])[0])[0]
    assert "a.c.d" in flat2
    merged = _vals(_step({"type": "merge-key-value"}, [r])[0])[0]
    assert merged["id"] == 1 and merged["x"] == 1
    # unwrap-key-value drops the key (UnwrapKeyValueStep.java), unwrap-key moves it to the value
    kv = SimpleRecord.of(json.dumps({"id": 5}), json.dumps({"v": 1}))
    out = _step({"type": "unwrap-key-value"}, [kv])[0].result_records[0]
    assert out.key() is None and _j(out.value()) == {"v": 1}
    out = _step({"type": "unwrap-key-value", "unwrap-key": True}, [kv])[0].result_records[0]
    assert _j(out.value()) == {"id": 5}


def test_drop_step_when_and_cast():
    recs = [SimpleRecord.of(None, json.dumps({"n": i})) for i in range(4)]
    res = _step({"type": "drop", "when": "value.n % 2 == 0"}, recs)
    kept = [json.loads(r.result_records[0].value())["n"] for r in res if r.result_records]
    assert sorted(kept) == [1, 3]
    cast = _step({"type": "cast", "schema-type": "string"}, [SimpleRecord.of(None, json.dumps({"n": 1}))])[0]
    assert isinstance(cast.result_records[0].value(), str)


# ------------------------------------------------------------------ text processing
def test_text_splitter_chunks_overlap_and_headers():
    text = " ".join(f"w{i}" for i in range(120))
    res = _run("text-splitter", {"chunk_size": 50, "chunk_overlap": 10, "length_function": "length"},
               [SimpleRecord.of("doc", text)])[0]
    chunks = res.result_records
    assert len(chunks) > 3
    hdr = [{h.key: h.value for h in c.headers()} for c in chunks]
    assert all(c.key() == "doc" for c in chunks)
    assert [int(h["chunk_id"]) for h in hdr] == list(range(len(chunks)))
    assert all(int(h["text_num_chunks"]) == len(chunks) for h in hdr)
    assert all(len(c.value()) <= 50 for c in chunks)
    # consecutive chunks overlap
    assert chunks[0].value().split()[-1] in chunks[1].value()
    joined = " ".join(c.value() for c in chunks)
    assert all(f"w{i}" in joined for i in range(120))


def test_text_normaliser_document_to_json_language_extractor():
    out = _run("text-normaliser", {"make-lowercase": True, "trim-spaces": True},
               [SimpleRecord.of(None, "  Hello   World  ")])[0]
    assert out.result_records[0].value() in ("hello world", "hello   world")
    d2j = _run("document-to-json", {"text-field": "question", "copy-properties": True},
               [SimpleRecord.of(None, "what?", [Header("h", "1")])])[0].result_records[0]
    v = json.loads(d2j.value()) if isinstance(d2j.value(), str) else d2j.value()
    assert v["question"] == "what?"
    lang = _run("language-detector", {"property": "language"},
                [SimpleRecord.of(None, "The quick brown fox jumps over the lazy dog and then it runs away")])[0]
    assert {h.key: h.value for h in lang.result_records[0].headers()}["language"] == "en"
    html = _run("text-extractor", {}, [SimpleRecord.of(None, b"<html><body><h1>Title</h1><p>Body text</p>"
                                                            b"<script>x()</script></body></html>")])[0]
    txt = html.result_records[0].value()
    assert "Title" in txt and "Body text" in txt and "x()" not in txt


# ------------------------------------------------------------------ re-rank / flare
def test_rerank_mmr_prefers_relevant_then_diverse():
    docs = [{"text": "cats are small furry animals", "embeddings": [1.0, 0.0, 0.0]},
            {"text": "cats are small furry pets", "embeddings": [0.99, 0.01, 0.0]},
            {"text": "dogs bark loudly at night", "embeddings": [0.0, 1.0, 0.0]},
            {"text": "quantum chromodynamics", "embeddings": [0.0, 0.0, 1.0]}]
    rec = SimpleRecord.of(None, json.dumps({"q": "small furry cats", "docs": docs}))
    cfg = {"field": "value.docs", "output-field": "value.ranked", "query-text": "value.q",
           "text-field": "record.text", "embeddings-field": "record.embeddings", "max": 2, "lambda": 0.5,
           "algorithm": "MMR"}
    ranked = _vals(_run("re-rank", cfg, [rec])[0])[0]["ranked"]
    assert len(ranked) == 2
    assert "cats" in ranked[0]["text"]
    # algorithm none keeps the whole list in order (ReRankAgent.java:148-149)
    none = _vals(_run("re-rank", dict(cfg, algorithm="none", max=3), [rec])[0])[0]["ranked"]
    assert [d["text"] for d in none] == [d["text"] for d in docs]


def test_flare_low_confidence_spans():
    from langstream_amd.agents.flare import low_confidence_spans
    toks = ["The", " cap", "ital", " of", " Mars", " is", " Olympus", "."]
    lps = [-0.01, -0.02, -0.01, -0.05, -3.0, -0.1, -4.0, -0.01]
    spans = low_confidence_spans(toks, lps, 0.2, 5, 2)
    assert spans and all(isinstance(s, str) for s in spans)
    assert any("Mars" in s for s in spans)
    assert low_confidence_spans(toks, [-0.01] * len(toks), 0.2, 5, 2) == []


# ------------------------------------------------------------------ flow control
class _FakeProducer:
    def __init__(self):
        self.records = []

    def start(self):
        pass

    def write(self, r):
        from concurrent.futures import Future
        self.records.append(r)
        f = Future()
        f.set_result(None)
        return f

    def close(self):
        pass


class _Ctx:
    def __init__(self):
        self.producers = {}

    def get_topic_producer(self, topic):
        return self.producers.setdefault(topic, _FakeProducer())

    def __getattr__(self, name):
        raise AttributeError(name)


def test_dispatch_routes_and_drops(monkeypatch):
    import langstream_amd.agents.flow as flow
    prods = {}
    monkeypatch.setattr(flow, "_producer", lambda agent, topic: prods.setdefault(topic, _FakeProducer()))
    recs = [SimpleRecord.of(None, json.dumps({"lang": l})) for l in ("en", "fr", "de")]
    cfg = {"routes": [{"when": "value.lang == 'en'", "destination": "english"},
                      {"when": "value.lang == 'de'", "action": "drop"}]}
    a = create_agent("dispatch")
    a.init(cfg)
    a.start()
    out = []
    a.process(recs, out.append)
    deadline = time.time() + 5
    while len(out) < 3 and time.time() < deadline:
        time.sleep(0.01)
    by = {json.loads(r.source_record.value())["lang"]: r for r in out}
    assert by["de"].result_records == []
    fr = by["fr"].result_records
    assert len(fr) == 1
    # routed records go to the destination topic's producer, not downstream
    assert by["en"].result_records == []
    assert [json.loads(r.value())["lang"] for r in prods["english"].records] == ["en"]


# ------------------------------------------------------------------ runtime utilities
def test_chunk_coalescer_doubles_up_to_min_chunks():
    sent = []
    co = ChunkCoalescer(lambda aid, idx, text, last: sent.append((idx, text, last)), 4, "a1")
    for i in range(12):
        co.accept(str(i % 10), i == 11)
    sizes = [len(t) for _, t, _ in sent]
    assert sizes[:3] == [1, 2, 4] and all(s <= 4 for s in sizes)
    assert sent[-1][2] is True and "".join(t for _, t, _ in sent) == "".join(str(i % 10) for i in range(12))
    assert [i for i, _, _ in sent] == list(range(1, len(sent) + 1))


def test_ordered_async_batch_executor_keeps_per_key_order():
    seen, lock = [], threading.Lock()

    def proc(batch, fut):
        def later():
            time.sleep(0.001 * (len(batch) % 3))
            with lock:
                seen.extend(batch)
            fut.set_result(None)
        threading.Thread(target=later).start()

    ex = OrderedAsyncBatchExecutor(3, proc, 0, 4, lambda item: hash(item[0]))
    ex.start()
    for i in range(60):
        ex.add((f"k{i % 5}", i))
    ex.stop()
    deadline = time.time() + 5
    while len(seen) < 60 and time.time() < deadline:
        time.sleep(0.01)
    for k in range(5):
        idx = [i for kk, i in seen if kk == f"k{k}"]
        assert idx == sorted(idx) and len(idx) == 12


def test_source_record_tracker_commits_in_source_order():
    committed = []

    class Src:
        def commit(self, recs):
            committed.extend(r.value() for r in recs)

    t = SourceRecordTracker(Src())
    s = [SimpleRecord.of(None, f"s{i}") for i in range(3)]
    outs = [[SimpleRecord.of(None, f"o{i}{j}") for j in range(n)] for i, n in enumerate((2, 1, 0))]
    t.track([SourceRecordAndResult(s[i], outs[i], None) for i in range(3)])
    t.commit([outs[1][0]])                     # s1 done, but s0 is still pending
    assert committed == []
    t.commit([outs[0][0]])
    assert committed == []
    t.commit([outs[0][1]])                     # s0 done -> s0, s1 and the empty-fan-out s2 commit
    assert committed == ["s0", "s1", "s2"] and t.pending() == 0


def test_gctune_freezes_startup_heap(monkeypatch):
    import gc
    from langstream_amd.utils import gctune
    old = gc.get_threshold()
    monkeypatch.setattr(gctune, "_done", False)
    monkeypatch.setenv("LANGSTREAM_GC", "default")
    assert gctune.tune() is False and gc.get_threshold() == old
    monkeypatch.setenv("LANGSTREAM_GC", "tuned")
    try:
        assert gctune.tune() is True
        assert gc.get_threshold() == (50_000, 20, 100) and gc.get_freeze_count() > 0
        assert gctune.tune() is False   # once per process
    finally:
        gc.unfreeze()
        gc.set_threshold(*old)
