"""Local vector store: explicit limits (k > 64, dims without a kernel), batched deletes,
WAL + snapshot persistence, and a kill -9 / restart of an ingest pipeline on shared-
memory topics that must lose no chunk (write-ahead of upserts relative to the offset
commit; parity: VEC/jdbc/JdbcWriter.java:33-208 persists before the commit)."""
import os
import signal
import subprocess
import sys
import textwrap
import time
import uuid

import numpy as np
import pytest
import torch

from langstream_amd.engine.vector_store import VectorStore, VectorStoreRegistry

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _brute(vecs, q, k):
    X = torch.nn.functional.normalize(torch.tensor(vecs, dtype=torch.float32), dim=-1)
    qq = torch.nn.functional.normalize(torch.tensor(q, dtype=torch.float32), dim=-1)
    return torch.topk(qq @ X.t(), k, dim=-1).indices.tolist()


def test_k_above_64_is_exact_not_clamped():
    g = torch.Generator().manual_seed(0)
    vecs = torch.randn(500, 64, generator=g).tolist()
    s = VectorStore(64, device="cpu", dtype=torch.float32)
    s.upsert(list(range(500)), vecs)
    q = torch.randn(3, 64, generator=g).tolist()
    res = s.search(q, 100)
    assert all(len(r) == 100 for r in res)
    assert [[d["id"] for d in r] for r in res] == _brute(vecs, q, 100)


def test_dim_without_kernel_instantiation_works():
    s = VectorStore(100, device="cpu", dtype=torch.float32)
    assert not s.kernel_dim
    g = torch.Generator().manual_seed(1)
    vecs = torch.randn(50, 100, generator=g).tolist()
    s.upsert([f"r{i}" for i in range(50)], vecs)
    res = s.search([vecs[7]], 3)[0]
    assert res[0]["id"] == "r7" and abs(res[0]["similarity"] - 1.0) < 1e-5
    with pytest.raises(ValueError):
        s.upsert(["bad"], [[0.0] * 99])


def test_batched_delete_keeps_dense_rows_consistent():
    g = torch.Generator().manual_seed(2)
    vecs = torch.randn(40, 32, generator=g)
    s = VectorStore(32, device="cpu", dtype=torch.float32)
    s.upsert(list(range(40)), vecs.tolist(), [{"i": i} for i in range(40)])
    dead = [0, 3, 39, 38, 20, 21, 22, 7, 999]
    assert s.delete(dead) == 8
    alive = [i for i in range(40) if i not in dead]
    assert len(s) == len(alive)
    for i in alive:  # every survivor is still found as its own nearest neighbour
        r = s.search([vecs[i].tolist()], 1)[0][0]
        assert r["id"] == i and r["i"] == i
    # duplicate ids in one upsert: last wins
    s.upsert([1, 1], [vecs[5].tolist(), vecs[6].tolist()], [{"v": 5}, {"v": 6}])
    assert s.get(1) == {"v": 6}


def test_search_redoes_payloads_when_a_delete_renumbers_rows(monkeypatch):
    """A search enqueues its top-k under the store lock and waits for it outside; a
    delete landing in that window renumbers rows, so the search must resolve its row
    numbers again instead of returning the payloads of the rows that moved in."""
    import langstream_amd.engine.vector_store as vs
    g = torch.Generator().manual_seed(3)
    vecs = torch.randn(30, 32, generator=g)
    s = VectorStore(32, device="cpu", dtype=torch.float32)
    s.upsert(list(range(30)), vecs.tolist(), [{"i": i} for i in range(30)])
    real = vs.to_host_async
    calls = {"n": 0}

    def racing(*t):
        calls["n"] += 1
        out = real(*t)
        if calls["n"] == 1:
            s.delete([0, 1, 2])   # another thread's delete between top-k and payloads
        return out

    topk = {"n": 0}
    real_topk = s.topk_rows

    def counted(*a):
        topk["n"] += 1
        return real_topk(*a)

    monkeypatch.setattr(vs, "to_host_async", racing)
    monkeypatch.setattr(s, "topk_rows", counted)
    res = s.search([vecs[25].tolist(), vecs[0].tolist()], 3, with_vectors=True)
    assert topk["n"] == 2   # the top-k ran again after the renumbering
    assert res[0][0]["id"] == 25 and res[0][0]["i"] == 25
    assert all(d["id"] == d["i"] and d["id"] not in (0, 1, 2) for r in res for d in r)
    assert np.allclose(res[0][0]["vector"], torch.nn.functional.normalize(vecs[25], dim=0).numpy(), atol=1e-6)


def test_wal_and_snapshot_restore(tmp_path):
    d = str(tmp_path / "coll")
    g = torch.Generator().manual_seed(3)
    vecs = torch.randn(30, 16, generator=g)
    s = VectorStore(16, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    s.upsert(list(range(20)), vecs[:20].tolist(), [{"t": str(i)} for i in range(20)])
    s.delete([2, 4])
    s.snapshot()                                   # compaction point
    s.upsert(list(range(20, 30)), vecs[20:].tolist(), [{"t": str(i)} for i in range(20, 30)])
    s.delete([25])
    s.upsert(["x"], [vecs[0].tolist()], [{"t": "x"}])
    s.close()
    r = VectorStore(16, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    assert len(r) == 28
    assert r.get(3) == {"t": "3"} and r.get(2) is None and r.get(25) is None and r.get("x") == {"t": "x"}
    assert r.search([vecs[27].tolist()], 1)[0][0]["id"] == 27


def test_registry_restores_collection_after_restart(tmp_path):
    VectorStoreRegistry.reset()
    VectorStoreRegistry.configure(persist_dir=str(tmp_path))
    try:
        VectorStoreRegistry.get("docs", 8, device="cpu").upsert(["a"], [[1.0] * 8], [{"text": "hello"}])
        VectorStoreRegistry.reset()                   # "process restart"
        assert VectorStoreRegistry.exists("docs")
        assert VectorStoreRegistry.get("docs", device="cpu").get("a") == {"text": "hello"}
        VectorStoreRegistry.drop("docs", purge=True)
        assert not VectorStoreRegistry.exists("docs")
    finally:
        VectorStoreRegistry.reset()
        VectorStoreRegistry.persist_dir = None


def test_query_agent_created_before_sink_becomes_durable(tmp_path, caplog):
    """a collection created (empty, non-persistent) by a query agent before the
    sink configures persistence is attached to the WAL when persistence is configured;
    one that already holds rows is reported as not durable."""
    VectorStoreRegistry.reset()
    VectorStoreRegistry.persist_dir = None
    try:
        q = VectorStoreRegistry.get("docs", 8, device="cpu")           # the query agent, first
        early = VectorStoreRegistry.get("early", 8, device="cpu")
        early.upsert(["x"], [[1.0] * 8])
        assert not q.persistent
        with caplog.at_level("WARNING"):
            VectorStoreRegistry.configure(persist_dir=str(tmp_path))   # the sink's set_context
        assert q.persistent and not early.persistent
        assert any("early" in r.getMessage() and "NOT durable" in r.getMessage() for r in caplog.records)
        q.upsert(["a"], [[1.0] * 8], [{"text": "kept"}])
        VectorStoreRegistry.reset()                                      # "process restart"
        assert VectorStoreRegistry.get("docs", device="cpu").get("a") == {"text": "kept"}
    finally:
        VectorStoreRegistry.reset()
        VectorStoreRegistry.persist_dir = None


WORKER = textwrap.dedent('''
    import sys, time
    sys.path.insert(0, {root!r})
    from langstream_amd.runtime.local import LocalApplicationRunner
    APP = """
    topics:
      - name: "chunks"
        creation-mode: create-if-not-exists
        partitions: 2
    pipeline:
      - name: "write"
        id: "write"
        type: "vector-db-sink"
        input: "chunks"
        configuration:
          datasource: "LocalVectors"
          collection-name: "docs"
          fields:
            - name: "id"
              expression: "key"
            - name: "vector"
              expression: "value.vec"
            - name: "text"
              expression: "value.text"
    """
    CONF = """
    configuration:
      resources:
        - type: "vector-database"
          name: "LocalVectors"
          configuration:
            service: "local"
            persist-directory: "{store}"
    """
    INSTANCE = """
    instance:
      streamingCluster:
        type: "shm"
        configuration:
          name: "{log}"
          size-mb: 64
          block-kb: 64
      computeCluster:
        type: "none"
    """
    r = LocalApplicationRunner.from_yaml({{"pipeline.yaml": APP, "configuration.yaml": CONF}}, instance=INSTANCE,
                                         application_id="durable")
    r.start()
    print("started", flush=True)
    while not r.errors:
        time.sleep(0.05)
    raise r.errors[0]
''')


def _wait_started(proc):
    """Read the worker's merged stdout/stderr up to its 'started' line (log lines such as the
    restored store's kernel-path notice may come first)."""
    seen = []
    for _ in range(50):
        line = proc.stdout.readline()
        if not line:
            break
        if line.strip() == b"started":
            return
        seen.append(line)
    raise AssertionError(f"worker did not start: {seen!r}")


def test_kill_restart_replays_committed_offsets_without_loss(tmp_path):
    from langstream_amd.api.model import StreamingCluster
    from langstream_amd.api.record import SimpleRecord
    from langstream_amd.topics.shm import ShmTopicConnectionsRuntime, unlink_shmlog
    logname = f"dur-{uuid.uuid4().hex[:8]}"
    store = str(tmp_path / "store")
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT, store=store, log=logname))
    rt = ShmTopicConnectionsRuntime()
    rt.init(StreamingCluster("shm", {"name": logname, "size-mb": 64, "block-kb": 64}))
    rt.log.create_topic("chunks", 2, 0)
    group = "langstream-agent-write"
    prod = rt.create_producer("t", None, {"topic": "chunks"})
    n = 400
    try:
        a = subprocess.Popen([sys.executable, str(script)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        _wait_started(a)
        for i in range(n):
            prod.write(SimpleRecord.of(f"c{i}", {"vec": [float(i % 7 + 1), 1.0, float(i % 3)], "text": f"t{i}"})) \
                .result(5)
        deadline = time.time() + 60
        while sum(rt.log.committed("chunks", group)) < 40 and time.time() < deadline:
            time.sleep(0.001)
        a.send_signal(signal.SIGKILL)                     # crash mid-stream
        a.wait(30)
        done_at_kill = sum(rt.log.committed("chunks", group))
        assert 0 < done_at_kill
        b = subprocess.Popen([sys.executable, str(script)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        _wait_started(b)
        deadline = time.time() + 90
        while sum(rt.log.committed("chunks", group)) < n and time.time() < deadline:
            time.sleep(0.05)
        assert sum(rt.log.committed("chunks", group)) == n
        b.send_signal(signal.SIGKILL)
        b.wait(30)
        VectorStoreRegistry.reset()
        VectorStoreRegistry.configure(persist_dir=store)
        s = VectorStoreRegistry.get("docs", device="cpu")
        assert len(s) == n                                # every chunk indexed exactly once
        assert s.get("c123") == {"text": "t123"}
    finally:
        VectorStoreRegistry.reset()
        VectorStoreRegistry.persist_dir = None
        unlink_shmlog(logname, size_mb=64)


def test_torn_wal_tail_is_truncated_before_new_writes(tmp_path):
    """a crash mid-append leaves a torn entry; the next process must cut the
    log there BEFORE appending, or the entries written after the restart are parsed
    across the garbage on the restart after that."""
    d = str(tmp_path / "coll")
    s = VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    s.upsert(["a", "b"], [[1, 0, 0, 0], [0, 1, 0, 0]], [{"t": "a"}, {"t": "b"}])
    s.close()
    with open(os.path.join(d, "wal.log"), "ab") as f:     # torn write: length says 500 bytes
        f.write((500).to_bytes(4, "little") + b"\x93\xa1u")
    r = VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    assert len(r) == 2
    r.upsert(["c"], [[0, 0, 1, 0]], [{"t": "c"}])          # acknowledged after the restart
    r.delete(["a"])
    r.close()
    q = VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    assert len(q) == 2 and q.get("c") == {"t": "c"} and q.get("a") is None and q.get("b") == {"t": "b"}


def test_snapshot_swap_is_atomic_and_replay_idempotent(tmp_path):
    """The snapshot is one file swapped by one rename: a crash while writing it leaves the
    previous snapshot (plus a stray temp file) intact; a crash after the swap but before
    the WAL reset replays entries the snapshot already holds, harmlessly."""
    d = str(tmp_path / "coll")
    s = VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    s.upsert(list(range(6)), [[i, 1, 0, 0] for i in range(6)], [{"i": i} for i in range(6)])
    s.snapshot()
    s.upsert([6, 7], [[6, 1, 0, 0], [7, 1, 0, 0]], [{"i": 6}, {"i": 7}])
    s.delete([0])
    wal = open(os.path.join(d, "wal.log"), "rb").read()
    s.snapshot()
    s.close()
    # crash after the swap, before the WAL reset: the old WAL comes back
    open(os.path.join(d, "wal.log"), "wb").write(wal)
    # and a half-written next snapshot lies around
    open(os.path.join(d, "snapshot.lsv.tmp"), "wb").write(b"LSVS0001" + b"\xff" * 40)
    r = VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=d, name="c")
    assert len(r) == 7 and r.get(0) is None and r.get(7) == {"i": 7}
    assert sorted(r._ids) == list(range(1, 8))


def test_legacy_two_file_snapshot_still_loads(tmp_path):
    import json as _json
    d = tmp_path / "coll"
    d.mkdir()
    _json.dump({"dim": 4, "dtype": "float32", "ids": ["x"], "meta": [{"t": "x"}]}, open(d / "snapshot.json", "w"))
    np.asarray([[1, 0, 0, 0]], dtype=np.float32).tofile(d / "snapshot.vec")
    r = VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=str(d), name="c")
    assert r.get("x") == {"t": "x"}
    r.snapshot()
    assert not (d / "snapshot.json").exists() and (d / "snapshot.lsv").exists()
    r.close()
    assert VectorStore(4, device="cpu", dtype=torch.float32, persist_dir=str(d), name="c").get("x") == {"t": "x"}


def test_vector_sink_is_durable_by_default_in_its_state_dir(tmp_path):
    """Zero config: a local vector-db-sink keeps its WAL in the agent's persistent state
    directory, and the planner gives it a disk (the pod's PVC)."""
    from langstream_amd.agents.vector import VectorDBSinkAgent
    from langstream_amd.api.agent import AgentContext
    from langstream_amd.api.record import SimpleRecord
    VectorStoreRegistry.reset()
    VectorStoreRegistry.persist_dir = None
    try:
        def agent():
            a = VectorDBSinkAgent()
            a.set_metadata("sink1", "vector-db-sink", 0) if hasattr(a, "set_metadata") else None
            a.init({"datasource": {"service": "local"}, "collection-name": "durable",
                    "fields": [{"name": "id", "expression": "key"}, {"name": "vector", "expression": "value.vec"},
                               {"name": "text", "expression": "value.text"}]})
            a.set_context(AgentContext(agent_id="sink1", global_agent_id="app-sink1",
                                       persistent_state_directory=str(tmp_path)))
            a.start()
            return a
        a = agent()
        for i in range(5):
            a.write(SimpleRecord.of(f"k{i}", {"vec": [1.0, float(i), 0.0], "text": f"t{i}"})).result(10)
        a.close()
        # only this sink's collection is bound to its state dir; no process-wide default
        assert VectorStoreRegistry.persist_dir is None
        assert VectorStoreRegistry._dir_of("durable").startswith(str(tmp_path))
        assert VectorStoreRegistry._dir_of("other") is None
        VectorStoreRegistry.reset()                  # pod restart: in-memory state gone
        agent()
        s = VectorStoreRegistry.get("durable", device="cpu")
        assert len(s) == 5 and s.get("k3") == {"text": "t3"}
    finally:
        VectorStoreRegistry.reset()
        VectorStoreRegistry.persist_dir = None


def test_planner_gives_local_vector_sinks_a_disk():
    from langstream_amd.core.catalog import _vector_sink_disks
    from langstream_amd.api.model import AgentConfiguration
    assert _vector_sink_disks(AgentConfiguration(id="w", type="vector-db-sink",
                                                 configuration={"datasource": "LocalVectors"}))
    assert not _vector_sink_disks(AgentConfiguration(id="w", type="vector-db-sink",
                                                     configuration={"datasource": {"service": "opensearch"}}))


def test_two_sinks_persist_in_their_own_state_dirs(tmp_path):
    """ADVICE r3 / VERDICT r4: the first sink's state directory must not become the
    persistence default of every other collection in the process."""
    from langstream_amd.agents.vector import VectorDBSinkAgent
    from langstream_amd.api.agent import AgentContext
    from langstream_amd.api.record import SimpleRecord
    VectorStoreRegistry.reset()
    VectorStoreRegistry.persist_dir = None

    def sink(agent_id, coll):
        a = VectorDBSinkAgent()
        a.set_metadata(agent_id, "vector-db-sink", 0)
        a.init({"datasource": {"service": "local"}, "collection-name": coll,
                "fields": [{"name": "id", "expression": "key"}, {"name": "vector", "expression": "value.vec"}]})
        a.set_context(AgentContext(agent_id=agent_id, global_agent_id=f"app-{agent_id}",
                                   persistent_state_directory=str(tmp_path / agent_id)))
        a.start()
        return a
    try:
        a, b = sink("s1", "c1"), sink("s2", "c2")
        a.write(SimpleRecord.of("x", {"vec": [1.0, 0.0]})).result(10)
        b.write(SimpleRecord.of("y", {"vec": [0.0, 1.0]})).result(10)
        a.close()
        b.close()
        assert VectorStoreRegistry._dir_of("c1").startswith(str(tmp_path / "s1"))
        assert VectorStoreRegistry._dir_of("c2").startswith(str(tmp_path / "s2"))
        # a collection no sink owns is not persisted anywhere
        assert not VectorStoreRegistry.get("scratch", 2, device="cpu").persistent
        assert os.listdir(tmp_path / "s1" / "s1" / "vector-store") == ["c1"]
        VectorStoreRegistry.reset()
        sink("s2", "c2")
        assert VectorStoreRegistry.get("c2", device="cpu").get("y") is not None
        assert not VectorStoreRegistry.exists("c1")       # s1 has not restarted yet
    finally:
        VectorStoreRegistry.reset()


def test_search_finishes_under_a_stream_of_deletes(monkeypatch):
    """a delete between every lock-free top-k and its row resolution cannot
    make a search repeat forever -- after SEARCH_RETRIES invalidated attempts the search
    holds the lock from the top-k through the resolution."""
    import langstream_amd.engine.vector_store as vs
    g = torch.Generator().manual_seed(4)
    vecs = torch.randn(40, 32, generator=g)
    s = VectorStore(32, device="cpu", dtype=torch.float32)
    s.upsert(list(range(40)), vecs.tolist(), [{"i": i} for i in range(40)])
    real = vs.to_host_async
    calls = {"n": 0}

    def racing(*t):
        calls["n"] += 1
        out = real(*t)
        if calls["n"] <= vs.SEARCH_RETRIES:
            s.delete([calls["n"]])     # every lock-free attempt loses its rows
        return out

    monkeypatch.setattr(vs, "to_host_async", racing)
    res = s.search([vecs[30].tolist()], 2)
    assert calls["n"] == vs.SEARCH_RETRIES + 1 and s.search_retries == vs.SEARCH_RETRIES
    assert res[0][0]["id"] == 30 and res[0][0]["i"] == 30
