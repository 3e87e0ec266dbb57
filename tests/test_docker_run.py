"""`langstream run` / `docker run` parity (LocalRunApplicationCmd.java:63-440,
entrypoint.sh:18-34): the reference's example applications run UNMODIFIED with the
reference's example secrets -- jdbc:herddb:server:herddb.herddb-dev.svc.cluster.local:7000,
MinIO at minio.minio-dev.svc.cluster.local:9000, Kafka at localhost:9092 -- against the
bundled services `run` starts, hosted model names served by the local engines
(LANGSTREAM_LOCAL_AI=1; tiny CPU models here).  Also: --only-agent, --watch-files hot
reload, remote application sources (BaseCmd.java:430-487), and the service stand-ins'
protocol details (SigV4, HerdDB dialect and credentials, host aliases).
"""
from __future__ import annotations

import asyncio
import json
import os
import re
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.request

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = "/root/reference/examples"
SECRETS = f"{EX}/secrets/secrets.yaml"
needs_ref = pytest.mark.skipif(not os.path.isdir(f"{EX}/applications/s3-source"), reason="reference examples absent")

TINY = {"local-ai": True, "device": "cpu", "force-chat-model": "llama-tiny", "force-embeddings-model": "bert-tiny",
        "use-graphs": "false", "num-blocks": 64, "max-model-len": 1024}


class _Run:
    """`python -m langstream_amd.cli run ...` in its own process group; endpoints parsed
    from its output."""

    def __init__(self, tmp_path, name, app, *extra, secrets=SECRETS, timeout=90.0, services=None):
        env = dict(os.environ, LANGSTREAM_CLI_CONFIG=str(tmp_path / "cli.yaml"), LANGSTREAM_LOCAL_AI="1",
                   LANGSTREAM_LOCAL_SERVICES_PORTS="random", PYTHONPATH=REPO,
                   LANGSTREAM_SERVICES_CONFIG=json.dumps(TINY if services is None else services))
        cmd = [sys.executable, "-u", "-m", "langstream_amd.cli", "run", name, "-app", app, "--no-start-ui",
               "--web-port", "0", "--gateway-port", "0", "--agents-port", "0", *extra]
        if secrets:
            cmd += ["-s", secrets]
        self.p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                  start_new_session=True, cwd=str(tmp_path))
        self.lines = []
        self.info = {}
        deadline = time.time() + timeout
        for line in self.p.stdout:
            self.lines.append(line)
            for key, rx in (("s3", r"Start S3: True \((\S+)\)"),
                            ("db", r"Start Database: True \(jdbc:herddb:server:(\S+:\d+)\)"),
                            ("broker", r"kafka bootstrap (\S+)\)")):
                m = re.search(rx, line)
                if m:
                    self.info[key] = m.group(1)
            m = re.search(r"running: webservice (\S+)\s+gateway (\S+)\s+agents (\S+)", line)
            if m:
                self.info.update(web=m.group(1), gw=m.group(2), agents=m.group(3))
                break
            if time.time() > deadline:
                break
        threading.Thread(target=self._drain, daemon=True).start()
        if "gw" not in self.info:
            self.stop()
            raise AssertionError("run did not start:\n" + "".join(self.lines[-40:]))

    def _drain(self):
        for line in self.p.stdout:
            self.lines.append(line)

    def output(self) -> str:
        return "".join(self.lines)

    def stop(self) -> int:
        if self.p.poll() is None:
            os.killpg(self.p.pid, signal.SIGTERM)
            try:
                self.p.wait(30)
            except subprocess.TimeoutExpired:
                os.killpg(self.p.pid, signal.SIGKILL)
                self.p.wait(10)
        return self.p.returncode

    def agent_info(self):
        return json.loads(urllib.request.urlopen(self.info["agents"] + "/info", timeout=10).read())

    def db(self):
        from langstream_amd.agents.vector.pgwire import PgConnection
        h, p = self.info["db"].rsplit(":", 1)
        return PgConnection(h, int(p), "sa", "hdb", "herd")


async def _ask(gw, app, question, session="s1", consume_gateway="bot-output", timeout=90.0):
    import aiohttp
    out = []
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(f"{gw}/v1/consume/default/{app}/{consume_gateway}?param:sessionId={session}") as cons, \
                s.ws_connect(f"{gw}/v1/produce/default/{app}/user-input?param:sessionId={session}") as prod:
            await prod.send_str(json.dumps({"value": question}))
            ack = json.loads((await prod.receive()).data)
            assert ack["status"] == "OK", ack
            while True:
                m = await asyncio.wait_for(cons.receive(), timeout)
                rec = json.loads(m.data)["record"]
                out.append(rec)
                if rec["headers"].get("stream-last-message") == "true":
                    return out


@needs_ref
def test_s3_source_example_runs_unmodified(tmp_path):
    """examples/applications/s3-source with examples/secrets/secrets.yaml: s3-source on the
    S3 service (bucket created by the agent, object deleted after commit), text pipeline,
    embeddings, vector-db-sink into jdbc:herddb:server:herddb.herddb-dev...:7000, and the
    chatbot answering over the produce / consume gateways with the streaming headers."""
    _s3_source_example(tmp_path, None, 128)


@pytest.mark.gpu
def test_s3_source_example_runs_unmodified_on_gpu(tmp_path):
    """The same, on the GPU engines behind the hosted model names: gpt-3.5-turbo ->
    Llama-3-8B (bf16, HIP kernels, random init), text-embedding-ada-002 -> bge-small-en.
    Where the reference checkout is absent (the GPU box gets only this repository) the
    in-tree app of the same shape runs instead (tests/apps/s3_rag: s3-source on the
    bundled S3 service -> text pipeline -> embeddings -> vector-db-sink on the HerdDB-URL
    database, and the chatbot over the produce / consume gateways)."""
    gpu = {"local-ai": True, "max-model-len": 2048, "max-batch": 16, "kv-fraction": 0.1}
    if os.path.isdir(f"{EX}/applications/s3-source"):
        _s3_source_example(tmp_path, gpu, 384, timeout=600.0)
    else:
        _s3_source_example(tmp_path, gpu, 384, timeout=600.0, app=os.path.join(REPO, "tests", "apps", "s3_rag"),
                           secrets=os.path.join(REPO, "tests", "apps", "s3_rag_secrets.yaml"))


def test_in_tree_s3_rag_app_runs(tmp_path):
    """tests/apps/s3_rag (the GPU variant's fallback app) on the tiny CPU models."""
    _s3_source_example(tmp_path, None, 128, app=os.path.join(REPO, "tests", "apps", "s3_rag"),
                       secrets=os.path.join(REPO, "tests", "apps", "s3_rag_secrets.yaml"))


def _s3_source_example(tmp_path, services, dim, timeout=90.0, app=f"{EX}/applications/s3-source", secrets=SECRETS):
    from langstream_amd.agents.storage import S3Client
    r = _Run(tmp_path, "s3test", app, services=services, timeout=timeout, secrets=secrets)
    try:
        assert "Using default instance file that connects to the Kafka broker" in r.output()
        c = S3Client(r.info["s3"], "minioadmin", "minioadmin")
        for _ in range(150):
            if c.bucket_exists("documents"):
                break
            time.sleep(0.2)
        text = (b"LangStream is a framework for building event-driven LLM applications. It runs pipelines of agents "
                b"connected by topics, and the agents compute embeddings, query vector databases and call large "
                b"language models to answer questions about your documents.")
        c.put_object("documents", "intro.txt", text)
        db = r.db()
        rows = []
        for _ in range(200):
            rows = db.execute("SELECT filename, chunk_id, lang, num_tokens, embeddings_vector FROM documents", [])[0]
            if rows:
                break
            time.sleep(0.25)
        assert rows and rows[0]["filename"] == "intro.txt" and rows[0]["lang"] == "en"
        vec = rows[0]["embeddings_vector"]
        vec = json.loads(vec) if isinstance(vec, str) else vec
        assert len(vec) == dim                      # the encoder behind text-embedding-ada-002
        for _ in range(50):                         # S3Source.commit deletes the object
            if c.list_objects("documents") == []:
                break
            time.sleep(0.2)
        assert c.list_objects("documents") == []
        recs = asyncio.new_event_loop().run_until_complete(_ask(r.info["gw"], "s3test", "What is LangStream?"))
        ids = {x["headers"]["stream-id"] for x in recs}
        assert len(ids) == 1
        assert [int(x["headers"]["stream-index"]) for x in recs] == list(range(1, len(recs) + 1))
        assert all(x["headers"]["langstream-client-session-id"] == "s1" for x in recs)
    finally:
        assert r.stop() in (0, -signal.SIGTERM), r.output()[-3000:]


@needs_ref
def test_docker_chatbot_example_retrieves_from_the_database_service(tmp_path):
    """examples/applications/docker-chatbot (the headline RAG pipeline) unmodified: the
    crawler cannot reach docs.langstream.ai (no network) but the chatbot answers; a
    document written into the database service over its wire endpoint is what the
    query-vector-db step retrieves into the prompt (log-topic, llm-debug gateway)."""
    r = _Run(tmp_path, "chat", f"{EX}/applications/docker-chatbot")
    try:
        db = r.db()
        for _ in range(100):     # the jdbc-table asset is created at deploy
            if db.execute("SELECT table_name FROM information_schema.tables WHERE table_name = 'documents'", [])[0]:
                break
            time.sleep(0.1)
        vec = [0.01 * (i % 7) for i in range(128)]
        db.execute("INSERT INTO documents (filename, chunk_id, num_tokens, lang, text, embeddings_vector) "
                   "VALUES ($1, $2, $3, $4, $5, $6)", ["kb.txt", 0, 5, "en", "MI355X pipelines stream records", vec])

        async def both():
            import aiohttp
            async with aiohttp.ClientSession() as s:
                async with s.ws_connect(f"{r.info['gw']}/v1/consume/default/chat/llm-debug?option:position=earliest") as dbg:
                    recs = await _ask(r.info["gw"], "chat", "how do pipelines stream?", session="q1")
                    m = await asyncio.wait_for(dbg.receive(), 60)
                    return recs, json.loads(m.data)["record"]
        recs, logged = asyncio.new_event_loop().run_until_complete(both())
        assert recs[-1]["headers"]["stream-last-message"] == "true"
        val = logged["value"] if isinstance(logged["value"], dict) else json.loads(logged["value"])
        prompt = json.dumps(val["prompt"])
        assert "MI355X pipelines stream records" in prompt
        assert "answer" in val and "question_embeddings" not in val and "related_documents" not in val
    finally:
        r.stop()


def _python_app(tmp_path, suffix):
    app = tmp_path / "app"
    (app / "python").mkdir(parents=True)
    (app / "pipeline.yaml").write_text(
        "topics:\n  - name: in\n    creation-mode: create-if-not-exists\n"
        "  - name: out\n    creation-mode: create-if-not-exists\n"
        "pipeline:\n  - name: upper\n    id: upper\n    type: python-processor\n    input: in\n"
        "    configuration:\n      className: proc.Proc\n"
        "  - name: tail\n    id: tail\n    type: identity\n    output: out\n"
        "    resources:\n      parallelism: 2\n")
    (app / "gateways.yaml").write_text(
        "gateways:\n  - id: produce-in\n    type: produce\n    topic: in\n"
        "  - id: consume-out\n    type: consume\n    topic: out\n")
    (app / "python" / "proc.py").write_text(_proc(suffix))
    return app


def _proc(suffix):
    return ("from langstream import SimpleRecord, Processor\n\n\nclass Proc(Processor):\n"
            "    def process(self, record):\n"
            f"        return [SimpleRecord(record.value().upper() + {suffix!r})]\n")


async def _roundtrip(gw, value):
    import aiohttp
    async with aiohttp.ClientSession() as s:
        async with s.ws_connect(f"{gw}/v1/consume/default/py/consume-out") as cons, \
                s.ws_connect(f"{gw}/v1/produce/default/py/produce-in") as prod:
            await prod.send_str(json.dumps({"value": value}))
            assert json.loads((await prod.receive()).data)["status"] == "OK"
            while True:
                rec = json.loads((await asyncio.wait_for(cons.receive(), 30)).data)["record"]
                if rec["value"].startswith(value.upper()):
                    return rec["value"]


def test_watch_files_hot_reloads_python_and_only_agent(tmp_path):
    """--watch-files (ApplicationWatcher + POST /commands/restart): editing python/ changes
    the running processor without a redeploy.  No broker (--no-start-broker): the
    in-process memory streaming cluster carries the topics."""
    app = _python_app(tmp_path, "-v1")
    r = _Run(tmp_path, "py", str(app), "--no-start-broker", "--no-start-s3", "--no-start-database", secrets=None)
    try:
        assert "Start broker: False" in r.output() and "memory streaming cluster" in r.output()
        assert asyncio.new_event_loop().run_until_complete(_roundtrip(r.info["gw"], "abc")) == "ABC-v1"
        time.sleep(1.1)                                 # a new mtime second for the poller
        (app / "python" / "proc.py").write_text(_proc("-v2"))
        deadline = time.time() + 30
        while "restarting the application" not in r.output() and time.time() < deadline:
            time.sleep(0.2)
        assert "A python file has changed, restarting the application" in r.output()
        time.sleep(1.0)
        assert asyncio.new_event_loop().run_until_complete(_roundtrip(r.info["gw"], "def")) == "DEF-v2"
        ids = {a["agent-id"] for a in r.agent_info()}
        assert ids == {"upper", "tail"}
    finally:
        r.stop()
    # --only-agent: just that agent's runner (all replicas) starts
    r = _Run(tmp_path, "py", str(app), "--no-start-broker", "--no-start-s3", "--no-start-database",
             "--no-watch-files", "--only-agent", "tail", secrets=None)
    try:
        info = r.agent_info()
        assert "Filter agent: tail" in r.output()
        assert {a["agent-id"] for a in info} == {"tail"}
        assert len([a for a in info if a["component-type"] == "SOURCE"]) == 2   # parallelism 2
    finally:
        r.stop()


def test_run_dry_run_and_picocli_boolean_syntax(tmp_path):
    app = _python_app(tmp_path, "")
    env = dict(os.environ, PYTHONPATH=REPO, LANGSTREAM_CLI_CONFIG=str(tmp_path / "c.yaml"))
    out = subprocess.run([sys.executable, "-m", "langstream_amd.cli", "docker", "run", "py", "-app", str(app),
                          "--dry-run", "--start-broker=false"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "Start broker: False" in out.stdout and "modules:" in out.stdout
    assert "upper" in out.stdout


# ---------------------------------------------------------------- remote sources
def test_remote_sources_github_https_file(tmp_path, monkeypatch):
    from langstream_amd.cli import sources
    # a "GitHub" repository served from a local directory (LANGSTREAM_GITHUB_URL)
    gh = tmp_path / "gh"
    work = tmp_path / "work"
    subprocess.run(["git", "init", "-q", "-b", "main", str(work)], check=True)
    (work / "apps" / "demo").mkdir(parents=True)
    (work / "apps" / "demo" / "pipeline.yaml").write_text("pipeline:\n  - type: identity\n")
    (work / "secrets.yaml").write_text("secrets: []\n")
    git = ["git", "-C", str(work), "-c", "user.email=a@b", "-c", "user.name=a"]
    subprocess.run(git + ["add", "."], check=True)
    subprocess.run(git + ["commit", "-q", "-m", "v1"], check=True)
    (gh / "acme").mkdir(parents=True)
    subprocess.run(["git", "clone", "-q", "--bare", str(work), str(gh / "acme" / "demo.git")], check=True)
    monkeypatch.setenv("LANGSTREAM_GITHUB_URL", f"file://{gh}")
    monkeypatch.setenv("LANGSTREAM_CLI_CONFIG", str(tmp_path / "home" / "config.yaml"))
    sources._cloned.clear()
    p = sources.check_file_exists_or_download("https://github.com/acme/demo/tree/main/apps/demo")
    assert p == str(tmp_path / "home" / "ghrepos" / "acme" / "demo" / "main" / "apps" / "demo")
    assert open(os.path.join(p, "pipeline.yaml")).read().startswith("pipeline:")
    # same process, same repository: no second clone (secrets from the same repo)
    s = sources.check_file_exists_or_download("https://github.com/acme/demo/blob/main/secrets.yaml")
    assert s.endswith("secrets.yaml") and os.path.exists(s)
    # a later process updates the cached clone instead of cloning again
    (work / "apps" / "demo" / "pipeline.yaml").write_text("pipeline:\n  - type: noop\n")
    subprocess.run(git + ["commit", "-q", "-am", "v2"], check=True)
    subprocess.run(["git", "-C", str(work), "push", "-q", str(gh / "acme" / "demo.git"), "main"], check=True)
    sources._cloned.clear()
    p2 = sources.check_file_exists_or_download("https://github.com/acme/demo/tree/main/apps/demo")
    assert p2 == p and "noop" in open(os.path.join(p2, "pipeline.yaml")).read()
    # --disable-local-repositories-cache: a fresh temporary clone
    p3 = sources.check_file_exists_or_download("https://github.com/acme/demo/tree/main/apps/demo", use_cache=False)
    assert p3 != p and os.path.exists(os.path.join(p3, "pipeline.yaml"))
    with pytest.raises(ValueError, match="Invalid github url"):
        sources.parse_github("https://github.com/acme/demo")
    # http:// refused, file:// stripped, missing file fails
    with pytest.raises(ValueError, match="http is not supported"):
        sources.check_file_exists_or_download("http://example.com/app.zip")
    assert sources.check_file_exists_or_download(f"file://{work}/secrets.yaml") == f"{work}/secrets.yaml"
    with pytest.raises(FileNotFoundError):
        sources.check_file_exists_or_download(str(tmp_path / "nope.yaml"))
    # https download (transport injected) and an app zip unpacked to a directory
    import io
    import zipfile
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        z.writestr("demo/pipeline.yaml", "pipeline:\n  - type: identity\n")
    path = sources.download_https("https://example.com/app.zip", fetch=lambda u: (200, buf.getvalue()))
    d = sources.as_app_directory(path)
    assert os.path.exists(os.path.join(d, "pipeline.yaml"))
    with pytest.raises(RuntimeError, match="Received status code: 404"):
        sources.download_https("https://example.com/x", fetch=lambda u: (404, b"not found"))


# ---------------------------------------------------------------- stand-ins
def test_host_aliases_redirect_connections():
    from langstream_amd.utils import hostmap
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    try:
        hostmap.add({"svc.example.internal:7000": f"127.0.0.1:{port}"})
        assert hostmap.resolve("SVC.example.internal", 7000) == ("127.0.0.1", port)
        assert hostmap.resolve("svc.example.internal", 7001) == ("svc.example.internal", 7001)
        c = socket.create_connection(("svc.example.internal", 7000), timeout=5)
        a, _ = srv.accept()
        c.close()
        a.close()
        assert json.loads(os.environ[hostmap.ENV])["svc.example.internal:7000"] == f"127.0.0.1:{port}"
    finally:
        hostmap.remove(["svc.example.internal:7000"])
        srv.close()
    assert hostmap.resolve("svc.example.internal", 7000) == ("svc.example.internal", 7000)


def test_s3_standalone_sigv4_list_and_errors():
    from langstream_amd.agents.s3_standalone import S3Standalone
    from langstream_amd.agents.storage import S3Client
    srv = S3Standalone().start()
    try:
        c = S3Client(srv.endpoint, "minioadmin", "minioadmin")
        assert not c.bucket_exists("b")
        c.make_bucket("b")
        c.make_bucket("b")                      # 409 BucketAlreadyOwnedByYou is accepted by the client
        for i in range(5):
            c.put_object("b", f"dir/k{i}.txt", b"x" * i)
        c.put_object("b", "other", b"y")
        assert c.list_objects("b", "dir/") == [f"dir/k{i}.txt" for i in range(5)]
        assert c.get_object("b", "dir/k3.txt") == b"xxx"
        assert c.get_object("b", "missing") is None
        c.remove_object("b", "other")
        assert "other" not in c.list_objects("b")
        bad = S3Client(srv.endpoint, "minioadmin", "wrong-secret")
        with pytest.raises(IOError, match="403"):
            bad.put_object("b", "k", b"z")
        with pytest.raises(IOError, match="404"):
            c.put_object("nobucket", "k", b"z")
    finally:
        srv.stop()


def test_s3_standalone_paginates_list_objects_v2():
    import requests
    from langstream_amd.agents.s3_standalone import S3Standalone
    from langstream_amd.agents.storage import S3Client
    srv = S3Standalone(verify_signatures=False).start()
    try:
        c = S3Client(srv.endpoint, "a", "b")
        c.make_bucket("p")
        for i in range(7):
            c.put_object("p", f"k{i}", b"")
        r = requests.get(f"{srv.endpoint}/p?list-type=2&max-keys=3")
        assert "<IsTruncated>true</IsTruncated>" in r.text and "<KeyCount>3</KeyCount>" in r.text
        assert c.list_objects("p") == [f"k{i}" for i in range(7)]
    finally:
        srv.stop()


def test_herddb_service_in_process_and_wire_share_one_database():
    """jdbc:herddb:server: in the service's process -> SQLite + GPU-kNN mirror; over the
    wire from elsewhere -> the PostgreSQL-protocol endpoint; one database either way,
    HerdDB's CAST(? AS FLOAT ARRAY), credentials checked."""
    from langstream_amd.agents.vector import herddb
    from langstream_amd.agents.vector.datasources import jdbc_datasource
    from langstream_amd.agents.vector.pgwire import PgConnection
    from langstream_amd.utils import hostmap
    srv = herddb.HerdDBServer().start()
    hostmap.add({f"herddb.test.local:{herddb.DEFAULT_PORT}": f"127.0.0.1:{srv.port}"})
    try:
        cfg = {"service": "jdbc", "url": f"jdbc:herddb:server:herddb.test.local:{herddb.DEFAULT_PORT}",
               "user": "sa", "password": "hdb"}
        ds = jdbc_datasource(cfg)
        assert isinstance(ds, herddb._HerdDBDataSource)
        ds.script(["CREATE TABLE documents (filename TEXT, chunk_id int, text TEXT, embeddings_vector FLOATA, "
                   "PRIMARY KEY (filename, chunk_id))"])
        for i in range(4):
            ds.execute_statement("INSERT INTO documents (filename, chunk_id, text, embeddings_vector) VALUES (?,?,?,?)",
                                 [], ["f", i, f"t{i}", [1.0 if j == i else 0.0 for j in range(4)]])
        q = ("SELECT text,embeddings_vector FROM documents ORDER BY cosine_similarity(embeddings_vector, "
             "CAST(? as FLOAT ARRAY)) DESC LIMIT 2")
        assert [r["text"] for r in ds.fetch_data(q, [[0.0, 0.1, 1.0, 0.0]])] == ["t2", "t1"]
        # a wire client (another process in real runs) sees the rows and its writes reach the mirror
        db = PgConnection("127.0.0.1", srv.port, "sa", "hdb", "herd")
        assert len(db.execute("SELECT * FROM documents", [])[0]) == 4
        db.execute("INSERT INTO documents (filename, chunk_id, text, embeddings_vector) VALUES ($1,$2,$3,$4)",
                   ["g", 0, "wire", [0.0, 0.0, 0.0, 1.0]])
        assert ds.fetch_data(q, [[0.0, 0.0, 0.0, 1.0]])[0]["text"] == "wire"
        rows = db.execute("SELECT text FROM documents ORDER BY cosine_similarity(embeddings_vector, "
                          "CAST($1 AS FLOAT ARRAY)) DESC LIMIT 1", [[1.0, 0.0, 0.0, 0.0]])[0]
        assert rows == [{"text": "t0"}]
        with pytest.raises(PermissionError):
            jdbc_datasource(dict(cfg, password="nope"))
        # the remote path (no service in this process for that address): over the wire
        remote = herddb._remote_class()(dict(cfg, url=f"jdbc:herddb:server:127.0.0.1:{srv.port}"), "127.0.0.1",
                                        srv.port)
        assert len(remote.fetch_data("SELECT filename FROM documents WHERE chunk_id = ?", [0])) == 2
        assert remote.table_exists("documents")
    finally:
        hostmap.remove([f"herddb.test.local:{herddb.DEFAULT_PORT}"])
        srv.stop()
        herddb.reset()


def test_herddb_url_without_service_fails_with_a_clear_message():
    from langstream_amd.agents.vector.datasources import jdbc_datasource
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with pytest.raises(ConnectionError, match="--start-database"):
        jdbc_datasource({"service": "jdbc", "url": f"jdbc:herddb:server:127.0.0.1:{port}"})


def test_local_services_fall_back_to_free_ports_with_aliases():
    from langstream_amd.runtime.local_services import LocalServices
    from langstream_amd.utils import hostmap
    svc = LocalServices(well_known_ports=False).start()
    try:
        al = hostmap.current()
        assert al["minio.minio-dev.svc.cluster.local:9000"] == f"127.0.0.1:{svc.s3.port}"
        assert al["herddb.herddb-dev.svc.cluster.local:7000"] == f"127.0.0.1:{svc.database.port}"
        assert al["my-cluster-kafka-bootstrap.kafka:9092"] == f"127.0.0.1:{svc.broker.port}"
        assert "bootstrap.servers: localhost:9092" in svc.default_instance()
        from langstream_amd.agents.storage import S3Client
        S3Client("http://minio.minio-dev.svc.cluster.local:9000", "minioadmin", "minioadmin").make_bucket("x")
        assert "x" in svc.s3.store.buckets
    finally:
        svc.stop()
    assert "minio.minio-dev.svc.cluster.local:9000" not in hostmap.current()
