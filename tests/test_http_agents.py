"""http-request and langserve-invoke against a local HTTP server (no network needed).

Mirrors the reference's HttpRequestAgentTest / LangServeInvokeAgentTest (WireMock):
templated URL/query/headers/body, JSON parsing of the response, /invoke output
extraction, /stream SSE chunk coalescing into stream-to-topic records."""
import json
import threading
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from langstream_amd.runtime.local import LocalApplicationRunner
from langstream_amd.topics.memory import reset_memlogs


class _H(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def _body(self):
        n = int(self.headers.get("Content-Length") or 0)
        return self.rfile.read(n).decode() if n else ""

    def do_GET(self):
        out = json.dumps({"path": self.path, "hdr": self.headers.get("X-Who")}).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(out)))
        self.end_headers()
        self.wfile.write(out)

    def do_POST(self):
        body = json.loads(self._body() or "{}")
        if self.path.endswith("/invoke"):
            out = json.dumps({"output": {"content": "answer to " + body["input"]["question"]}}).encode()
            self.send_response(200)
            self.send_header("Content-Length", str(len(out)))
            self.end_headers()
            self.wfile.write(out)
        elif self.path.endswith("/stream"):
            self.send_response(200)
            self.send_header("Content-Type", "text/event-stream")
            self.end_headers()
            for w in ["a", "b", "c", "d", "e", "f", "g"]:
                self.wfile.write(f'event: data\ndata: {{"content": "{w}"}}\n\n'.encode())
            self.wfile.write(b"event: end\n\n")
        else:
            self.send_response(500)
            self.end_headers()


@pytest.fixture(scope="module")
def server():
    s = ThreadingHTTPServer(("127.0.0.1", 0), _H)
    t = threading.Thread(target=s.serve_forever, daemon=True)
    t.start()
    yield f"http://127.0.0.1:{s.server_address[1]}"
    s.shutdown()


@pytest.fixture(autouse=True)
def _topics():
    reset_memlogs()
    yield
    reset_memlogs()


def _t():
    return "t" + uuid.uuid4().hex[:8]


def test_http_request(server):
    tin, tout = _t(), _t()
    pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
  - name: {tout}
    creation-mode: create-if-not-exists
pipeline:
  - name: call
    type: http-request
    input: {tin}
    output: {tout}
    configuration:
      url: "{server}/api/items"
      query-string:
        q: "{{{{ value.name }}}}"
      headers:
        X-Who: "{{{{ value.name }}}}"
      output-field: value.response
"""
    with LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}) as app:
        app.produce(tin, json.dumps({"name": "a b"}))
        recs = app.consume(tout, 1, timeout=20)
    v = json.loads(recs[0].value())
    assert v["response"] == {"path": "/api/items?q=a+b", "hdr": "a b"}


def test_langserve_invoke_and_stream(server):
    tin, tout, tstream = _t(), _t(), _t()
    for endpoint, expect in (("invoke", "answer to why"), ("stream", "abcdefg")):
        pipe = f"""
topics:
  - name: {tin}
    creation-mode: create-if-not-exists
  - name: {tout}
    creation-mode: create-if-not-exists
  - name: {tstream}
    creation-mode: create-if-not-exists
pipeline:
  - name: ls
    type: langserve-invoke
    input: {tin}
    output: {tout}
    configuration:
      url: "{server}/chain/{endpoint}"
      output-field: value.answer
      stream-to-topic: {tstream}
      stream-response-field: value
      min-chunks-per-message: 2
      fields:
        - name: question
          expression: value.q
"""
        reset_memlogs()
        with LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}) as app:
            app.produce(tin, json.dumps({"q": "why"}))
            recs = app.consume(tout, 1, timeout=20)
            assert json.loads(recs[0].value())["answer"] == expect
            if endpoint == "stream":
                chunks = app.consume(tstream, 5, timeout=10)
                # 1, 2, 2, 2 chunks per message, then the empty terminal message of
                # "event: end" (LangServeClient.java: last=true flushes the empty buffer)
                assert [c.value() for c in chunks] == ["a", "bc", "de", "fg", ""]
                assert chunks[-1].header_value("stream-last-message") in ("true", True)
                assert [int(c.header_value("stream-index")) for c in chunks] == [1, 2, 3, 4, 5]
