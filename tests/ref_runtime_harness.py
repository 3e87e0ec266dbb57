"""Harness for the ported reference runtime scenarios (tests/test_ref_runtime_*.py).

The reference runs these as ``AbstractKafkaApplicationRunner`` tests
(``langstream-runtime-impl/src/test/java/ai/langstream/AbstractApplicationRunner.java``):
deploy an application map, produce to topics, ``executeAgentRunners`` (every agent pod as
a thread for a few loops) and ``waitForMessages`` on consumers that read from the
beginning.  Here the same application maps run through ``LocalApplicationRunner`` on
either the in-process ``memory`` streaming cluster or the in-tree Kafka-protocol broker
(the ``streaming`` fixture runs every ported case on both), with:

* ``produce(topic, value, headers)`` -- ``sendMessage``;
* ``wait_for(topic, values)`` -- ``waitForMessages``: the values read from the start of
  the topic equal ``values`` exactly (order and count), with a short grace period that
  catches duplicates;
* ``wait_any_order(topic, values)`` -- ``waitForMessagesInAnyOrder``;
* ``wait_failure()`` -- the PermanentFailureException ``executeAgentRunners`` rethrows.

The mock agents of ``mockagents/MockProcessorAgentsCodeProvider.java`` are registered on
import: ``mock-failing-processor``, ``mock-failing-sink``, ``mock-async-processor``,
``mock-service``, ``mock-stateful-processor``.
"""
from __future__ import annotations

import json
import os
import random
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, List, Optional

from langstream_amd.api.agent import (AbstractAgentCode, AgentProcessor, AgentService, AgentSink, ComponentType,
                                      SingleRecordAgentProcessor, completed, failed)
from langstream_amd.api.record import SimpleRecord, SourceRecordAndResult
from langstream_amd.api.topics import TopicOffsetPosition
from langstream_amd.core.catalog import AgentSpec, register_agent_type
from langstream_amd.runtime.local import LocalApplicationRunner
from langstream_amd.runtime.registry import register_agent


# ---------------------------------------------------------------- mock agents
class InjectedFailure(RuntimeError):
    pass


class FailingProcessor(SingleRecordAgentProcessor):
    def init(self, configuration):
        self.fail_on = str(configuration.get("fail-on-content", "") or "")

    def process_record(self, record):
        v = record.value()
        if v == self.fail_on:
            raise InjectedFailure(f"Failing on content: {self.fail_on}")
        if isinstance(v, str) and self.fail_on and self.fail_on in v:
            raise InjectedFailure(f"Failing on content: {v}")
        return [record]


class FailingSink(AgentSink):
    accepted: List[Any] = []

    def init(self, configuration):
        FailingSink.accepted.clear()
        self.fail_on = str(configuration.get("fail-on-content", "") or "")

    def write(self, record):
        v = record.value()
        if v == self.fail_on or (isinstance(v, str) and self.fail_on in v):
            return failed(InjectedFailure(f"Failing on content: {self.fail_on}"))
        FailingSink.accepted.append(record)
        return completed(None)


class AsyncProcessor(AgentProcessor):
    """Emits every record after a random delay (< 500 ms) from an 8-thread pool."""

    def start(self):
        self.pool = ThreadPoolExecutor(8)
        self.rng = random.Random()

    def process(self, records, sink):
        for r in records:
            delay = self.rng.random() * 0.5

            def emit(r=r, d=delay):
                time.sleep(d)
                sink(SourceRecordAndResult(r, [r], None))
            try:
                self.pool.submit(emit)
            except RuntimeError as e:        # rejected after shutdown
                sink(SourceRecordAndResult(r, [r], e))

    def close(self):
        if getattr(self, "pool", None) is not None:
            self.pool.shutdown(wait=True)


class MockService(AgentService):
    starts = joins = closes = 0

    @classmethod
    def reset(cls):
        cls.starts = cls.joins = cls.closes = 0

    def start(self):
        MockService.starts += 1

    def join(self):
        MockService.joins += 1

    def join_timeout(self, timeout):
        self.join()
        return True

    def close(self):
        MockService.closes += 1


class StatefulProcessor(SingleRecordAgentProcessor):
    def set_context(self, context):
        super().set_context(context)
        self.status_file = os.path.join(context.get_persistent_state_directory_for_agent(self.agent_id()), "status")

    def start(self):
        self.status = open(self.status_file).read() if os.path.exists(self.status_file) else ""

    def process_record(self, record):
        self.status += str(record.value())
        with open(self.status_file, "w") as f:
            f.write(self.status)
        return [SimpleRecord.of(record.key(), self.status)]


register_agent("mock-failing-processor")(FailingProcessor)
register_agent("mock-failing-sink")(FailingSink)
register_agent("mock-async-processor")(AsyncProcessor)
register_agent("mock-service")(MockService)
register_agent("mock-stateful-processor")(StatefulProcessor)
register_agent_type(AgentSpec(("mock-failing-processor", "mock-async-processor", "mock-stateful-processor"),
                              ComponentType.PROCESSOR))
register_agent_type(AgentSpec(("mock-failing-sink",), ComponentType.SINK))
register_agent_type(AgentSpec(("mock-service",), ComponentType.SERVICE))


# ---------------------------------------------------------------- runs
def instance_yaml(streaming: str, bootstrap, globals_: Optional[Dict[str, str]] = None,
                  extra_admin: Optional[Dict[str, str]] = None) -> str:
    """``bootstrap``: the Kafka bootstrap servers; for ``pulsar`` (web url, service url,
    tenant, namespace); for ``pravega`` the controller URI."""
    g = "".join(f"    {k}: {v}\n" for k, v in (globals_ or {}).items())
    if streaming == "pulsar":
        web, svc, tenant, ns = bootstrap
        sc = (f"  streamingCluster:\n    type: \"pulsar\"\n    configuration:\n      admin:\n"
              f"        serviceUrl: \"{web}\"\n      service:\n        serviceUrl: \"{svc}\"\n"
              f"      default-tenant: \"{tenant}\"\n      default-namespace: \"{ns}\"\n")
    elif streaming == "pravega":
        sc = (f"  streamingCluster:\n    type: \"pravega\"\n    configuration:\n      client:\n"
              f"        controller-uri: \"{bootstrap}\"\n        scope: \"langstream\"\n")
    elif streaming == "kafka":
        admin = {"bootstrap.servers": bootstrap, **(extra_admin or {})}
        conf = "".join(f"        {k}: \"{v}\"\n" for k, v in admin.items())
        sc = f"  streamingCluster:\n    type: \"kafka\"\n    configuration:\n      admin:\n{conf}"
    else:
        sc = "  streamingCluster:\n    type: \"memory\"\n"
    return "instance:\n" + (f"  globals:\n{g}" if g else "") + sc + "  computeCluster:\n    type: \"kubernetes\"\n"


def uniq(prefix: str) -> str:
    return f"{prefix}-{uuid.uuid4().hex[:10]}"


class Run:
    def __init__(self, streaming: str, bootstrap: Optional[str], files: Dict[str, str],
                 globals_: Optional[Dict[str, str]] = None, app_id: str = "app", state_dir: Optional[str] = None,
                 extra_admin: Optional[Dict[str, str]] = None, secrets: Optional[str] = None, services=None):
        self.instance = instance_yaml(streaming, bootstrap, globals_, extra_admin)
        self.app = LocalApplicationRunner.from_yaml(files, instance=self.instance, secrets=secrets,
                                                    application_id=app_id, state_dir=state_dir, services=services)
        self.bootstrap = bootstrap
        self.streaming = streaming

    def __enter__(self) -> "Run":
        self.app.start()
        return self

    def __exit__(self, *exc):
        self.app.stop(timeout=20)

    @property
    def plan(self):
        return self.app.plan

    def produce(self, topic: str, value: Any, key: Any = None, headers: Optional[Dict[str, Any]] = None) -> None:
        self.app.produce(topic, value, key, headers)

    def read_all(self, topic: str, n: int, timeout: float):
        rd = self.app.reader(topic, TopicOffsetPosition.EARLIEST)
        out = []
        deadline = time.time() + timeout
        while len(out) < n and time.time() < deadline:
            out.extend(rd.read().records)
        return out, rd

    def wait_for(self, topic: str, values: List[Any], timeout: float = 30.0, grace: float = 0.5):
        recs, rd = self.read_all(topic, len(values), timeout)
        end = time.time() + grace
        while time.time() < end:
            recs.extend(rd.read().records)
        got = [_norm(r.value()) for r in recs]
        assert got == [_norm(v) for v in values], f"{topic}: {got!r} != {values!r}"
        return recs

    def wait_any_order(self, topic: str, values, timeout: float = 60.0, grace: float = 0.5):
        recs, rd = self.read_all(topic, len(values), timeout)
        end = time.time() + grace
        while time.time() < end:
            recs.extend(rd.read().records)
        got = sorted(str(_norm(r.value())) for r in recs)
        assert got == sorted(str(v) for v in values), f"{topic}: {len(got)} records, want {len(values)}"
        return recs

    def wait_failure(self, timeout: float = 30.0) -> BaseException:
        deadline = time.time() + timeout
        while not self.app.errors and time.time() < deadline:
            time.sleep(0.02)
        assert self.app.errors, "expected the agent to fail"
        return self.app.errors[0]


def _norm(v):
    if isinstance(v, (bytes, bytearray)):
        v = bytes(v).decode()
    return v


def header(rec, name):
    for h in rec.headers():
        if h.key == name:
            v = h.value
            return v.decode() if isinstance(v, (bytes, bytearray)) else v
    return None


def as_json(v):
    v = _norm(v)
    return json.loads(v) if isinstance(v, str) else v


_lock = threading.Lock()


# ---------------------------------------------------------------- WireMock stand-in
class FakeHTTP:
    """Stub server for the reference's @WireMockTest cases: ``stub(method, path, body,
    status=200, json_body=..., text=...)`` where ``path`` includes the query string and
    ``body`` (optional) must equal the request body exactly and ``headers`` (optional) must
    all be present with these values; the latest matching stub answers (``data``: a bytes
    body, ``status=FakeHTTP.RESET``: the connection is reset); unmatched requests get 404."""

    def __init__(self):
        import http.server
        import socketserver
        self.stubs = []
        self.requests = []
        outer = self

        class H(http.server.BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _do(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n).decode("latin-1") if n else ""
                outer.requests.append((self.command, self.path, body, dict(self.headers)))
                for m, path, want, status, ctype, payload, hdrs, rhdrs in outer.stubs:
                    if m == self.command and path == self.path and (want is None or want == body) and \
                            all(self.headers.get(k) == v for k, v in hdrs.items()):
                        if status == FakeHTTP.RESET:   # WireMock's Fault.CONNECTION_RESET_BY_PEER
                            import socket
                            import struct
                            self.connection.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
                            self.close_connection = True
                            return
                        data = payload if isinstance(payload, bytes) else payload.encode()
                        self.send_response(status)
                        self.send_header("Content-Type", ctype)
                        for k, v in rhdrs.items():
                            self.send_header(k, v)
                        self.send_header("Content-Length", str(len(data)))
                        self.end_headers()
                        self.wfile.write(data)
                        return
                data = f"no stub for {self.command} {self.path} {body}".encode()
                self.send_response(404)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            do_GET = do_POST = do_PUT = do_PATCH = do_DELETE = _do

        class S(socketserver.ThreadingMixIn, http.server.HTTPServer):
            daemon_threads = True
        self.srv = S(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    RESET = -1   # status: reset the connection instead of answering

    def stub(self, method, path, body=None, status=200, json_body=None, text=None, ctype=None, headers=None,
             data=None, response_headers=None):
        if json_body is not None:
            payload, ct = json.dumps(json_body), "application/json"
        elif data is not None:
            payload, ct = bytes(data), "application/octet-stream"
        else:
            payload, ct = text or "", "application/json"
        # the most recent stub for a request wins (as in WireMock)
        self.stubs.insert(0, (method, path, body, status, ctype or ct, payload, dict(headers or {}),
                              dict(response_headers or {})))

    def reset(self):
        self.stubs.clear()
        self.requests.clear()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()
