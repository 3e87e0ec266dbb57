"""python-source / python-processor / python-sink / python-service, run IN-PROCESS.

Parity: the reference spawns ``python3 -m langstream_grpc`` and streams records over
gRPC (GRPC/java/.../PythonGrpcServer.java:53-146, AbstractGrpcAgent.java:69-436,
RTPY/langstream_grpc/grpc_service.py:75-456).  The MI355X runtime is Python, so the
user class (``className``, resolved from ``<code dir>/python`` and its ``lib`` dir) is
imported directly; records are converted between the runtime Record and the user
API (``langstream.Record``: objects, dicts or tuples).  Sync processors run on a small
thread pool (one record at a time per agent, like ``asyncio.to_thread`` in the
reference); Future results are awaited asynchronously.  ``restart()`` reloads the
user module (dev-mode hot reload).
"""
from __future__ import annotations

import importlib
import logging
import os
import sys
import threading
from concurrent.futures import Future, ThreadPoolExecutor
from typing import Any, Dict, List

from ..api.agent import AgentProcessor, AgentService, AgentSink, AgentSource, completed, failed
from ..api.record import Header, Record, SimpleRecord, SourceRecordAndResult
from ..runtime.registry import register_agent

log = logging.getLogger(__name__)


def _to_user(v: Any) -> Any:
    """Avro records reach Python agents as ``langstream.AvroValue(schema, value)`` -- the
    schema as its JSON dict, the value as plain dicts (the reference decodes them with
    fastavro.schemaless_reader: RTPY/langstream_grpc/grpc_service.py:239-248)."""
    from ..api.avro import AvroRecord
    if isinstance(v, AvroRecord) and v.schema is not None:
        from langstream import AvroValue
        return AvroValue(schema=v.schema.to_json(), value=_plain(v))
    return v


def _plain(v: Any) -> Any:
    if isinstance(v, dict):
        return {k: _plain(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_plain(x) for x in v]
    return v


def _from_user(v: Any) -> Any:
    """``AvroValue`` results become AvroRecords (encoded with their schema downstream,
    grpc_service.py:294-305's schemaless_writer path)."""
    if type(v).__name__ == "AvroValue" and hasattr(v, "schema") and hasattr(v, "value"):
        from ..api.avro import AvroRecord
        return AvroRecord(v.value, v.schema)
    return v


class _UserRecord:
    """Runtime Record viewed through the user API (key(), value(), headers() as tuples)."""

    def __init__(self, r: Record):
        self._r = r

    def key(self):
        return _to_user(self._text_form(self._r.key(), 0))

    def value(self):
        return _to_user(self._text_form(self._r.value(), 1))

    def _text_form(self, v, i):
        # a map an upstream agent parsed from JSON text reaches user code as that text,
        # compact, as the reference's Java agents hand it to the Python runtime
        # (MutableRecord.convertMapToStringOrBytes -> gRPC string / bytes value)
        if isinstance(v, dict):
            from .genai.mutable import _text_origin, text_form
            ref = getattr(self._r, "_source_ref", None)
            if isinstance(ref, dict) and "json_origin" in ref:
                return text_form(v, ref["json_origin"][i])
        return v

    def origin(self):
        return self._r.origin()

    def timestamp(self):
        return self._r.timestamp()

    def headers(self):
        return [(h.key, h.value) for h in self._r.headers()]

    def __repr__(self):
        return repr(self._r)


def to_runtime_record(x: Any) -> Record:
    if isinstance(x, _UserRecord):
        return x._r
    if isinstance(x, Record):
        return x
    f = _from_user
    if isinstance(x, dict):
        return SimpleRecord.of(f(x.get("key")), f(x.get("value")),
                               [Header(k, f(v)) for k, v in (x.get("headers") or [])], x.get("origin"),
                               x.get("timestamp"))
    if isinstance(x, (tuple, list)):
        vals = list(x) + [None] * (5 - len(x))
        value, key, headers, origin, ts = vals[:5]
        return SimpleRecord.of(f(key), f(value), [Header(k, f(v)) for k, v in (headers or [])], origin, ts)
    if hasattr(x, "value") and callable(x.value):
        hs = [Header(k, f(v)) for k, v in (x.headers() or [])] if hasattr(x, "headers") else []
        return SimpleRecord.of(f(x.key()) if hasattr(x, "key") else None, f(x.value()), hs,
                               x.origin() if hasattr(x, "origin") else None,
                               x.timestamp() if hasattr(x, "timestamp") else None)
    return SimpleRecord.of(None, f(x))


class _Ctx:
    def __init__(self, ctx):
        self._ctx = ctx

    def get_persistent_state_directory(self):
        return self._ctx.get_persistent_state_directory() if self._ctx is not None else None

    def __getattr__(self, item):
        return getattr(self._ctx, item)


class _PythonAgentMixin:
    def _load_user(self, configuration: Dict[str, Any]):
        self.cfg = dict(configuration)
        cls_name = self.cfg.get("className")
        if not cls_name:
            raise ValueError("className is required")
        self.class_name = cls_name
        self.user = None

    def _instantiate(self):
        code_dir = getattr(self.context, "code_directory", "") or ""
        for p in (os.path.join(code_dir, "python"), os.path.join(code_dir, "python", "lib"), code_dir):
            if p and os.path.isdir(p) and p not in sys.path:
                sys.path.insert(0, p)
        mod_name, _, cls = self.class_name.rpartition(".")
        mod = importlib.import_module(mod_name)
        self._module = mod
        self.user = getattr(mod, cls)()
        init = getattr(self.user, "init", None)
        if init is not None:
            try:
                init(self.cfg, _Ctx(self.context))
            except TypeError:
                init(self.cfg)

    def _start_user(self):
        if self.user is None:
            self._instantiate()
        s = getattr(self.user, "start", None)
        if s is not None:
            s()

    def _close_user(self):
        if self.user is not None and hasattr(self.user, "close"):
            self.user.close()

    def _restart_user(self):
        self._close_user()
        importlib.reload(self._module)
        self.user = None
        self._start_user()

    def _info(self):
        ai = getattr(self.user, "agent_info", None)
        return ai() if ai is not None else {}


@register_agent("python-processor", "python-function")
class PythonProcessor(_PythonAgentMixin, AgentProcessor):
    def init(self, configuration):
        self._load_user(configuration)
        self.pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix=f"agent-{self.agent_id()}-py")

    def start(self):
        self._start_user()

    def close(self):
        self._close_user()
        self.pool.shutdown(wait=False)

    def restart(self):
        self._restart_user()

    def build_additional_info(self):
        return self._info()

    def process(self, records, sink):
        for r in records:
            self.pool.submit(self._one, r, sink)

    def _one(self, r, sink):
        try:
            res = self.user.process(_UserRecord(r))
        except Exception as e:  # noqa: BLE001
            sink(SourceRecordAndResult(r, None, e))
            return
        if isinstance(res, Future):
            def done(f, r=r):
                if f.exception() is not None:
                    sink(SourceRecordAndResult(r, None, f.exception()))
                else:
                    out = [to_runtime_record(x) for x in (f.result() or [])]
                    self.processed(1, len(out))
                    sink(SourceRecordAndResult(r, out, None))
            res.add_done_callback(done)
            return
        if res is not None and not isinstance(res, list):
            res = [res]
        out = [to_runtime_record(x) for x in (res or [])]
        self.processed(1, len(out))
        sink(SourceRecordAndResult(r, out, None))


@register_agent("python-source")
class PythonSource(_PythonAgentMixin, AgentSource):
    def init(self, configuration):
        self._load_user(configuration)

    def start(self):
        self._start_user()

    def close(self):
        self._close_user()

    def restart(self):
        self._restart_user()

    def build_additional_info(self):
        return self._info()

    def read(self):
        out = [to_runtime_record(x) for x in (self.user.read() or [])]
        self._map = getattr(self, "_map", {})
        self.processed(0, len(out))
        return out

    def commit(self, records):
        c = getattr(self.user, "commit", None)
        if c is not None:
            for r in records:
                c(_UserRecord(r))

    def permanent_failure(self, record, error):
        pf = getattr(self.user, "permanent_failure", None)
        if pf is None:
            raise error
        pf(_UserRecord(record), error)


@register_agent("python-sink")
class PythonSink(_PythonAgentMixin, AgentSink):
    def init(self, configuration):
        self._load_user(configuration)

    def start(self):
        self._start_user()

    def close(self):
        self._close_user()

    def restart(self):
        self._restart_user()

    def build_additional_info(self):
        return self._info()

    def write(self, record) -> Future:
        self.processed(1, 0)
        try:
            res = self.user.write(_UserRecord(record))
        except Exception as e:  # noqa: BLE001
            return failed(e)
        if isinstance(res, Future):
            return res
        return completed(None)


@register_agent("python-service")
class PythonService(_PythonAgentMixin, AgentService):
    def init(self, configuration):
        self._load_user(configuration)
        self._thread = None
        self._error = None

    def start(self):
        self._start_user()

        def run():
            try:
                self.user.main()
            except BaseException as e:  # noqa: BLE001
                self._error = e
                log.exception("python service failed")
                if self.context is not None:
                    self.context.critical_failure(e)

        self._thread = threading.Thread(target=run, name=f"py-service-{self.agent_id()}", daemon=True)
        self._thread.start()

    def join_timeout(self, t: float) -> bool:
        self._thread.join(t)
        return not self._thread.is_alive()

    def join(self):
        self._thread.join()

    def close(self):
        self._close_user()
