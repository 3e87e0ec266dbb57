"""Kafka Connect adapters: agent types ``sink`` and ``source``.

Parity: KRT/kafkaconnect/KafkaConnectSinkAgent.java:64-552 and KafkaConnectSourceAgent.java.
The reference loads Java connector classes (``connector.class``) from the application's
``java/lib`` jars and drives their tasks.  This runtime is Python, so connectors are
Python classes implementing the same contract as Kafka Connect's API:

  SinkConnector.task_class() / task_configs(max_tasks) / start(props) / stop()
  SinkTask.start(props) / put(records) / flush(offsets) / pre_commit(offsets) -> offsets / stop()
  SourceConnector ... / SourceTask.start(props) / poll() -> [SourceRecord] /
                        commit() / commit_record(record) / stop()

``connector.class`` is either a dotted Python path (``pkg.module.Class`` or
``pkg.module:Class``, importable from the application's ``python/`` directory) or one of
the Kafka-bundled class names mapped to built-in Python connectors:
``org.apache.kafka.connect.file.FileStreamSinkConnector`` (``file``: append one line per
record), ``org.apache.kafka.connect.file.FileStreamSourceConnector`` (``file``:
emit new lines, ``batch.size``) and ``com.datastax.oss.kafka.sink.CassandraSinkConnector``
(the reference's kafka-connect example: ``topic.<t>.<ks>.<table>.mapping`` upserts over
the in-tree CQL client, see CassandraSinkTask).

Sink agent semantics (as KafkaConnectSinkAgent): it HANDLES ITS OWN COMMITS -- records
are buffered and handed to ``put`` in batches of ``adapterConfig.batchSize`` (16384) or
after ``adapterConfig.lingerTimeMs`` (60000 ms, tests use less); on flush the task's
``pre_commit`` (default: ``flush`` + the offsets given) returns the offsets that are safe
to commit, and only those records are committed on the source consumer.  Source agent
semantics: ``poll`` feeds the pipeline; when the runtime commits a record the task's
``commit_record`` is called, and ``commit`` after each committed batch.
"""
from __future__ import annotations

import importlib
import logging
import os
import re
import threading
import time
from concurrent.futures import Future
from typing import Any, Dict, List, Optional

from ..api.agent import AgentSink, AgentSource, completed
from ..api.record import Header, Record, SimpleRecord
from ..runtime.registry import register_agent

log = logging.getLogger(__name__)


# ---------------------------------------------------------------- connector API
class ConnectRecord:
    """SinkRecord / SourceRecord: topic, partition, offset, key, value, headers, timestamp."""

    def __init__(self, topic: Optional[str], partition: Optional[int], offset: Optional[int], key: Any, value: Any,
                 headers: Optional[Dict[str, Any]] = None, timestamp: Optional[int] = None,
                 source_partition: Optional[Dict[str, Any]] = None, source_offset: Optional[Dict[str, Any]] = None):
        self.topic, self.partition, self.offset = topic, partition, offset
        self.key, self.value = key, value
        self.headers = headers or {}
        self.timestamp = timestamp
        self.source_partition, self.source_offset = source_partition, source_offset


class SinkTask:
    def start(self, props: Dict[str, str]) -> None: ...
    def put(self, records: List[ConnectRecord]) -> None: raise NotImplementedError
    def flush(self, offsets: Dict[tuple, int]) -> None: ...

    def pre_commit(self, offsets: Dict[tuple, int]) -> Dict[tuple, int]:
        self.flush(offsets)
        return offsets

    def stop(self) -> None: ...


class SourceTask:
    def start(self, props: Dict[str, str]) -> None: ...
    def poll(self) -> List[ConnectRecord]: raise NotImplementedError
    def commit(self) -> None: ...
    def commit_record(self, record: ConnectRecord) -> None: ...
    def stop(self) -> None: ...


class Connector:
    def start(self, props: Dict[str, str]) -> None:
        self.props = dict(props)

    def task_class(self): raise NotImplementedError

    def task_configs(self, max_tasks: int) -> List[Dict[str, str]]:
        return [dict(self.props)]

    def stop(self) -> None: ...


class FileStreamSinkTask(SinkTask):
    def start(self, props):
        self.path = props.get("file")
        if not self.path:
            raise ValueError("FileStreamSinkConnector needs 'file'")
        self.f = open(self.path, "a", encoding="utf-8")

    def put(self, records):
        for r in records:
            v = r.value.decode() if isinstance(r.value, bytes) else r.value
            self.f.write(f"{v}\n")

    def flush(self, offsets):
        self.f.flush()
        os.fsync(self.f.fileno())

    def stop(self):
        self.f.close()


class FileStreamSourceTask(SourceTask):
    def start(self, props):
        self.path = props.get("file")
        if not self.path:
            raise ValueError("FileStreamSourceConnector needs 'file'")
        self.batch = int(props.get("batch.size", 2000))
        self.topic = props.get("topic")
        self.pos = 0

    def poll(self):
        if not os.path.exists(self.path):
            time.sleep(0.05)
            return []
        out = []
        with open(self.path, "rb") as f:
            f.seek(self.pos)
            for line in f:
                if not line.endswith(b"\n"):
                    break
                self.pos += len(line)
                out.append(ConnectRecord(self.topic, None, None, None, line[:-1].decode("utf-8", "replace"),
                                         source_partition={"filename": self.path},
                                         source_offset={"position": self.pos}))
                if len(out) >= self.batch:
                    break
        if not out:
            time.sleep(0.05)
        return out


class FileStreamSinkConnector(Connector):
    def task_class(self):
        return FileStreamSinkTask


class FileStreamSourceConnector(Connector):
    def task_class(self):
        return FileStreamSourceTask


# ---------------------------------------------------------------- DataStax Cassandra sink
_TABLE_KEY = re.compile(r"^topic\.(.+)\.([A-Za-z0-9_]+)\.([A-Za-z0-9_]+)\.(mapping|deletesEnabled|ttl|"
                        r"consistencyLevel|nullToUnset|ttlTimeUnit|timestampTimeUnit)$")


def _secure_bundle(path: str) -> Dict[str, Any]:
    """Astra secure-connect bundle (zip with config.json + CA): -> host, CQL port,
    keyspace and the CA PEM.  (The bundle's SNI proxy routing by host id is not
    implemented: the CQL endpoint in config.json is dialled directly over TLS.)"""
    import base64 as _b64
    import json as _json
    import zipfile
    data = path
    if not os.path.exists(path) and not path.endswith(".zip"):
        import io
        data = io.BytesIO(_b64.b64decode(path))   # the bundle inlined as base64 (a secret)
    with zipfile.ZipFile(data) as z:
        cfg = _json.loads(z.read("config.json"))
        ca = z.read("ca.crt").decode() if "ca.crt" in z.namelist() else None
    return {"host": cfg.get("host"), "port": int(cfg.get("cql_port") or cfg.get("port") or 9042),
            "keyspace": cfg.get("keyspace"), "ca": ca}


class CassandraSinkTask(SinkTask):
    """Python port of the behaviour of com.datastax.oss.kafka.sink.CassandraSinkConnector,
    the connector of the reference's examples/applications/kafka-connect/pipeline.yaml,
    on the in-tree CQL native-protocol client (agents/vector/cql.py):

      contactPoints / port / loadBalancing.localDc / auth.username / auth.password, or
      cloud.secureConnectBundle (Astra);
      topic.<topic>.<keyspace>.<table>.mapping = "col=value.f, col2=key, col3=header.h, ..."
        (one INSERT -- a Cassandra upsert -- per record per mapped table; string values
        holding JSON are parsed, as the DataStax sink does for StringConverter records);
      topic.<topic>.<keyspace>.<table>.deletesEnabled (true): a record whose value is null
        deletes the row by its primary key (read from system_schema.columns);
      topic.<topic>.<keyspace>.<table>.ttl (seconds, -1 = none), .consistencyLevel,
      .nullToUnset (true: null mapped fields are left out of the INSERT instead of writing
        tombstones).
    Records are written in put(); flush/pre_commit then acknowledge them (the agent
    commits source offsets only after that)."""

    def start(self, props):
        from .vector.cql import CqlSession
        self.tables: Dict[str, List[Dict[str, Any]]] = {}
        per: Dict[tuple, Dict[str, str]] = {}
        for k, v in props.items():
            m = _TABLE_KEY.match(k)
            if m:
                per.setdefault((m.group(1), m.group(2), m.group(3)), {})[m.group(4)] = v
        for (topic, ks, table), opts in per.items():
            if "mapping" not in opts:
                raise ValueError(f"topic.{topic}.{ks}.{table}: a mapping is required")
            mapping = []
            for part in opts["mapping"].split(","):
                if part.strip():
                    col, _, expr = part.partition("=")
                    mapping.append((col.strip(), expr.strip()))
            self.tables.setdefault(topic, []).append({
                "ks": ks, "table": table, "mapping": mapping,
                "deletes": str(opts.get("deletesEnabled", "true")).lower() != "false",
                "ttl": int(opts.get("ttl", -1)),
                "null_to_unset": str(opts.get("nullToUnset", "true")).lower() != "false",
                "pk": None})
        if not self.tables:
            raise ValueError("CassandraSinkConnector: no topic.<topic>.<keyspace>.<table>.mapping configured")
        user, pwd = props.get("auth.username"), props.get("auth.password")
        bundle = props.get("cloud.secureConnectBundle")
        if bundle:
            b = _secure_bundle(bundle)
            ctx = None
            if b["ca"]:
                import ssl
                ctx = ssl.create_default_context(cadata=b["ca"])
                ctx.check_hostname = False   # Astra's proxy certificate names the host id, not the DNS name
            self.session = CqlSession([f"{b['host']}:{b['port']}"], b["port"], user, pwd, None, False,
                                      ssl_context=ctx)
        else:
            cps = [c.strip() for c in props.get("contactPoints", "localhost").split(",") if c.strip()]
            self.session = CqlSession(cps, int(props.get("port", 9042)), user, pwd, None,
                                      str(props.get("ssl.provider", "None")).lower() not in ("none", ""))
        self.written = 0

    @staticmethod
    def _parse(v):
        if isinstance(v, (bytes, bytearray)):
            v = v.decode("utf-8", "replace")
        if isinstance(v, str):
            t = v.strip()
            if t[:1] in ("{", "["):
                try:
                    import json as _json
                    return _json.loads(t)
                except ValueError:
                    return v
        return v

    def _field(self, expr: str, rec: ConnectRecord):
        root, _, path = expr.partition(".")
        if root == "key":
            base = self._parse(rec.key)
        elif root == "value":
            base = self._parse(rec.value)
        elif root == "header":
            return (rec.headers or {}).get(path)
        else:
            raise ValueError(f"unsupported mapping expression {expr!r} (key[.f], value[.f], header.h)")
        for p in [x for x in path.split(".") if x]:
            base = base.get(p) if isinstance(base, dict) else None
        return base

    def _pk(self, t) -> List[str]:
        if t["pk"] is None:
            rows = self.session.execute(
                "SELECT column_name, kind, position FROM system_schema.columns WHERE keyspace_name = ? "
                "AND table_name = ?", [t["ks"], t["table"]])
            pk = [r for r in rows if r.get("kind") in ("partition_key", "clustering")]
            pk.sort(key=lambda r: (r["kind"] != "partition_key", r.get("position") or 0))
            t["pk"] = [r["column_name"] for r in pk]
        return t["pk"]

    def put(self, records):
        for rec in records:
            for t in self.tables.get(rec.topic, []):
                q = f"{t['ks']}.{t['table']}"
                vals = {col: self._field(expr, rec) for col, expr in t["mapping"] if not col.startswith("__")}
                if rec.value is None:
                    if t["deletes"]:
                        pk = self._pk(t)
                        self.session.execute(f"DELETE FROM {q} WHERE " + " AND ".join(f"{c} = ?" for c in pk),
                                             [vals.get(c) for c in pk])
                    continue
                cols = [c for c, v in vals.items() if v is not None or not t["null_to_unset"]]
                ttl = f" USING TTL {t['ttl']}" if t["ttl"] > 0 else ""
                self.session.execute(f"INSERT INTO {q} ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))}){ttl}",
                                     [vals[c] for c in cols])
                self.written += 1

    def stop(self):
        self.session.close()


class CassandraSinkConnector(Connector):
    def task_class(self):
        return CassandraSinkTask


BUILTIN_CONNECTORS = {
    "org.apache.kafka.connect.file.FileStreamSinkConnector": FileStreamSinkConnector,
    "org.apache.kafka.connect.file.FileStreamSourceConnector": FileStreamSourceConnector,
    "com.datastax.oss.kafka.sink.CassandraSinkConnector": CassandraSinkConnector,
}


def load_connector(class_name: str, code_directory: str = "") -> Connector:
    cls = BUILTIN_CONNECTORS.get(class_name)
    if cls is None:
        py = os.path.join(code_directory, "python") if code_directory else None
        if py and os.path.isdir(py):
            import sys
            if py not in sys.path:
                sys.path.insert(0, py)
        mod, _, attr = class_name.replace(":", ".").rpartition(".")
        try:
            cls = getattr(importlib.import_module(mod), attr)
        except (ImportError, AttributeError, ValueError) as e:
            raise ValueError(f"Kafka Connect connector class {class_name} not found: Java connectors cannot run "
                             f"in this runtime; provide a Python connector (see agents/kafka_connect.py)") from e
    return cls()


def _str_props(cfg: Dict[str, Any]) -> Dict[str, str]:
    return {k: (v if isinstance(v, str) else str(v)) for k, v in cfg.items() if not isinstance(v, (dict, list))}


# ---------------------------------------------------------------- agents
@register_agent("sink")
class KafkaConnectSinkAgent(AgentSink):
    def init(self, configuration: Dict[str, Any]) -> None:
        cfg = dict(configuration)
        self.adapter = dict(cfg.pop("adapterConfig", None) or {})
        self.class_name = cfg.get("connector.class")
        if not self.class_name:
            raise ValueError("Kafka connector sink class is not set (connector.class)")
        self.props = _str_props(cfg)
        self.max_batch = int(self.adapter.get("batchSize", 16384))
        self.linger_s = float(self.adapter.get("lingerTimeMs", 60000)) / 1000.0
        self._buf: List[tuple] = []          # (ConnectRecord, source Record)
        self._pending: List[Record] = []     # put to the task, not yet committed
        self._lock = threading.Lock()
        self._last_flush = time.time()
        self.task: Optional[SinkTask] = None
        # the reference's test hook (KafkaConnectSinkAgent.java:429-431): the first N records
        # fail conversion and go through the bad-record handler (errors.on-failure)
        self._inject_errors = int(self.adapter.get("__test_inject_conversion_error", 0) or 0)
        self._stopped = False

    def set_context(self, context) -> None:
        super().set_context(context)
        self.ctx = context

    def start(self) -> None:
        conn = load_connector(self.class_name, getattr(self.ctx, "code_directory", "") if hasattr(self, "ctx") else "")
        conn.start(self.props)
        self.connector = conn
        self.task = conn.task_class()()
        self.task.start(conn.task_configs(1)[0])

    def handles_commit(self) -> bool:
        return True

    def _stop_on_failure(self) -> None:
        """errors.on-failure=fail: the sink stops before the error propagates; records not
        yet handed to the task are dropped (they stay uncommitted, so they are redelivered)
        -- the reference's close() from the bad-record handler."""
        with self._lock:
            self._stopped = True
            self._buf.clear()

    def write(self, record: Record) -> Future:
        self.processed(1, 0)
        if self._stopped:
            raise RuntimeError("Sink is stopped. Cannot send the records")
        try:
            if self._inject_errors > 0:
                self._inject_errors -= 1
                raise RuntimeError("Injected record conversion error")
            cr = self._to_connect(record)
        except Exception as e:  # noqa: BLE001
            # a record that cannot be converted: skip / dead-letter / fail by errors.on-failure
            # (the handler raises for "fail"; the runner then stops with this cause)
            handler = getattr(getattr(self, "ctx", None), "bad_record_handler", None)
            if handler is None:
                raise
            handler.handle(record, e, self._stop_on_failure)
            return completed(None)
        with self._lock:
            self._buf.append((cr, record))
            full = len(self._buf) >= self.max_batch
        if full:
            self._put()
        return completed(None)

    @staticmethod
    def _to_connect(record: Record) -> "ConnectRecord":
        part = getattr(record, "partition", None)
        off = getattr(record, "offset", None)
        return ConnectRecord(record.origin(), part, off, record.key(), record.value(),
                             {h.key: h.value for h in record.headers()}, record.timestamp())

    def _put(self) -> None:
        with self._lock:
            batch, self._buf = self._buf, []
        if batch:
            self.task.put([b[0] for b in batch])
            with self._lock:
                self._pending.extend(b[1] for b in batch)

    def commit(self) -> None:
        """Called by the runner every loop: put buffered records after the linger time and
        commit what the task's pre_commit acknowledges."""
        if time.time() - self._last_flush < self.linger_s and len(self._buf) < self.max_batch:
            return
        self.flush()

    def flush(self) -> None:
        self._put()
        self._last_flush = time.time()
        with self._lock:
            pending = list(self._pending)
        if not pending:
            return
        offsets: Dict[tuple, int] = {}
        for r in pending:
            key = (r.origin(), getattr(r, "partition", None))
            offsets[key] = max(offsets.get(key, -1), (getattr(r, "offset", None) or 0) + 1)
        ok = self.task.pre_commit(dict(offsets)) or {}
        done = [r for r in pending
                if ok.get((r.origin(), getattr(r, "partition", None)), -1) > (getattr(r, "offset", None) or 0)]
        consumer = getattr(getattr(self, "ctx", None), "consumer", None)
        if consumer is not None and done:
            consumer.commit(done)
        with self._lock:
            ids = {id(r) for r in done}
            self._pending = [r for r in self._pending if id(r) not in ids]

    def close(self) -> None:
        if self.task is not None:
            try:
                if not self._stopped:
                    self.flush()
            finally:
                self.task.stop()
                self.connector.stop()
                self.task = None

    def build_additional_info(self) -> Dict[str, Any]:
        return {"connector.class": self.class_name}


@register_agent("source")
class KafkaConnectSourceAgent(AgentSource):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.cfg = dict(configuration)
        self.class_name = self.cfg.get("connector.class")
        if not self.class_name:
            raise ValueError("Connector class is required")
        self.props = _str_props(self.cfg)
        self.task: Optional[SourceTask] = None
        self._by_id: Dict[int, ConnectRecord] = {}

    def set_context(self, context) -> None:
        super().set_context(context)
        self.ctx = context

    def start(self) -> None:
        conn = load_connector(self.class_name, getattr(getattr(self, "ctx", None), "code_directory", ""))
        conn.start(self.props)
        self.connector = conn
        self.task = conn.task_class()()
        self.task.start(conn.task_configs(1)[0])

    def read(self) -> List[Record]:
        out = []
        for cr in self.task.poll() or []:
            hs = [Header(k, v) for k, v in (cr.headers or {}).items()]
            r = SimpleRecord.of(cr.key, cr.value, hs)
            self._by_id[id(r)] = cr
            out.append(r)
        self.processed(0, len(out))
        return out

    def commit(self, records: List[Record]) -> None:
        for r in records:
            cr = self._by_id.pop(id(r), None)
            if cr is not None:
                self.task.commit_record(cr)
        self.task.commit()

    def close(self) -> None:
        if self.task is not None:
            self.task.stop()
            self.connector.stop()
            self.task = None

    def build_additional_info(self) -> Dict[str, Any]:
        return {"connector.class": self.class_name}
