"""Vector agents: ``query-vector-db`` (PROCESSOR) and ``vector-db-sink`` (SINK).

Parity: VEC/QueryVectorDBAgent.java:27-93 (a QueryStep over a vector datasource),
VEC/VectorDBSinkAgent.java:25-56 (``VectorDatabaseWriter.upsert`` per record; a null
value deletes), VEC/jdbc/JdbcWriter.java:33-208 (prepared UPDATE, then INSERT when no
row matched; DELETE on null value).
"""
from __future__ import annotations

import json
import os
import logging
import threading
from concurrent.futures import Future
from typing import Any, Dict, List

from ...api.agent import AgentProcessor, AgentSink, completed, failed
from ...api.record import SourceRecordAndResult
from ...engine.vector_store import VectorStoreRegistry
from ...engine.vector_store import _safe as _safe_name
from ...runtime.registry import register_agent
from ..genai.el import eval_expression
from ..genai.mutable import MutableRecord
from ..genai.steps import QueryStep
from .datasources import LocalVectorDataSource, SqliteDataSource, datasource_for, jdbc_datasource


@register_agent("query-vector-db")
class QueryVectorDBAgent(AgentProcessor):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.cfg = dict(configuration)
        self.step = QueryStep(self.cfg, datasource_for(self.cfg.get("datasource")))

    def process(self, records, sink) -> None:
        for r in records:
            mr = MutableRecord.from_record(r)
            if not self.step.applies(mr):
                sink(SourceRecordAndResult(r, [r], None))
                continue
            fut = self.step.process_async(mr)

            def done(f, r=r, mr=mr):
                if f.exception() is not None:
                    sink(SourceRecordAndResult(r, None, f.exception()))
                else:
                    out = mr.to_record()
                    self.processed(1, 1)
                    sink(SourceRecordAndResult(r, [out] if out is not None else [], None))

            fut.add_done_callback(done)


class _UpsertBatcher:
    """Coalesces the sink's per-record writes into batched store mutations: one
    normalise + one ``index_copy_`` (+ one WAL append) per batch instead of per record.
    A single flusher thread applies operations in submission order, so per-id order
    is kept; each record's future completes once its batch is applied (and logged)."""

    def __init__(self, collection: str, max_batch: int = 512, linger_s: float = 0.002):
        self.collection = collection
        self.max_batch = max_batch
        self.linger_s = linger_s
        self._q: List[tuple] = []
        self._cv = threading.Condition()
        self._stop = False
        self._t = threading.Thread(target=self._loop, name=f"vector-upsert-{collection}", daemon=True)
        self._t.start()

    def submit(self, op: str, rid, vec, vals) -> Future:
        f: Future = Future()
        with self._cv:
            self._q.append((op, rid, vec, vals, f))
            self._cv.notify()
        return f

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._t.join(5)

    def _loop(self) -> None:
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if not self._q and self._stop:
                    return
                if len(self._q) < self.max_batch and not self._stop:
                    self._cv.wait(self.linger_s)
                batch, self._q = self._q[: self.max_batch], self._q[self.max_batch:]
            i = 0
            while i < len(batch):   # runs of the same operation
                j = i
                while j < len(batch) and batch[j][0] == batch[i][0]:
                    j += 1
                self._apply(batch[i][0], batch[i:j])
                i = j

    def _apply(self, op: str, items) -> None:
        try:
            if op == "d":
                if VectorStoreRegistry.exists(self.collection):
                    VectorStoreRegistry.get(self.collection).delete([it[1] for it in items])
            else:
                dim = len(items[0][2])
                VectorStoreRegistry.get(self.collection, dim).upsert(
                    [it[1] for it in items], [it[2] for it in items], [it[3] for it in items])
            for it in items:
                it[4].set_result(None)
        except Exception as e:  # noqa: BLE001
            for it in items:
                if not it[4].done():
                    it[4].set_exception(e)


class _LocalWriter:
    """fields: id / vector / anything else -> metadata; collection-name."""

    def __init__(self, cfg: Dict[str, Any]):
        self.collection = cfg.get("collection-name") or (cfg.get("datasource") or {}).get("collection-name") \
            or "default"
        self.fields = cfg.get("fields") or []
        names = {f.get("name") for f in self.fields}
        if "vector" not in names:
            raise ValueError("vector-db-sink (local): a field named 'vector' is required")
        self.batcher = _UpsertBatcher(self.collection, int(cfg.get("batch-size", 512)))

    def upsert(self, mr: MutableRecord) -> Future:
        ctx = mr.el_context()
        vals = {f["name"]: eval_expression(f["expression"], ctx) for f in self.fields}
        rid = vals.pop("id", None)
        if rid is None:
            rid = mr.key if mr.key is not None else json.dumps(mr.value, sort_keys=True)[:256]
        if isinstance(rid, (dict, list)):
            rid = json.dumps(rid, sort_keys=True)
        vec = vals.pop("vector")
        if mr.value is None or vec is None:
            return self.batcher.submit("d", rid, None, None)
        if isinstance(vec, str):
            vec = json.loads(vec)
        return self.batcher.submit("u", rid, vec, vals)

    def close(self) -> None:
        self.batcher.close()


class _JdbcWriter:
    def __init__(self, cfg: Dict[str, Any]):
        self.ds = jdbc_datasource(cfg["datasource"])
        self.table = cfg.get("table-name") or cfg.get("table")
        if not self.table:
            raise ValueError("vector-db-sink (jdbc): table-name is required")
        self.fields = cfg.get("fields") or []
        self.pk = [f["name"] for f in self.fields if f.get("primary-key")]
        self.cols = [f["name"] for f in self.fields if not f.get("primary-key")]
        if not self.pk:
            raise ValueError("vector-db-sink (jdbc): at least one primary-key field is required")

    def upsert(self, mr: MutableRecord) -> None:
        ctx = mr.el_context()
        vals = {f["name"]: eval_expression(f["expression"], ctx) for f in self.fields}
        if not isinstance(self.ds, SqliteDataSource):
            self._upsert_generic(mr, vals)
            return
        enc = lambda v: json.dumps(v) if isinstance(v, (list, dict)) else v  # noqa: E731
        ds = self.ds
        with ds.lock:
            where = " AND ".join(f"{c} = ?" for c in self.pk)
            pkv = [enc(vals[c]) for c in self.pk]
            if mr.value is None:
                rowids = [r[0] for r in ds.conn.execute(f"SELECT rowid FROM {self.table} WHERE {where}", pkv)]
                ds.conn.execute(f"DELETE FROM {self.table} WHERE {where}", pkv)
                ds.conn.commit()
                self._mirror_delete(rowids)
                return
            sets = ", ".join(f"{c} = ?" for c in self.cols)
            cur = ds.conn.execute(f"UPDATE {self.table} SET {sets} WHERE {where}",
                                  [enc(vals[c]) for c in self.cols] + pkv) if self.cols else None
            if cur is None or cur.rowcount == 0:
                allc = self.pk + self.cols
                ds.conn.execute(f"INSERT INTO {self.table} ({', '.join(allc)}) VALUES ({', '.join('?' * len(allc))})",
                                [enc(vals[c]) for c in allc])
            ds.conn.commit()
            rowid = ds.conn.execute(f"SELECT rowid FROM {self.table} WHERE {where}", pkv).fetchone()[0]
        self._mirror_upsert(rowid, vals)

    def _upsert_generic(self, mr: MutableRecord, vals: Dict[str, Any]) -> None:
        """JdbcWriter.upsert on a server database: prepared UPDATE, INSERT when it matched
        no row, DELETE for a null value (one statement at a time, autocommit)."""
        ds = self.ds
        where = " AND ".join(f"{c}=?" for c in self.pk)
        pkv = [vals[c] for c in self.pk]
        if mr.value is None:
            ds.execute_statement(f"DELETE FROM {self.table} WHERE {where}", [], pkv)
            return
        n = 0
        if self.cols:
            sets = "=?, ".join(self.cols) + " = ?"
            n = ds.execute_statement(f"UPDATE {self.table} SET {sets} WHERE {where}", [],
                                     [vals[c] for c in self.cols] + pkv)["count"]
        if n == 0:
            allc = self.pk + self.cols
            ds.execute_statement(f"INSERT INTO {self.table} ({', '.join(allc)}) VALUES ({','.join('?' * len(allc))})",
                                 [], [vals[c] for c in allc])

    def _mirror_upsert(self, rowid, vals) -> None:
        for (table, col), name in list(self.ds.vector_cols.items()):
            if table == self.table.lower():
                for k, v in vals.items():
                    if k.lower() == col and isinstance(v, list):
                        VectorStoreRegistry.get(name, len(v), persist=False).upsert([rowid], [v])

    def _mirror_delete(self, rowids) -> None:
        for (table, col), name in list(self.ds.vector_cols.items()):
            if table == self.table.lower() and VectorStoreRegistry.exists(name):
                VectorStoreRegistry.get(name, persist=False).delete(rowids)


def _remote_writers():
    from .remote import WRITERS
    return WRITERS


@register_agent("vector-db-sink")
class VectorDBSinkAgent(AgentSink):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.cfg = dict(configuration)
        ds = self.cfg.get("datasource") or {}
        svc = ds.get("service", "local")
        self._local = svc in ("local", "local-gpu")
        if self._local:
            if ds.get("persist-directory"):
                VectorStoreRegistry.configure(persist_dir=ds["persist-directory"], fsync=ds.get("fsync"))
            self.writer = None   # built in set_context, once the durable default is known
        elif svc in ("jdbc", "sqlite"):
            self.writer = _JdbcWriter(self.cfg)
        elif svc in _remote_writers():
            self.writer = _remote_writers()[svc](self.cfg)
        else:
            from .datasources import UnavailableDataSource
            self.writer = None
            self._unavailable = UnavailableDataSource(svc)

    def set_context(self, context) -> None:
        super().set_context(context)
        if not self._local:
            return
        # Durable by default (parity: the reference sink writes to a database before the
        # offset commit, VEC/jdbc/JdbcWriter.java:140+, and agents get a persistent state
        # directory, API/runner/code/AgentContext.java:64): with no persist-directory /
        # $LANGSTREAM_VECTOR_STORE_DIR configured, the local store's WAL + snapshots live
        # in this agent's persistent state directory (the pod's PVC: the planner gives
        # every vector-db-sink a disk), so a pod restart never loses indexed rows whose
        # source offsets were committed.
        # Only THIS sink's collection is bound to its directory; the process-wide default
        # stays unset, so a later sink of another collection uses its own state dir.
        self.writer = _LocalWriter(self.cfg)
        if VectorStoreRegistry.persist_dir is None:
            d = context.get_persistent_state_directory_for_agent(self.agent_id()) if context is not None else None
            if d:
                VectorStoreRegistry.bind(self.writer.collection,
                                         os.path.join(d, "vector-store", _safe_name(self.writer.collection)))

    def write(self, record) -> Future:
        self.processed(1, 0)
        if self.writer is None and self._local:
            self.writer = _LocalWriter(self.cfg)   # no context was ever set (unit use)
        if self.writer is None:
            try:
                self._unavailable.execute_statement("", [], [])
            except Exception as e:  # noqa: BLE001
                return failed(e)
        try:
            res = self.writer.upsert(MutableRecord.from_record(record))
            return res if isinstance(res, Future) else completed(None)
        except Exception as e:  # noqa: BLE001
            return failed(e)

    def close(self) -> None:
        close = getattr(self.writer, "close", None)
        if close is not None:
            close()
