"""Datasources for ``query`` / ``query-vector-db`` and writers for ``vector-db-sink``.

Parity: F6/F9 (AIA/.../datasource/*, VEC/*): QueryStepDataSource.fetchData(query, params)
/ executeStatement(query, generatedKeys, params) and VectorDatabaseWriter.upsert(record).

MI355X-native services:
* ``local`` / ``local-gpu``: HBM vector collections (engine/vector_store.py) with a JSON
  query language -- ``{"collection-name": "docs", "vector": ?, "top-k": 5,
  "filter": {"field": ?}, "include-vector": false}`` (``?`` = positional params).
* ``jdbc`` by URL (``JdbcDataSourceProvider.java:147-160`` picks the driver the same way):
  - ``jdbc:postgresql://...``: a real server through the in-tree v3 wire client
    (``pgwire.py``: SCRAM-SHA-256 / MD5 auth, prepared statements, typed results);
  - ``jdbc:sqlite:<path>`` (or ``service: sqlite``): SQLite (stdlib) with a
    ``cosine_similarity`` UDF; the RAG pattern ``... ORDER BY cosine_similarity(<vector
    col>, ?) DESC LIMIT k`` runs as a GPU kNN over an HBM mirror of the vector column
    (the reference example ``EX/docker-chatbot/chatbot.yaml:36`` runs that query on HerdDB);
  - ``jdbc:herddb:local`` (HerdDB's embedded, in-process mode) -> an in-process SQLite
    database shared by the process's agents;
  - ``jdbc:herddb:server:<host>:<port>`` -> the local database service that ``langstream
    run --start-database`` starts (the HerdDB of the reference's docker image; herddb.py):
    in its own process straight on its SQLite database (GPU kNN mirror included), from
    other processes over its PostgreSQL-protocol endpoint;
  - any other URL (``jdbc:mysql:...``) fails at init: no driver for it ships in this
    build, and a silent stand-in would not share data between pods.
* cassandra / astra / astra-vector-db / milvus / opensearch / pinecone / solr: the REST /
  CQL clients of ``remote.py`` / ``cql.py``.
"""
from __future__ import annotations

import json
import logging
import math
import re
import sqlite3
import threading
from typing import Any, Dict, List, Optional, Sequence

from ...engine.vector_store import VectorStoreRegistry

log = logging.getLogger(__name__)


class DataSource:

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        raise NotImplementedError

    def execute_statement(self, query: str, generated_keys: Sequence[str], params: List[Any]) -> Dict[str, Any]:
        raise NotImplementedError

    def close(self) -> None:
        pass


_SENT = "\u0000ls-param-"
_TEMPLATES: Dict[str, Any] = {}


def _bind_json(query: str, params: List[Any]) -> Any:
    """Replace bare ``?`` placeholders (outside strings) with the params.  The query is
    parsed once per distinct text with sentinel strings in the placeholders' places and
    bound by substitution: JSON-encoding a 384-float query vector into the text and
    parsing it back cost ~0.4 ms per record."""
    tpl = _TEMPLATES.get(query)
    if tpl is None:
        n = [0]

        def sent(_):
            n[0] += 1
            return json.dumps(f"{_SENT}{n[0] - 1}")
        try:
            tpl = (json.loads(_bind_text(query, None, sent)), n[0])
        except ValueError:
            tpl = (None, 0)
        if len(_TEMPLATES) < 256:
            _TEMPLATES[query] = tpl
    obj, nph = tpl
    if obj is None:
        return json.loads(_bind_text(query, params, None))
    if nph > len(params):
        raise ValueError("not enough parameters for query")
    return _subst(obj, params)


def _subst(o: Any, params: List[Any]) -> Any:
    if isinstance(o, str):
        if o.startswith(_SENT):
            v = params[int(o[len(_SENT):])]
            # JSON types as the text binding produced them (tuples -> lists, keys -> str)
            return v if isinstance(v, (str, int, float, bool, type(None), list)) else json.loads(json.dumps(v))
        return o
    if isinstance(o, dict):
        return {k: _subst(v, params) for k, v in o.items()}
    if isinstance(o, list):
        return [_subst(v, params) for v in o]
    return o


def _bind_text(query: str, params: Optional[List[Any]], sent) -> str:
    out, i, pi, in_str = [], 0, 0, None
    while i < len(query):
        c = query[i]
        if in_str:
            out.append(c)
            if c == "\\":
                out.append(query[i + 1])
                i += 1
            elif c == in_str:
                in_str = None
        elif c in ('"', "'"):
            in_str = c
            out.append(c)
        elif c == "?":
            if sent is not None:
                out.append(sent(pi))
            else:
                if pi >= len(params):
                    raise ValueError("not enough parameters for query")
                out.append(json.dumps(params[pi]))
            pi += 1
        else:
            out.append(c)
        i += 1
    return "".join(out)


class LocalVectorDataSource(DataSource):

    def __init__(self, cfg: Dict[str, Any]):
        self.cfg = cfg
        if cfg.get("persist-directory"):
            VectorStoreRegistry.configure(persist_dir=cfg["persist-directory"], fsync=cfg.get("fsync"))
        self.default_collection = cfg.get("collection-name") or cfg.get("collection") or "default"

    def _store(self, name: Optional[str], dim: Optional[int] = None):
        return VectorStoreRegistry.get(name or self.default_collection, dim)

    def fetch_data(self, query, params):
        return self.fetch_data_batch(query, [params])[0]

    def fetch_data_batch(self, query, params_list):
        """Many queries of the same shape -> ONE kNN kernel launch per collection."""
        parsed = [_bind_json(query, p) if isinstance(query, str) else query for p in params_list]
        out: List[Any] = [None] * len(parsed)
        groups: Dict[tuple, List[int]] = {}
        for i, q in enumerate(parsed):
            if q.get("vector") is None:
                raise ValueError("local vector query needs a 'vector'")
            coll = q.get("collection-name") or q.get("collection") or self.default_collection
            k = int(q.get("top-k", q.get("topK", q.get("limit", 10))))
            flt = q.get("filter") or {}
            key = (coll, k, json.dumps(flt, sort_keys=True), bool(q.get("include-vector", False)))
            groups.setdefault(key, []).append(i)
        from ...engine import dist_knn
        sharded = dist_knn.active()   # DP replicas: global top-k over every rank's shard
        for (coll, k, flt_s, inc), idxs in groups.items():
            if sharded is None and not VectorStoreRegistry.exists(coll):
                for i in idxs:
                    out[i] = []
                continue
            flt = json.loads(flt_s)
            over = k if not flt else k * 4
            vecs = [parsed[i]["vector"] for i in idxs]
            if sharded is not None:
                res = sharded.search(coll, vecs, over, with_vectors=inc).result()
            else:
                res = self._store(coll).search(vecs, over, with_vectors=inc)
            for i, rows in zip(idxs, res):
                if flt:
                    rows = [r for r in rows if all(r.get(f) == v for f, v in flt.items())]
                out[i] = rows[:k]
        return out

    def execute_statement(self, query, generated_keys, params):
        q = _bind_json(query, params) if isinstance(query, str) else query
        action = q.get("action", "upsert")
        coll = q.get("collection-name") or q.get("collection")
        if action == "delete":
            n = self._store(coll).delete([q["id"]]) if VectorStoreRegistry.exists(coll or
                                                                               self.default_collection) else 0
            return {"deleted": n}
        vec = q["vector"]
        store = self._store(coll, len(vec))
        store.upsert([q["id"]], [vec], [q.get("metadata") or {}])
        return {"id": q["id"]}


def _cosine(a, b) -> Optional[float]:
    if a is None or b is None:
        return None
    if isinstance(a, str):
        a = json.loads(a)
    if isinstance(b, str):
        b = json.loads(b)
    num = sum(x * y for x, y in zip(a, b))
    da = math.sqrt(sum(x * x for x in a))
    db = math.sqrt(sum(y * y for y in b))
    return num / (da * db) if da and db else 0.0


_KNN = re.compile(
    r"^\s*select\s+(?P<cols>.+?)\s+from\s+(?P<table>[\w.]+)\s*(?P<where>where\s+.+?)?\s*order\s+by\s+"
    r"cosine_similarity\s*\(\s*(?P<col>\w+)\s*,\s*(?:cast\s*\(\s*)?\?(?:\s+as\s+[\w\s]+\))?\s*\)\s+desc\s+"
    r"limit\s+(?P<k>\d+)\s*;?\s*$", re.I | re.S)

_dbs: Dict[str, "SqliteDataSource"] = {}
_dbs_lock = threading.Lock()


class SqliteDataSource(DataSource):
    """JDBC-compatible SQL on SQLite with GPU kNN for cosine-similarity ORDER BY."""

    def __init__(self, cfg: Dict[str, Any], uri: Optional[str] = None, lock: Optional[Any] = None):
        """``uri`` / ``lock``: open that SQLite URI and serialise on that lock (a database
        this process also serves to other processes: herddb.py)."""
        url = str(cfg.get("url") or cfg.get("path") or "memory")
        m = re.match(r"^jdbc:sqlite:(.+)$", url)
        self.path = m.group(1) if m else (url if cfg.get("path") else None)
        self.name = url
        if uri is not None:
            self.conn = sqlite3.connect(uri, uri=True, check_same_thread=False)
        elif self.path is None or self.path == ":memory:":
            # an in-process database shared by this process's agents (jdbc:herddb:local,
            # jdbc:sqlite::memory:, service sqlite without a path)
            self.conn = sqlite3.connect(f"file:{re.sub(r'[^A-Za-z0-9]', '_', url)}?mode=memory&cache=shared",
                                        uri=True, check_same_thread=False)
        else:
            self.conn = sqlite3.connect(self.path, check_same_thread=False)
        self.conn.create_function("cosine_similarity", 2, _cosine, deterministic=True)
        self.conn.row_factory = sqlite3.Row
        self.lock = lock if lock is not None else threading.RLock()
        self.vector_cols: Dict[tuple, str] = {}  # (table, column) -> store name

    @staticmethod
    def shared(cfg: Dict[str, Any]) -> "SqliteDataSource":
        key = str(cfg.get("url") or cfg.get("path") or "memory")
        with _dbs_lock:
            ds = _dbs.get(key)
            if ds is None:
                ds = SqliteDataSource(cfg)
                _dbs[key] = ds
            return ds

    def _store_name(self, table: str, col: str) -> str:
        return f"sqlite:{self.name}:{table.lower()}:{col.lower()}"

    def _sql_param(self, p):
        if isinstance(p, (list, dict)):
            return json.dumps(p)
        return p

    def fetch_data(self, query, params):
        m = _KNN.match(query)
        if m and not m.group("where"):
            table, col, k = m.group("table"), m.group("col"), int(m.group("k"))
            name = self._store_name(table, col)
            vec = params[-1]
            if isinstance(vec, str):
                vec = json.loads(vec)
            self._ensure_mirror(table, col, len(vec))
            store = VectorStoreRegistry.get(name, persist=False)
            hits = store.search([vec], k)[0] if len(store) else []
            if not hits:
                return []
            ids = [h["id"] for h in hits]
            with self.lock:
                cur = self.conn.execute(
                    f"SELECT {m.group('cols')}, rowid AS __rowid FROM {table} WHERE rowid IN "
                    f"({','.join('?' * len(ids))})", ids)
                rows = {r["__rowid"]: {k2: r[k2] for k2 in r.keys() if k2 != "__rowid"} for r in cur.fetchall()}
            return [_decode_row(rows[i]) for i in ids if i in rows]
        with self.lock:
            cur = self.conn.execute(query, [self._sql_param(p) for p in params])
            return [_decode_row({k: r[k] for k in r.keys()}) for r in cur.fetchall()]

    def execute_statement(self, query, generated_keys, params):
        with self.lock:
            cur = self.conn.execute(query, [self._sql_param(p) for p in params])
            self.conn.commit()
            res = {"count": cur.rowcount}
            if generated_keys:   # the key name JdbcDataSourceProvider.executeStatement returns
                res["generatedKeys"] = {generated_keys[0]: cur.lastrowid}
            self._invalidate_mirrors_for(query)
            return res

    # --- HBM mirror of vector columns
    def _ensure_mirror(self, table: str, col: str, dim: int) -> None:
        key = (table.lower(), col.lower())
        if key in self.vector_cols:
            return
        name = self._store_name(table, col)
        store = VectorStoreRegistry.get(name, dim, persist=False)  # a mirror: rebuilt from SQL
        with self.lock:
            rows = self.conn.execute(f"SELECT rowid, {col} FROM {table}").fetchall()
        ids, vecs = [], []
        for r in rows:
            v = r[1]
            if v is None:
                continue
            v = json.loads(v) if isinstance(v, str) else v
            if len(v) == dim:
                ids.append(r[0])
                vecs.append(v)
        if ids:
            store.upsert(ids, vecs)
        self.vector_cols[key] = name

    def script(self, statements: Sequence[str]) -> None:
        with self.lock:
            for stmt in statements:
                self.conn.executescript(stmt)
            self.conn.commit()
        for stmt in statements:
            self._invalidate_mirrors_for(stmt)

    def table_exists(self, table: str) -> bool:
        with self.lock:
            r = self.conn.execute("SELECT name FROM sqlite_master WHERE type='table' AND lower(name)=lower(?)",
                                  [table]).fetchone()
        return r is not None

    def _invalidate_mirrors_for(self, query: str) -> None:
        ql = query.lower()
        for (table, col), name in list(self.vector_cols.items()):
            if re.search(rf"\b{re.escape(table)}\b", ql):
                VectorStoreRegistry.drop(name)
                self.vector_cols.pop((table, col), None)


def _decode_row(r: Dict[str, Any]) -> Dict[str, Any]:
    out = {}
    for k, v in r.items():
        if isinstance(v, str) and v[:1] == "[" and v[-1:] == "]":
            try:
                v = json.loads(v)
            except ValueError:
                pass
        out[k] = v
    return out


class UnavailableDataSource(DataSource):
    def __init__(self, service: str):
        self.service = service

    def _fail(self, *a, **k):
        raise RuntimeError(f"datasource service '{self.service}' needs its client library and network access, "
                           f"which are not available in this build; use service 'local' (GPU vector store) or "
                           f"'jdbc' (SQLite + GPU kNN)")

    fetch_data = _fail
    execute_statement = _fail


_pg_lock = threading.Lock()
_pg: Dict[tuple, Any] = {}


def jdbc_datasource(cfg: Dict[str, Any]):
    """The JDBC datasource for ``cfg['url']`` (see the module docstring); unsupported URLs
    raise at init."""
    url = str(cfg.get("url") or "")
    svc = cfg.get("service", "jdbc")
    if svc == "sqlite" or url.startswith("jdbc:sqlite:") or url.startswith("jdbc:herddb:local") or \
            (not url and cfg.get("path")):
        return SqliteDataSource.shared(cfg)
    if url.startswith("jdbc:herddb:server:"):
        from .herddb import herddb_datasource
        return herddb_datasource(cfg)
    if url.startswith("jdbc:postgresql:"):
        from .pgwire import PostgresDataSource
        key = (url, str(cfg.get("user")), str(cfg.get("password")))
        with _pg_lock:
            ds = _pg.get(key)
            if ds is None:
                ds = _pg[key] = PostgresDataSource(cfg)
            return ds
    raise ValueError(f"JDBC URL {url or '(none)'!r} is not supported by this build: it speaks "
                     f"jdbc:postgresql:// (wire protocol), jdbc:sqlite:<path>, jdbc:herddb:local "
                     f"(in-process) and jdbc:herddb:server: (the local database service, herddb.py); "
                     f"set one of those")


def reset_jdbc_datasources() -> None:
    """Close the shared PostgreSQL connections (tests)."""
    with _pg_lock:
        for ds in _pg.values():
            ds.close()
        _pg.clear()


def datasource_for(cfg: Optional[Dict[str, Any]]) -> DataSource:
    if cfg is None:
        raise ValueError("datasource is required")
    svc = cfg.get("service", "local")
    if svc in ("local", "local-gpu"):
        return LocalVectorDataSource(cfg)
    if svc in ("jdbc", "sqlite"):
        return jdbc_datasource(cfg)
    from .remote import DATASOURCES
    if svc in DATASOURCES:
        return DATASOURCES[svc](cfg)
    return UnavailableDataSource(svc)
