"""Remote vector databases for ``query-vector-db`` / ``vector-db-sink`` over their REST
APIs: OpenSearch, Solr, Pinecone, Milvus (REST v2) and Astra DB
(Data API).  The GPU-resident store (``service: local``) is the fast path; these keep
the reference's datasource types usable against external services.

Parity (configuration keys and result shapes) with the reference's
``langstream-vector-agents``:
* queries are JSON templates whose ``?`` placeholders are replaced, in order and
  anywhere in the text, by the JSON of each parameter (``InterpolationUtils.java:30-46``);
* opensearch (``opensearch/OpenSearchDataSource.java:60-238``, ``OpenSearchWriter.java``):
  ``host``/``port`` (9200)/``https`` (true)/``username``/``password``/``index-name``;
  search body -> ``POST /<index>/_search``; rows ``{id, document, score, index}``; the
  writer batches through ``OrderedAsyncBatchExecutor`` (``batch-size`` 10,
  ``flush-interval`` 1000 ms) into ``_bulk`` index / delete (null value) operations with
  ``bulk-parameters`` (refresh, pipeline, routing, timeout, require_alias,
  wait_for_active_shards); ``id`` and ``fields[].expression`` are EL expressions;
* solr (``solr/SolrDataSource.java``, ``SolrWriter.java``): ``protocol``/``host``/``port``/
  ``user``/``password``/``collection-name``; the query map is POSTed as form parameters
  to ``/solr/<collection>/select``; rows are the documents; the writer sends
  ``/update?commitWithin=<commit-within>`` adds, or a delete by id for null values;
* pinecone (``pinecone/PineconeDataSource.java:53-309``, ``PineconeWriter.java:72-170``):
  ``api-key``/``index-name``/``project-name``/``environment``/``endpoint``; query
  ``{vector, filter, topK, includeMetadata, includeValues, namespace}`` -> ``/query``;
  rows ``{id, <metadata as strings>}``; writer ``vector.id``/``vector.vector``/
  ``vector.namespace``/``vector.metadata.*`` -> ``/vectors/upsert`` (``/vectors/delete``
  for null values);
* milvus (``milvus/MilvusDataSource.java``, ``MilvusWriter.java``): ``url`` or
  ``host``/``port`` (19530), ``token`` or ``user``/``password``; query
  ``{collection-name, vectors, top-k, output-fields, filter, database-name}`` ->
  ``/v2/vectordb/entities/search``; writer ``collection-name``/``database-name``/
  ``fields``, ``write-mode`` upsert|insert, null values are skipped (Milvus rejects nulls),
  null record value -> delete by primary key (``primary-key`` field, default ``id``);
* astra-vector-db (``astra/AstraVectorDBDataSource.java``, ``AstraVectorDBWriter.java``):
  ``token``/``endpoint`` (+ ``keyspace``); query ``{collection-name, vector, limit,
  filter, select, include-similarity}`` -> Data API ``find`` sorted by ``$vector``;
  rows ``{id, similarity?, vector?, ...document}``; execute actions ``findOneAndUpdate``,
  ``deleteOne``, ``deleteMany``, ``insertOne``; writer fields ``id``/``vector``/others
  -> ``findOneAndReplace`` with upsert, or ``deleteOne`` for null values.
"""
from __future__ import annotations

import json
import urllib.parse
import hashlib
import logging
import threading
from concurrent.futures import Future
from typing import Any, Dict, List, Optional, Sequence

import requests

from ...api.util import OrderedAsyncBatchExecutor
from ..genai.el import eval_expression
from ..genai.mutable import MutableRecord
from .datasources import DataSource

log = logging.getLogger(__name__)


def interpolate(query: str, params: List[Any]) -> str:
    """Replace the first ``?`` by JSON(param) for each param, anywhere in the text."""
    for p in params:
        i = query.find("?")
        if i < 0:
            break
        query = query[:i] + json.dumps(p) + query[i + 1:]
    return query


def build_object(query: str, params: List[Any]) -> Any:
    try:
        return json.loads(interpolate(query, params))
    except json.JSONDecodeError as e:
        raise ValueError(f"invalid query after interpolation: {e}") from e


def _bool(v: Any, default: bool) -> bool:
    if v is None:
        return default
    if isinstance(v, str):
        return v.strip().lower() in ("true", "1", "yes")
    return bool(v)


class _Http:
    def __init__(self, base: str, headers: Optional[Dict[str, str]] = None, auth=None, timeout: float = 30.0):
        self.base = base.rstrip("/")
        self.s = requests.Session()
        self.s.headers.update(headers or {})
        self.s.auth = auth
        self.timeout = timeout

    def call(self, method: str, path: str, **kw) -> Any:
        r = self.s.request(method, self.base + path, timeout=self.timeout, **kw)
        if r.status_code >= 400:
            raise RuntimeError(f"{method} {self.base}{path} -> {r.status_code}: {r.text[:500]}")
        if not r.content:
            return None
        try:
            return r.json()
        except ValueError:
            return r.text

    def close(self) -> None:
        self.s.close()


class _SigV4Http(_Http):
    """_Http whose every request is SigV4-signed (AWS OpenSearch Serverless, service
    ``aoss``; the signed ``x-amz-content-sha256`` header AOSS requires is included)."""

    def __init__(self, base: str, region: str, service: str, access_key: str, secret_key: str,
                 session_token: Optional[str] = None, headers: Optional[Dict[str, str]] = None,
                 timeout: float = 30.0):
        super().__init__(base, headers, None, timeout)
        self.region, self.service = region, service
        self.ak, self.sk, self.token = access_key, secret_key, session_token

    def call(self, method: str, path: str, **kw) -> Any:
        from ...utils.cloudauth import sigv4_headers
        data = kw.pop("data", None)
        payload = (data.encode() if isinstance(data, str) else (data or b""))
        params = kw.pop("params", None)
        url = self.base + path
        if params:
            url += ("&" if "?" in url else "?") + urllib.parse.urlencode(params)
        hdrs = {**self.s.headers, **(kw.pop("headers", None) or {})}
        hdrs = {k: v for k, v in hdrs.items() if k.lower() in ("content-type",)}
        hdrs["x-amz-content-sha256"] = hashlib.sha256(payload).hexdigest()
        signed = sigv4_headers(method, url, self.region, self.service, self.ak, self.sk, payload, hdrs,
                               session_token=self.token)
        r = self.s.request(method, url, data=payload, headers=signed, timeout=self.timeout, **kw)
        if r.status_code >= 400:
            raise RuntimeError(f"{method} {url} -> {r.status_code}: {r.text[:500]}")
        if not r.content:
            return None
        try:
            return r.json()
        except ValueError:
            return r.text


# ============================================================== OpenSearch
class OpenSearchDataSource(DataSource):
    """OpenSearch REST.  A host ending in ``amazonaws.com`` is AWS OpenSearch Serverless:
    requests are SigV4-signed for service ``aoss`` in ``region`` with ``username`` /
    ``password`` as the access / secret key, over HTTPS on 443
    (OpenSearchDataSource.java:113-127, AwsSdk2Transport); any other host uses basic auth
    (:128-140)."""

    def __init__(self, cfg: Dict[str, Any]):
        host = cfg.get("host")
        if not host:
            raise ValueError("opensearch datasource: missing host")
        host = str(host).replace("https://", "").replace("http://", "").rstrip("/")
        self.index = cfg.get("index-name")
        if host.endswith("amazonaws.com"):
            region = cfg.get("region")
            if not region:
                raise ValueError("opensearch on AWS: region is required")
            if not cfg.get("username") or not cfg.get("password"):
                raise ValueError("opensearch on AWS: username (access key) and password (secret key) are required")
            self.http = _SigV4Http(f"https://{host}", str(region), "aoss", str(cfg["username"]),
                                   str(cfg["password"]), cfg.get("session-token"),
                                   {"Content-Type": "application/json"})
            return
        scheme = "https" if _bool(cfg.get("https"), True) else "http"
        port = int(cfg.get("port") or 9200)
        auth = (cfg.get("username"), cfg.get("password") or "") if cfg.get("username") else None
        self.http = _Http(f"{scheme}://{host}:{port}", {"Content-Type": "application/json"}, auth)

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        body = build_object(query, params)
        res = self.http.call("POST", f"/{self.index}/_search", data=json.dumps(body))
        return [{"id": h.get("_id"), "document": h.get("_source"), "score": h.get("_score"),
                 "index": h.get("_index")} for h in ((res or {}).get("hits") or {}).get("hits") or []]

    def close(self) -> None:
        self.http.close()


class OpenSearchWriter:
    def __init__(self, cfg: Dict[str, Any]):
        self.ds = OpenSearchDataSource(cfg["datasource"])
        self.fields = {f["name"]: f["expression"] for f in (cfg.get("fields") or [])}
        self.id_expr = cfg.get("id")
        bp = cfg.get("bulk-parameters") or {}
        self.params = {k: str(v).lower() if isinstance(v, bool) else str(v) for k, v in bp.items() if v is not None}
        self.executor = OrderedAsyncBatchExecutor(int(cfg.get("batch-size", 10)), self._flush,
                                                  int(cfg.get("flush-interval", 1000)), 1, lambda item: 0)
        self.executor.start()

    def upsert(self, mr: MutableRecord) -> Future:
        ctx = mr.el_context()
        rid = eval_expression(self.id_expr, ctx) if self.id_expr else None
        doc = None if mr.value is None else {k: eval_expression(e, ctx) for k, e in self.fields.items()}
        f: Future = Future()
        self.executor.add((rid, doc, f))
        return f

    def _flush(self, batch, done: Future) -> None:
        lines = []
        for rid, doc, _ in batch:
            meta: Dict[str, Any] = {"_index": self.ds.index}
            if rid is not None:
                meta["_id"] = str(rid)
            if doc is None:
                lines.append(json.dumps({"delete": meta}))
            else:
                lines.append(json.dumps({"index": meta}))
                lines.append(json.dumps(doc))
        try:
            res = self.ds.http.call("POST", "/_bulk", params=self.params, data="\n".join(lines) + "\n",
                                    headers={"Content-Type": "application/x-ndjson"})
            items = (res or {}).get("items") or []
            for (rid, doc, fut), item in zip(batch, items + [None] * (len(batch) - len(items))):
                op = next(iter(item.values())) if item else {}
                err = op.get("error")
                if err and not (doc is None and op.get("status") == 404):
                    fut.set_exception(RuntimeError(f"{err.get('type')} - {err.get('reason')}"))
                else:
                    fut.set_result(None)
            done.set_result(None)
        except Exception as e:  # noqa: BLE001
            for _, _, fut in batch:
                if not fut.done():
                    fut.set_exception(e)
            done.set_exception(e)

    def close(self) -> None:
        self.executor.stop()
        self.ds.close()


# ============================================================== Solr
class SolrDataSource(DataSource):
    def __init__(self, cfg: Dict[str, Any]):
        proto = cfg.get("protocol") or "http"
        host = cfg.get("host") or "localhost"
        port = int(cfg.get("port") or 8983)
        auth = (cfg.get("user"), cfg.get("password") or "") if cfg.get("user") else None
        self.collection = cfg.get("collection-name") or "documents"
        self.http = _Http(f"{proto}://{host}:{port}", auth=auth)

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        q = build_object(query, params)
        form = {k: (v if isinstance(v, str) else json.dumps(v)) for k, v in q.items()}
        form.setdefault("wt", "json")
        res = self.http.call("POST", f"/solr/{self.collection}/select", data=form)
        return list(((res or {}).get("response") or {}).get("docs") or [])

    def close(self) -> None:
        self.http.close()


class SolrWriter:
    def __init__(self, cfg: Dict[str, Any]):
        self.ds = SolrDataSource(cfg["datasource"])
        self.fields = {f["name"]: f["expression"] for f in (cfg.get("fields") or [])}
        self.commit_within = int(cfg.get("commit-within", 1000))

    def upsert(self, mr: MutableRecord) -> Future:
        f: Future = Future()
        try:
            ctx = mr.el_context()
            doc = {k: eval_expression(e, ctx) for k, e in self.fields.items()}
            path = f"/solr/{self.ds.collection}/update"
            params = {"commitWithin": self.commit_within, "wt": "json"}
            if mr.value is None:
                if doc.get("id") is None:
                    raise ValueError("solr delete needs an 'id' field")
                body: Any = {"delete": {"id": doc["id"]}}
            else:
                body = [{k: v for k, v in doc.items() if v is not None}]
            self.ds.http.call("POST", path, params=params, data=json.dumps(body),
                              headers={"Content-Type": "application/json"})
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def close(self) -> None:
        self.ds.close()


# ============================================================== Pinecone
def _pinecone_base(cfg: Dict[str, Any]) -> str:
    if cfg.get("endpoint"):
        return str(cfg["endpoint"])
    return f"https://{cfg['index-name']}-{cfg.get('project-name')}.svc.{cfg.get('environment', 'default')}.pinecone.io"


class PineconeDataSource(DataSource):
    def __init__(self, cfg: Dict[str, Any]):
        for k in ("api-key", "index-name"):
            if not cfg.get(k) and not (k == "index-name" and cfg.get("endpoint")):
                raise ValueError(f"pinecone datasource: missing {k}")
        self.http = _Http(_pinecone_base(cfg), {"Api-Key": str(cfg.get("api-key") or ""),
                                                "Content-Type": "application/json"},
                          timeout=float(cfg.get("server-side-timeout-sec", 10)) + 5)

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        q = build_object(query, params)
        body: Dict[str, Any] = {"topK": int(q.get("topK", 1)), "includeMetadata": bool(q.get("includeMetadata", True)),
                                "includeValues": bool(q.get("includeValues", False))}
        if q.get("vector") is not None:
            body["vector"] = [float(x) for x in q["vector"]]
        if q.get("sparseVector"):
            body["sparseVector"] = q["sparseVector"]
        if q.get("filter"):
            body["filter"] = q["filter"]
        if q.get("namespace") is not None:
            body["namespace"] = q["namespace"]
        res = self.http.call("POST", "/query", data=json.dumps(body)) or {}
        out = []
        for m in res.get("matches") or []:
            row: Dict[str, Any] = {}
            if body["includeMetadata"]:
                for k, v in (m.get("metadata") or {}).items():
                    row[k] = None if v is None else (v if isinstance(v, str) else json.dumps(v) if isinstance(
                        v, (dict, list)) else str(v))
            row["id"] = m.get("id")
            out.append(row)
        return out

    def close(self) -> None:
        self.http.close()


class PineconeWriter:
    def __init__(self, cfg: Dict[str, Any]):
        self.ds = PineconeDataSource(cfg["datasource"])
        self.id_expr = cfg.get("vector.id")
        self.vec_expr = cfg.get("vector.vector")
        self.ns_expr = cfg.get("vector.namespace")
        self.meta = {k[len("vector.metadata."):]: v for k, v in cfg.items() if k.startswith("vector.metadata.")}

    def upsert(self, mr: MutableRecord) -> Future:
        f: Future = Future()
        try:
            ctx = mr.el_context()
            rid = eval_expression(self.id_expr, ctx) if self.id_expr else None
            ns = eval_expression(self.ns_expr, ctx) if self.ns_expr else None
            if rid is None:
                raise ValueError("pinecone: vector.id evaluated to null")
            if mr.value is None:
                body: Dict[str, Any] = {"ids": [str(rid)]}
                if ns:
                    body["namespace"] = ns
                self.ds.http.call("POST", "/vectors/delete", data=json.dumps(body))
            else:
                vec = eval_expression(self.vec_expr, ctx)
                if isinstance(vec, str):
                    vec = json.loads(vec)
                meta = {k: eval_expression(e, ctx) for k, e in self.meta.items()}
                v: Dict[str, Any] = {"id": str(rid), "values": [float(x) for x in vec]}
                if meta:
                    v["metadata"] = {k: x for k, x in meta.items() if x is not None}
                body = {"vectors": [v]}
                if ns:
                    body["namespace"] = ns
                self.ds.http.call("POST", "/vectors/upsert", data=json.dumps(body))
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def close(self) -> None:
        self.ds.close()


# ============================================================== Milvus (REST v2)
class MilvusDataSource(DataSource):
    def __init__(self, cfg: Dict[str, Any]):
        url = cfg.get("url") or f"http://{cfg.get('host') or 'localhost'}:{int(cfg.get('port') or 19530)}"
        tok = cfg.get("token") or (f"{cfg.get('user')}:{cfg.get('password') or ''}" if cfg.get("user") else None)
        hdr = {"Content-Type": "application/json"}
        if tok:
            hdr["Authorization"] = f"Bearer {tok}"
        self.http = _Http(url, hdr)

    def call(self, path: str, body: Dict[str, Any]) -> Any:
        res = self.http.call("POST", path, data=json.dumps(body)) or {}
        if isinstance(res, dict) and res.get("code", 0) not in (0, 200):
            raise RuntimeError(f"milvus {path}: {res.get('code')} {res.get('message')}")
        return res.get("data") if isinstance(res, dict) else res

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        q = build_object(query, params)
        vecs = q.get("vectors")
        if vecs and not isinstance(vecs[0], list):
            vecs = [vecs]
        body: Dict[str, Any] = {"collectionName": q.get("collection-name") or q.get("collectionName"),
                                "data": vecs, "limit": int(q.get("top-k") or q.get("limit") or 10)}
        for src, dst in (("output-fields", "outputFields"), ("filter", "filter"), ("expr", "filter"),
                         ("database-name", "dbName"), ("vector-field-name", "annsField"),
                         ("offset", "offset"), ("params", "searchParams")):
            if q.get(src) is not None:
                body[dst] = q[src]
        return list(self.call("/v2/vectordb/entities/search", body) or [])

    def close(self) -> None:
        self.http.close()


class MilvusWriter:
    def __init__(self, cfg: Dict[str, Any]):
        ds_cfg = cfg["datasource"]
        self.ds = MilvusDataSource(ds_cfg)
        self.collection = cfg.get("collection-name") or ""
        self.db = cfg.get("database-name") or ""
        self.fields = {f["name"]: f["expression"] for f in (cfg.get("fields") or [])}
        self.mode = str(ds_cfg.get("write-mode") or cfg.get("write-mode") or "upsert")
        self.pk = cfg.get("primary-key") or "id"

    def upsert(self, mr: MutableRecord) -> Future:
        f: Future = Future()
        try:
            ctx = mr.el_context()
            row = {}
            for k, e in self.fields.items():
                v = eval_expression(e, ctx)
                if v is not None:  # Milvus rejects nulls
                    row[k] = v
            base: Dict[str, Any] = {"collectionName": self.collection}
            if self.db:
                base["dbName"] = self.db
            if mr.value is None:
                pkv = row.get(self.pk)
                self.ds.call("/v2/vectordb/entities/delete", {**base, "filter": f"{self.pk} in [{json.dumps(pkv)}]"})
            else:
                path = "/v2/vectordb/entities/insert" if self.mode == "insert" else "/v2/vectordb/entities/upsert"
                self.ds.call(path, {**base, "data": [row]})
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def close(self) -> None:
        self.ds.close()


# ============================================================== Astra DB (Data API)
class AstraVectorDBDataSource(DataSource):
    def __init__(self, cfg: Dict[str, Any]):
        endpoint = cfg.get("endpoint")
        if not endpoint:
            raise ValueError("astra-vector-db datasource: missing endpoint")
        self.keyspace = cfg.get("keyspace") or "default_keyspace"
        self.http = _Http(str(endpoint), {"Token": str(cfg.get("token") or ""), "Content-Type": "application/json"})

    def command(self, collection: str, cmd: Dict[str, Any]) -> Dict[str, Any]:
        res = self.http.call("POST", f"/api/json/v1/{self.keyspace}/{collection}", data=json.dumps(cmd)) or {}
        if res.get("errors"):
            raise RuntimeError(f"astra data api: {res['errors']}")
        return res

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        q = build_object(query, params)
        coll = q.pop("collection-name", None)
        vec = q.pop("vector", None)
        limit = q.pop("limit", None)
        sim = _bool(q.pop("include-similarity", None), True)
        flt = q.pop("filter", None) or {}
        select = q.pop("select", None)
        find: Dict[str, Any] = {"filter": flt}
        opts: Dict[str, Any] = {}
        if vec is not None:
            find["sort"] = {"$vector": [float(x) for x in vec]}
            opts["includeSimilarity"] = sim
        if limit is not None:
            opts["limit"] = int(limit)
        if select:
            find["projection"] = {s: 1 for s in select}
        if opts:
            find["options"] = opts
        docs = ((self.command(coll, {"find": find}).get("data") or {}).get("documents")) or []
        out = []
        for d in docs:
            r = {k: v for k, v in d.items() if k not in ("_id", "$similarity", "$vector")}
            r["id"] = d.get("_id")
            if "$similarity" in d:
                r["similarity"] = d["$similarity"]
            if "$vector" in d:
                r["vector"] = d["$vector"]
            out.append(r)
        return out

    def execute_statement(self, query: str, generated_keys: Sequence[str], params: List[Any]) -> Dict[str, Any]:
        q = build_object(query, params)
        coll = q.pop("collection-name", None)
        action = q.pop("action", None)
        if action == "findOneAndUpdate":
            cmd = {"filter": q.pop("filter", {}), "update": q.pop("update", {}),
                   "options": {"returnDocument": q.pop("return-document", "after")}}
            st = self.command(coll, {"findOneAndUpdate": cmd}).get("status") or {}
            return {"count": st.get("modifiedCount", 0)}
        if action in ("deleteOne", "deleteMany"):
            st = self.command(coll, {action: {"filter": q.pop("filter", {})}}).get("status") or {}
            return {"count": st.get("deletedCount", 0)}
        if action == "insertOne":
            doc = dict(q.pop("document", {}))
            d: Dict[str, Any] = {}
            for k, v in doc.items():
                d["_id" if k == "id" else "$vector" if k == "vector" else k] = v
            st = self.command(coll, {"insertOne": {"document": d}}).get("status") or {}
            ids = st.get("insertedIds") or [None]
            return {"id": ids[0]}
        raise ValueError(f"astra-vector-db: unsupported action {action}")

    def close(self) -> None:
        self.http.close()


class AstraVectorDBWriter:
    def __init__(self, cfg: Dict[str, Any]):
        self.ds = AstraVectorDBDataSource(cfg["datasource"])
        self.collection = cfg.get("collection-name") or ""
        self.fields = {f["name"]: f["expression"] for f in (cfg.get("fields") or [])}

    def upsert(self, mr: MutableRecord) -> Future:
        f: Future = Future()
        try:
            ctx = mr.el_context()
            doc: Dict[str, Any] = {}
            for k, e in self.fields.items():
                v = eval_expression(e, ctx)
                doc["_id" if k == "id" else "$vector" if k == "vector" else k] = v
            if "_id" not in doc:
                raise ValueError("astra-vector-db sink needs an 'id' field")
            if mr.value is None:
                self.ds.command(self.collection, {"deleteOne": {"filter": {"_id": doc["_id"]}}})
            else:
                self.ds.command(self.collection, {"findOneAndReplace": {
                    "filter": {"_id": doc["_id"]}, "replacement": doc, "options": {"upsert": True}}})
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def close(self) -> None:
        self.ds.close()


DATASOURCES = {"opensearch": OpenSearchDataSource, "solr": SolrDataSource, "pinecone": PineconeDataSource,
               "milvus": MilvusDataSource, "astra-vector-db": AstraVectorDBDataSource}
WRITERS = {"opensearch": OpenSearchWriter, "solr": SolrWriter, "pinecone": PineconeWriter, "milvus": MilvusWriter,
           "astra-vector-db": AstraVectorDBWriter}
_lock = threading.Lock()


# ============================================================== Cassandra / Astra (CQL native protocol)
class CassandraDataSource(DataSource):
    """``service: cassandra | astra`` (``AIA/.../datasource/CassandraDataSource.java``): the
    query is a CQL statement with ``?`` markers bound positionally through PREPARE/EXECUTE;
    rows come back as maps, vector columns as lists of floats."""

    def __init__(self, cfg: Dict[str, Any]):
        self.cfg = cfg
        self._session = None
        self._lock = threading.Lock()

    @property
    def session(self):
        with self._lock:
            if self._session is None:
                from .cql import session_from_datasource
                self._session = session_from_datasource(self.cfg)
            return self._session

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        return self.session.execute(query, params)

    def execute_statement(self, query: str, generated_keys: Sequence[str], params: List[Any]) -> Dict[str, Any]:
        self.session.execute(query, params)
        return {}

    def close(self) -> None:
        if self._session is not None:
            self._session.close()


def parse_cassandra_mapping(mapping: str) -> List[tuple]:
    """``"col=value.field, col2=key"`` (the DataStax sink mapping) -> [(col, EL expression)]."""
    out = []
    for part in (mapping or "").split(","):
        if not part.strip():
            continue
        col, _, expr = part.partition("=")
        out.append((col.strip(), expr.strip()))
    return out


class CassandraWriter:
    """``vector-db-sink`` on Cassandra / Astra (``VEC/cassandra/CassandraWriter.java``):
    ``table``/``table-name`` + ``keyspace`` + ``mapping``; each record is one INSERT of the
    mapped columns (an upsert in Cassandra); a null record value deletes the row by its
    primary key (read from ``system_schema.columns``)."""

    def __init__(self, cfg: Dict[str, Any]):
        self.ds = CassandraDataSource(cfg["datasource"])
        table = cfg.get("table") or cfg.get("table-name")
        if not table:
            raise ValueError("vector-db-sink (cassandra): table-name is required")
        self.keyspace = cfg.get("keyspace") or cfg["datasource"].get("keyspace")
        self.table = table
        self.qualified = f"{self.keyspace}.{table}" if self.keyspace else table
        self.mapping = parse_cassandra_mapping(cfg.get("mapping", ""))
        if not self.mapping:
            raise ValueError("vector-db-sink (cassandra): mapping is required")
        self._pk: Optional[List[str]] = None

    def _primary_key(self) -> List[str]:
        if self._pk is None:
            rows = self.ds.session.execute(
                "SELECT column_name, kind, position FROM system_schema.columns WHERE keyspace_name = ? "
                "AND table_name = ?", [self.keyspace, self.table])
            pk = [r for r in rows if r.get("kind") in ("partition_key", "clustering")]
            pk.sort(key=lambda r: (r["kind"] != "partition_key", r.get("position") or 0))
            self._pk = [r["column_name"] for r in pk]
        return self._pk

    def upsert(self, mr: MutableRecord) -> Future:
        f: Future = Future()
        try:
            ctx = mr.el_context()
            vals = {col: eval_expression(expr, ctx) for col, expr in self.mapping}
            if mr.value is None:
                pk = self._primary_key()
                where = " AND ".join(f"{c} = ?" for c in pk)
                self.ds.session.execute(f"DELETE FROM {self.qualified} WHERE {where}", [vals.get(c) for c in pk])
            else:
                cols = list(vals)
                self.ds.session.execute(
                    f"INSERT INTO {self.qualified} ({', '.join(cols)}) VALUES ({', '.join('?' * len(cols))})",
                    [vals[c] for c in cols])
            f.set_result(None)
        except Exception as e:  # noqa: BLE001
            f.set_exception(e)
        return f

    def close(self) -> None:
        self.ds.close()


DATASOURCES.update({"cassandra": CassandraDataSource, "astra": CassandraDataSource})
WRITERS.update({"cassandra": CassandraWriter, "astra": CassandraWriter})
