"""Asset managers for the remote vector databases: ``opensearch-index``,
``solr-collection``, ``milvus-collection`` and ``astra-collection``, over the same REST
clients as the datasources in ``remote.py``.

Parity with the reference providers (``VEC/opensearch/OpenSearchAssetsManagerProvider.java``,
``VEC/solr/SolrAssetsManagerProvider.java``, ``VEC/milvus/MilvusAssetsManagerProvider.java``,
``VEC/astra/AstraVectorDBAssetsManagerProvider.java``):
* opensearch-index: exists = ``HEAD /<index>``; deploy = ``PUT /<index>`` with the
  ``settings`` / ``mappings`` JSON strings of the asset; delete = ``DELETE /<index>``
  (index_not_found is "did not exist");
* solr-collection: exists = ``GET /api/collections/<name>`` (Solr 9 answers 400/404 when
  absent); ``create-statements`` are ``{api: /api/collections | /schema, method, body}``
  sent to the base / collection URL; delete = ``DELETE /api/collections/<name>``;
* milvus-collection: ``create-statements`` are JSON commands ``create-collection``
  (``field-types`` with ``primary-key``/``data-type``/``max-length``/``dimension``),
  ``create-index`` and ``load-collection``, mapped to Milvus REST v2
  (``/v2/vectordb/collections/create``, ``/indexes/create``, ``/collections/load``);
  exists = ``/collections/has``; delete = ``/collections/drop``;
* astra-collection: Data API ``createCollection`` with ``vector-dimension`` (default
  1536), ``findCollections``, ``deleteCollection``.
"""
from __future__ import annotations

import json
from typing import Any, Dict, List

from ..assets import AssetManager
from .remote import AstraVectorDBDataSource, MilvusDataSource, OpenSearchDataSource, SolrDataSource


def _ds_cfg(cfg: Dict[str, Any]) -> Dict[str, Any]:
    ds = dict(cfg.get("datasource") or {})
    return dict(ds.get("configuration") or {}, **{k: v for k, v in ds.items() if k != "configuration"})


def _json_or_none(v: Any) -> Any:
    if v is None or (isinstance(v, str) and not v.strip()):
        return None
    return json.loads(v) if isinstance(v, str) else v


class OpenSearchIndexManager(AssetManager):
    def _ds(self) -> OpenSearchDataSource:
        d = _ds_cfg(self.cfg)
        d.setdefault("index-name", self.cfg.get("index-name"))
        return OpenSearchDataSource(d)

    def asset_exists(self) -> bool:
        ds = self._ds()
        try:
            r = ds.http.s.head(f"{ds.http.base}/{ds.index}", timeout=ds.http.timeout)
            return r.status_code == 200
        finally:
            ds.close()

    def deploy_asset(self) -> None:
        ds = self._ds()
        body: Dict[str, Any] = {}
        for k in ("settings", "mappings"):
            v = _json_or_none(self.cfg.get(k))
            if v is not None:
                body[k] = v
        try:
            res = ds.http.call("PUT", f"/{ds.index}", data=json.dumps(body)) or {}
            if not res.get("acknowledged", True):
                raise RuntimeError(f"Failed to create index {ds.index}: {res}")
        finally:
            ds.close()

    def delete_asset_if_exists(self) -> None:
        ds = self._ds()
        try:
            r = ds.http.s.delete(f"{ds.http.base}/{ds.index}", timeout=ds.http.timeout)
            if r.status_code == 404:
                return
            if r.status_code >= 400:
                raise RuntimeError(f"deleting index {ds.index}: {r.status_code} {r.text[:300]}")
        finally:
            ds.close()


class SolrCollectionManager(AssetManager):
    def _ds(self) -> SolrDataSource:
        d = _ds_cfg(self.cfg)
        d.setdefault("collection-name", self.cfg.get("collection-name"))
        return SolrDataSource(d)

    def _exists(self, ds: SolrDataSource) -> bool:
        r = ds.http.s.get(f"{ds.http.base}/api/collections/{ds.collection}", timeout=ds.http.timeout)
        return r.status_code == 200

    def asset_exists(self) -> bool:
        ds = self._ds()
        try:
            return self._exists(ds)
        finally:
            ds.close()

    def deploy_asset(self) -> None:
        ds = self._ds()
        try:
            for st in self.cfg.get("create-statements") or []:
                body = str(st.get("body") or "").strip()
                body = body if body.startswith("{") else "{" + body + "}"
                api = st.get("api")
                if api == "/api/collections":
                    path = "/api/collections"
                elif api == "/schema":
                    path = f"/solr/{ds.collection}/schema"
                else:
                    raise ValueError(f"Unexpected api value: {api}")
                ds.http.call(st.get("method") or "POST", path, data=body,
                             headers={"Content-Type": "application/json"})
        finally:
            ds.close()

    def delete_asset_if_exists(self) -> None:
        ds = self._ds()
        try:
            if self._exists(ds):
                ds.http.call("DELETE", f"/api/collections/{ds.collection}")
        finally:
            ds.close()


_MILVUS_TYPES = {"varchar": "VarChar", "int64": "Int64", "int32": "Int32", "int16": "Int16", "int8": "Int8",
                 "bool": "Bool", "float": "Float", "double": "Double", "floatvector": "FloatVector",
                 "binaryvector": "BinaryVector", "json": "JSON", "array": "Array", "float16vector": "Float16Vector",
                 "bfloat16vector": "BFloat16Vector", "sparsefloatvector": "SparseFloatVector"}


class MilvusCollectionManager(AssetManager):
    def _ds(self) -> MilvusDataSource:
        return MilvusDataSource(_ds_cfg(self.cfg))

    def _base(self, stmt: Dict[str, Any]) -> Dict[str, Any]:
        body = {"collectionName": stmt.get("collection-name") or self.cfg.get("collection-name")}
        db = stmt.get("database-name") or self.cfg.get("database-name")
        if db:
            body["dbName"] = db
        return body

    def asset_exists(self) -> bool:
        ds = self._ds()
        try:
            res = ds.call("/v2/vectordb/collections/has", self._base({})) or {}
            return bool(res.get("has"))
        finally:
            ds.close()

    def deploy_asset(self) -> None:
        ds = self._ds()
        try:
            for raw in self.cfg.get("create-statements") or []:
                st = json.loads(raw) if isinstance(raw, str) else dict(raw)
                cmd = st.get("command") or ""
                body = self._base(st)
                if cmd == "create-collection":
                    fields: List[Dict[str, Any]] = []
                    for f in st.get("field-types") or []:
                        fd: Dict[str, Any] = {"fieldName": f["name"],
                                              "dataType": _MILVUS_TYPES.get(str(f.get("data-type", "")).lower(),
                                                                            f.get("data-type"))}
                        if f.get("primary-key"):
                            fd["isPrimary"] = True
                        if f.get("auto-id"):
                            body["autoId"] = True
                        params = {}
                        if f.get("max-length") is not None:
                            params["max_length"] = int(f["max-length"])
                        if f.get("dimension") is not None:
                            params["dim"] = int(f["dimension"])
                        if params:
                            fd["elementTypeParams"] = params
                        fields.append(fd)
                    body["schema"] = {"fields": fields}
                    if st.get("description"):
                        body["description"] = st["description"]
                    ds.call("/v2/vectordb/collections/create", body)
                elif cmd == "create-index":
                    idx = {"fieldName": st.get("field-name"), "indexName": st.get("index-name") or st.get("field-name"),
                           "metricType": st.get("metric-type") or "L2"}
                    if st.get("index-type"):
                        idx["params"] = {"index_type": st["index-type"]}
                    body["indexParams"] = [idx]
                    ds.call("/v2/vectordb/indexes/create", body)
                elif cmd == "load-collection":
                    ds.call("/v2/vectordb/collections/load", body)
                else:
                    raise ValueError(f"unknown milvus command {cmd!r}" if cmd else "Command is empty")
        finally:
            ds.close()

    def delete_asset_if_exists(self) -> None:
        if not self.asset_exists():
            return
        ds = self._ds()
        try:
            ds.call("/v2/vectordb/collections/drop", self._base({}))
        finally:
            ds.close()


class AstraCollectionManager(AssetManager):
    def _ds(self) -> AstraVectorDBDataSource:
        return AstraVectorDBDataSource(_ds_cfg(self.cfg))

    def _ks_command(self, ds: AstraVectorDBDataSource, cmd: Dict[str, Any]) -> Dict[str, Any]:
        res = ds.http.call("POST", f"/api/json/v1/{ds.keyspace}", data=json.dumps(cmd)) or {}
        if res.get("errors"):
            raise RuntimeError(f"astra data api: {res['errors']}")
        return res

    def asset_exists(self) -> bool:
        ds = self._ds()
        try:
            res = self._ks_command(ds, {"findCollections": {}})
            return self.cfg.get("collection-name") in ((res.get("status") or {}).get("collections") or [])
        finally:
            ds.close()

    def deploy_asset(self) -> None:
        ds = self._ds()
        try:
            self._ks_command(ds, {"createCollection": {
                "name": self.cfg.get("collection-name"),
                "options": {"vector": {"dimension": int(self.cfg.get("vector-dimension", 1536)),
                                       "metric": "cosine"}}}})
        finally:
            ds.close()

    def delete_asset_if_exists(self) -> None:
        ds = self._ds()
        try:
            self._ks_command(ds, {"deleteCollection": {"name": self.cfg.get("collection-name")}})
        finally:
            ds.close()


MANAGERS = {"opensearch-index": OpenSearchIndexManager, "solr-collection": SolrCollectionManager,
            "milvus-collection": MilvusCollectionManager, "astra-collection": AstraCollectionManager}
