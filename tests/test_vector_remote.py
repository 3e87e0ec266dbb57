"""Remote vector-DB datasources / writers (OpenSearch, Solr, Pinecone, Milvus, Astra
Data API) against an in-process fake HTTP service that records requests.

Request shapes follow the services' public REST APIs; result shapes follow the
reference's datasources (parity unpinned against live services: no network here)."""
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlsplit

import pytest

from langstream_amd.agents.genai.mutable import MutableRecord
from langstream_amd.agents.vector.remote import (AstraVectorDBDataSource, AstraVectorDBWriter, MilvusDataSource,
                                                 MilvusWriter, OpenSearchDataSource, OpenSearchWriter,
                                                 PineconeDataSource, PineconeWriter, SolrDataSource, SolrWriter,
                                                 interpolate)
from langstream_amd.api.record import SimpleRecord


class Fake:
    def __init__(self):
        self.requests = []
        self.responses = {}
        fake = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _do(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n).decode() if n else ""
                u = urlsplit(self.path)
                fake.requests.append({"method": self.command, "path": u.path, "query": parse_qs(u.query),
                                      "body": body, "headers": dict(self.headers)})
                resp = fake.responses.get(u.path, {})
                data = json.dumps(resp).encode()
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            do_GET = do_POST = do_PUT = do_DELETE = _do

            def do_HEAD(self):
                fake.requests.append({"method": "HEAD", "path": urlsplit(self.path).path, "query": {}, "body": "",
                                      "headers": dict(self.headers)})
                self.send_response(200)
                self.send_header("Content-Length", "0")
                self.end_headers()

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.srv.server_address[1]
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def last(self, path):
        return [r for r in self.requests if r["path"] == path][-1]


@pytest.fixture()
def fake():
    f = Fake()
    yield f
    f.srv.shutdown()


def _mr(value, key="k1"):
    return MutableRecord.from_record(SimpleRecord.of(key, json.dumps(value) if value is not None else None))


def test_interpolate_anywhere():
    assert interpolate('{"q": "{!knn f=v topK=5}?", "n": ?}', [[1.0, 2.0], 3]) == \
        '{"q": "{!knn f=v topK=5}[1.0, 2.0]", "n": 3}'


def test_opensearch(fake):
    fake.responses["/idx/_search"] = {"hits": {"hits": [{"_id": "a", "_source": {"text": "t"}, "_score": 0.9,
                                                         "_index": "idx"}]}}
    cfg = {"service": "opensearch", "host": "127.0.0.1", "port": fake.port, "https": False, "username": "u",
           "password": "p", "index-name": "idx"}
    ds = OpenSearchDataSource(cfg)
    rows = ds.fetch_data('{"size": 1, "query": {"knn": {"emb": {"vector": ?, "k": 1}}}}', [[0.5, 0.25]])
    assert rows == [{"id": "a", "document": {"text": "t"}, "score": 0.9, "index": "idx"}]
    sent = json.loads(fake.last("/idx/_search")["body"])
    assert sent["query"]["knn"]["emb"]["vector"] == [0.5, 0.25]
    assert fake.last("/idx/_search")["headers"]["Authorization"].startswith("Basic ")
    fake.responses["/_bulk"] = {"items": [{"index": {"status": 201}}, {"delete": {"status": 404}}]}
    w = OpenSearchWriter({"datasource": cfg, "id": "key", "fields": [{"name": "text", "expression": "value.t"}],
                          "batch-size": 2, "flush-interval": 60000, "bulk-parameters": {"refresh": "wait_for"}})
    f1 = w.upsert(_mr({"t": "hello"}, "doc1"))
    f2 = w.upsert(_mr(None, "doc2"))
    f1.result(5), f2.result(5)
    req = fake.last("/_bulk")
    lines = [json.loads(x) for x in req["body"].strip().split("\n")]
    assert lines == [{"index": {"_index": "idx", "_id": "doc1"}}, {"text": "hello"},
                     {"delete": {"_index": "idx", "_id": "doc2"}}]
    assert req["query"]["refresh"] == ["wait_for"]
    w.close()


def test_solr(fake):
    fake.responses["/solr/docs/select"] = {"response": {"docs": [{"id": "1", "text": "x"}]}}
    cfg = {"service": "solr", "host": "127.0.0.1", "port": fake.port, "collection-name": "docs"}
    rows = SolrDataSource(cfg).fetch_data('{"q": "{!knn f=embeddings topK=5}?"}', [[1.0, 2.0]])
    assert rows == [{"id": "1", "text": "x"}]
    form = parse_qs(fake.last("/solr/docs/select")["body"])
    assert form["q"] == ["{!knn f=embeddings topK=5}[1.0, 2.0]"]
    w = SolrWriter({"datasource": cfg, "fields": [{"name": "id", "expression": "key"},
                                                  {"name": "text", "expression": "value.t"}]})
    w.upsert(_mr({"t": "hi"})).result(5)
    assert json.loads(fake.last("/solr/docs/update")["body"]) == [{"id": "k1", "text": "hi"}]
    w.upsert(_mr(None)).result(5)
    assert json.loads(fake.last("/solr/docs/update")["body"]) == {"delete": {"id": "k1"}}
    assert fake.last("/solr/docs/update")["query"]["commitWithin"] == ["1000"]


def test_pinecone(fake):
    fake.responses["/query"] = {"matches": [{"id": "v1", "score": 0.8, "metadata": {"genre": "comedy", "year": 2019}}]}
    cfg = {"service": "pinecone", "api-key": "KEY", "index-name": "i", "project-name": "p",
           "endpoint": f"http://127.0.0.1:{fake.port}"}
    rows = PineconeDataSource(cfg).fetch_data('{"vector": ?, "topK": 5, "filter": {"genre": "comedy"}}', [[0.1, 0.2]])
    assert rows == [{"genre": "comedy", "year": "2019", "id": "v1"}]
    q = fake.last("/query")
    assert q["headers"]["Api-Key"] == "KEY" and json.loads(q["body"])["topK"] == 5
    w = PineconeWriter({"datasource": cfg, "vector.id": "value.id", "vector.vector": "value.emb",
                        "vector.namespace": "", "vector.metadata.genre": "value.genre"})
    w.upsert(_mr({"id": "x", "emb": [1, 2], "genre": "drama"})).result(5)
    assert json.loads(fake.last("/vectors/upsert")["body"]) == {
        "vectors": [{"id": "x", "values": [1.0, 2.0], "metadata": {"genre": "drama"}}]}


def test_milvus(fake):
    fake.responses["/v2/vectordb/entities/search"] = {"code": 0, "data": [{"id": 3, "distance": 0.1, "text": "t"}]}
    fake.responses["/v2/vectordb/entities/upsert"] = {"code": 0, "data": {"upsertCount": 1}}
    cfg = {"service": "milvus", "url": f"http://127.0.0.1:{fake.port}", "token": "root:Milvus"}
    rows = MilvusDataSource(cfg).fetch_data(
        '{"collection-name": "docs", "vectors": ?, "top-k": 10, "output-fields": ["text"]}', [[0.5, 0.5]])
    assert rows == [{"id": 3, "distance": 0.1, "text": "t"}]
    body = json.loads(fake.last("/v2/vectordb/entities/search")["body"])
    assert body == {"collectionName": "docs", "data": [[0.5, 0.5]], "limit": 10, "outputFields": ["text"]}
    w = MilvusWriter({"datasource": cfg, "collection-name": "docs",
                      "fields": [{"name": "id", "expression": "value.id"}, {"name": "vector", "expression": "value.v"},
                                 {"name": "missing", "expression": "value.nope"}]})
    w.upsert(_mr({"id": 7, "v": [1.0]})).result(5)
    assert json.loads(fake.last("/v2/vectordb/entities/upsert")["body"]) == {
        "collectionName": "docs", "data": [{"id": 7, "vector": [1.0]}]}
    fake.responses["/v2/vectordb/entities/search"] = {"code": 1100, "message": "bad"}
    with pytest.raises(RuntimeError):
        MilvusDataSource(cfg).fetch_data('{"collection-name": "docs", "vectors": ?}', [[0.5]])


def test_astra_data_api(fake):
    path = "/api/json/v1/default_keyspace/docs"
    fake.responses[path] = {"data": {"documents": [{"_id": "d1", "$similarity": 0.9, "text": "hello"}]}}
    cfg = {"service": "astra-vector-db", "token": "AstraCS:x", "endpoint": f"http://127.0.0.1:{fake.port}"}
    rows = AstraVectorDBDataSource(cfg).fetch_data(
        '{"collection-name": "docs", "vector": ?, "limit": 3, "filter": {"lang": "en"}}', [[0.1, 0.2]])
    assert rows == [{"text": "hello", "id": "d1", "similarity": 0.9}]
    cmd = json.loads(fake.last(path)["body"])
    assert cmd == {"find": {"filter": {"lang": "en"}, "sort": {"$vector": [0.1, 0.2]},
                            "options": {"includeSimilarity": True, "limit": 3}}}
    assert fake.last(path)["headers"]["Token"] == "AstraCS:x"
    w = AstraVectorDBWriter({"datasource": cfg, "collection-name": "docs",
                             "fields": [{"name": "id", "expression": "key"}, {"name": "vector", "expression": "value.v"},
                                        {"name": "text", "expression": "value.t"}]})
    w.upsert(_mr({"v": [1.0], "t": "x"})).result(5)
    assert json.loads(fake.last(path)["body"])["findOneAndReplace"]["replacement"] == {
        "_id": "k1", "$vector": [1.0], "text": "x"}
    w.upsert(_mr(None)).result(5)
    assert json.loads(fake.last(path)["body"]) == {"deleteOne": {"filter": {"_id": "k1"}}}
    fake.responses[path] = {"status": {"insertedIds": ["n1"]}}
    out = AstraVectorDBDataSource(cfg).execute_statement(
        '{"collection-name": "docs", "action": "insertOne", "document": {"id": "n1", "vector": ?}}', [], [[0.3]])
    assert out == {"id": "n1"}


def test_sink_agent_uses_remote_writer(fake):
    from langstream_amd.agents.vector import VectorDBSinkAgent
    cfg = {"service": "solr", "host": "127.0.0.1", "port": fake.port, "collection-name": "c"}
    a = VectorDBSinkAgent()
    a.init({"datasource": cfg, "fields": [{"name": "id", "expression": "key"}]})
    a.write(SimpleRecord.of("z", json.dumps({"a": 1}))).result(5)
    assert json.loads(fake.last("/solr/c/update")["body"]) == [{"id": "z"}]


def _asset(atype, cfg):
    from langstream_amd.agents.assets import AssetManagerRegistry
    from langstream_amd.api.model import AssetDefinition
    return AssetManagerRegistry.create(AssetDefinition(id="a", name="a", asset_type=atype, config=cfg))


def test_remote_asset_managers(fake):
    os_ds = {"service": "opensearch", "host": "127.0.0.1", "port": fake.port, "https": False}
    m = _asset("opensearch-index", {"index-name": "idx", "datasource": {"configuration": os_ds},
                                    "settings": '{"index": {"knn": true}}',
                                    "mappings": '{"properties": {"emb": {"type": "knn_vector", "dimension": 3}}}'})
    assert m.asset_exists()
    m.deploy_asset()
    put = [r for r in fake.requests if r["method"] == "PUT" and r["path"] == "/idx"][-1]
    assert json.loads(put["body"])["mappings"]["properties"]["emb"]["dimension"] == 3
    m.delete_asset_if_exists()
    assert fake.requests[-1]["method"] == "DELETE"

    solr = {"service": "solr", "host": "127.0.0.1", "port": fake.port, "collection-name": "documents"}
    m = _asset("solr-collection", {"collection-name": "documents", "datasource": solr, "create-statements": [
        {"api": "/api/collections", "method": "POST", "body": '{"name": "documents", "numShards": 1}'},
        {"api": "/schema", "body": '"add-field": {"name": "emb", "type": "knn_vector"}'}]})
    m.deploy_asset()
    assert json.loads(fake.last("/api/collections")["body"])["name"] == "documents"
    assert json.loads(fake.last("/solr/documents/schema")["body"]) == {"add-field": {"name": "emb", "type": "knn_vector"}}

    milvus = {"service": "milvus", "url": f"http://127.0.0.1:{fake.port}"}
    fake.responses["/v2/vectordb/collections/has"] = {"code": 0, "data": {"has": False}}
    m = _asset("milvus-collection", {"collection-name": "docs", "database-name": "default", "datasource": milvus,
                                     "create-statements": [
                                         json.dumps({"command": "create-collection", "collection-name": "docs",
                                                     "field-types": [{"name": "id", "primary-key": True,
                                                                      "data-type": "Varchar", "max-length": 64},
                                                                     {"name": "vector", "data-type": "FloatVector",
                                                                      "dimension": 4}]}),
                                         json.dumps({"command": "create-index", "field-name": "vector",
                                                     "index-type": "AUTOINDEX", "metric-type": "L2"}),
                                         json.dumps({"command": "load-collection"})]})
    assert not m.asset_exists()
    m.deploy_asset()
    create = json.loads(fake.last("/v2/vectordb/collections/create")["body"])
    assert create["dbName"] == "default" and create["schema"]["fields"][1] == {
        "fieldName": "vector", "dataType": "FloatVector", "elementTypeParams": {"dim": 4}}
    assert json.loads(fake.last("/v2/vectordb/indexes/create")["body"])["indexParams"][0]["metricType"] == "L2"
    assert json.loads(fake.last("/v2/vectordb/collections/load")["body"])["collectionName"] == "docs"

    astra = {"service": "astra-vector-db", "endpoint": f"http://127.0.0.1:{fake.port}", "token": "t"}
    fake.responses["/api/json/v1/default_keyspace"] = {"status": {"collections": ["docs"]}}
    m = _asset("astra-collection", {"collection-name": "docs", "vector-dimension": 8, "datasource": astra})
    assert m.asset_exists()
    m.deploy_asset()
    body = [json.loads(r["body"]) for r in fake.requests if r["path"] == "/api/json/v1/default_keyspace"]
    assert body[-1]["createCollection"]["options"]["vector"]["dimension"] == 8


def test_opensearch_aws_serverless_is_sigv4_signed(fake):
    """A host ending in amazonaws.com is AWS OpenSearch Serverless (OpenSearchDataSource.java
    :113-127): every request is SigV4-signed for service 'aoss' in the configured region,
    with username/password as the access/secret key.  The fake server re-computes the
    signature from what it received."""
    import datetime as dt
    from langstream_amd.utils.cloudauth import sigv4_headers
    fake.responses["/idx/_search"] = {"hits": {"hits": [{"_id": "a", "_source": {"t": 1}, "_score": 1.0}]}}
    cfg = {"service": "opensearch", "host": "https://abc123.us-east-1.aoss.amazonaws.com", "region": "us-east-1",
           "username": "AKIDEXAMPLE", "password": "SECRETKEY", "index-name": "idx"}
    ds = OpenSearchDataSource(cfg)
    assert ds.http.base == "https://abc123.us-east-1.aoss.amazonaws.com"
    ds.http.base = f"http://127.0.0.1:{fake.port}"          # point the transport at the fake
    rows = ds.fetch_data('{"query": {"match_all": {}}}', [])
    assert rows[0]["id"] == "a"
    req = fake.last("/idx/_search")
    h = {k.lower(): v for k, v in req["headers"].items()}
    assert h["authorization"].startswith("AWS4-HMAC-SHA256 Credential=AKIDEXAMPLE/")
    assert "/us-east-1/aoss/aws4_request" in h["authorization"]
    when = dt.datetime.strptime(h["x-amz-date"], "%Y%m%dT%H%M%SZ").replace(tzinfo=dt.timezone.utc)
    again = sigv4_headers("POST", f"http://127.0.0.1:{fake.port}/idx/_search", "us-east-1", "aoss", "AKIDEXAMPLE",
                          "SECRETKEY", req["body"].encode(),
                          {"Content-Type": h["content-type"], "x-amz-content-sha256": h["x-amz-content-sha256"]},
                          now=when)
    assert again["Authorization"] == h["authorization"]
    with pytest.raises(ValueError):
        OpenSearchDataSource({"host": "x.aoss.amazonaws.com", "username": "a", "password": "b"})   # no region
