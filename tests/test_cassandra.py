"""Cassandra / Astra (CQL native protocol v4) datasource, vector-db-sink writer and
cassandra-table / cassandra-keyspace asset managers, against an in-process fake CQL
server: STARTUP + SASL PLAIN, QUERY / PREPARE / EXECUTE frames, a tiny in-memory table
engine (CREATE KEYSPACE / TABLE, INSERT upsert, SELECT by key or ``ORDER BY <vec> ANN OF ?``,
DELETE, ``system_schema`` lookups) and the Cassandra 5 ``VectorType`` column type.

Mirrors the reference's ``CassandraDataSourceTest`` / ``CassandraWriterTest`` /
``CassandraAssetsManagerTest`` (which use a Testcontainers Cassandra; no containers
here, so the server side is a protocol-faithful fake: parity unpinned against a live
Cassandra)."""
import json
import math
import re
import socket
import struct
import threading

import pytest

from langstream_amd.agents.genai.mutable import MutableRecord
from langstream_amd.agents.vector import cql
from langstream_amd.agents.vector.remote import CassandraDataSource, CassandraWriter, parse_cassandra_mapping
from langstream_amd.api.record import SimpleRecord

VEC = "org.apache.cassandra.db.marshal.VectorType(org.apache.cassandra.db.marshal.FloatType, {})"


def _opt(t):
    m = re.fullmatch(r"vector<\s*float\s*,\s*(\d+)\s*>", t)
    if m:
        return (cql.T_CUSTOM, VEC.format(m.group(1)))
    return ({"text": cql.T_VARCHAR, "int": cql.T_INT, "bigint": cql.T_BIGINT, "float": cql.T_FLOAT,
             "double": cql.T_DOUBLE, "boolean": cql.T_BOOLEAN, "uuid": cql.T_UUID}[t],)


def _enc_opt(o):
    out = struct.pack(">H", o[0])
    if o[0] == cql.T_CUSTOM:
        out += cql._string(o[1])
    return out


class FakeCassandra:
    def __init__(self, user="u", password="p"):
        self.user, self.password = user, password
        self.keyspaces = {}           # ks -> {table -> {"cols": [(name, type)], "pk": [..], "kinds": {...}, "rows": {}}}
        self.statements = []
        self.prepared = {}
        self.lock = threading.Lock()
        self.srv = socket.socket()
        self.srv.bind(("127.0.0.1", 0))
        self.srv.listen(8)
        self.port = self.srv.getsockname()[1]
        threading.Thread(target=self._accept, daemon=True).start()

    # ---------------------------------------------------------------- network
    def _accept(self):
        while True:
            try:
                c, _ = self.srv.accept()
            except OSError:
                return
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    @staticmethod
    def _recv(c, n):
        b = b""
        while len(b) < n:
            x = c.recv(n - len(b))
            if not x:
                raise ConnectionError
            b += x
        return b

    def _serve(self, c):
        ks = [None]
        try:
            while True:
                _v, _f, stream, op, n = struct.unpack(">BBhBi", self._recv(c, 9))
                body = self._recv(c, n)
                try:
                    rop, rbody = self._handle(op, body, ks)
                except Exception as e:  # noqa: BLE001
                    rop, rbody = cql.OP_ERROR, struct.pack(">i", 0x2200) + cql._string(str(e))
                c.sendall(struct.pack(">BBhBi", 0x84, 0, stream, rop, len(rbody)) + rbody)
        except (ConnectionError, OSError):
            c.close()

    def _handle(self, op, body, ks):
        r = cql._Reader(body)
        if op == cql.OP_STARTUP:
            return (cql.OP_AUTHENTICATE, cql._string("org.apache.cassandra.auth.PasswordAuthenticator")) \
                if self.user else (cql.OP_READY, b"")
        if op == cql.OP_AUTH_RESPONSE:
            _, u, p = r.bytes().split(b"\x00")
            if (u.decode(), p.decode()) != (self.user, self.password):
                return cql.OP_ERROR, struct.pack(">i", 0x0100) + cql._string("bad credentials")
            return cql.OP_AUTH_SUCCESS, cql._bytes(None)
        if op == cql.OP_QUERY:
            return cql.OP_RESULT, self._run(r.long_string(), [], ks)
        if op == cql.OP_PREPARE:
            q = r.long_string()
            qid = struct.pack(">I", len(self.prepared))
            self.prepared[qid] = q
            names, types = self._binds(q, ks[0])
            meta = struct.pack(">iii", 0x0001, len(names), 0) + cql._string("ks") + cql._string("t")
            meta += b"".join(cql._string(nm) + _enc_opt(t) for nm, t in zip(names, types))
            return cql.OP_RESULT, struct.pack(">i", 4) + struct.pack(">H", 4) + qid + meta + struct.pack(">ii", 4, 0)
        if op == cql.OP_EXECUTE:
            qid = r.short_bytes()
            q = self.prepared[qid]
            _cons, flags = r.short(), r.byte()
            raw = [r.bytes() for _ in range(r.short())] if flags & 1 else []
            _, types = self._binds(q, ks[0])
            return cql.OP_RESULT, self._run(q, [cql.decode_value(t, b) for t, b in zip(types, raw)], ks)
        raise ValueError(f"opcode {op}")

    # ---------------------------------------------------------------- engine
    def _table(self, name, ks):
        k, _, t = name.rpartition(".")
        k = k or ks
        if name.startswith("system_schema."):
            return None
        return self.keyspaces[k][t]

    def _binds(self, q, ks):
        """(names, types) of the ``?`` markers, from the referenced table's schema."""
        m = re.match(r"\s*INSERT INTO (\S+) \(([^)]*)\)", q, re.I)
        if m:
            tab = self._table(m.group(1), ks)
            names = [c.strip() for c in m.group(2).split(",")]
            return names, [_opt(dict(tab["cols"])[n]) for n in names]
        m = re.search(r"FROM (\S+)", q, re.I)
        tab = self._table(m.group(1), ks) if m else None
        names = re.findall(r"(\w+)\s*=\s*\?", q)
        types = [(cql.T_VARCHAR,) if tab is None else _opt(dict(tab["cols"])[n]) for n in names]
        ann = re.search(r"ORDER BY (\w+) ANN OF \?", q, re.I)
        if ann:
            names.append(ann.group(1))
            types.append(_opt(dict(tab["cols"])[ann.group(1)]))
        return names, types

    @staticmethod
    def _rows(cols, rows):
        out = struct.pack(">iii", 2, 0x0001, len(cols)) + cql._string("ks") + cql._string("t")
        out += b"".join(cql._string(n) + _enc_opt(t) for n, t in cols)
        out += struct.pack(">i", len(rows))
        for row in rows:
            out += b"".join(cql._bytes(cql.encode_value(t, row.get(n))) for n, t in cols)
        return out

    def _run(self, q, vals, ks):
        with self.lock:
            self.statements.append((q, vals))
            s = q.strip().rstrip(";")
            if m := re.match(r"USE \"?(\w+)\"?", s, re.I):
                ks[0] = m.group(1)
                return struct.pack(">i", 3) + cql._string(ks[0])
            if m := re.match(r"CREATE KEYSPACE (IF NOT EXISTS )?(\w+)", s, re.I):
                self.keyspaces.setdefault(m.group(2), {})
                return struct.pack(">i", 1)
            if m := re.match(r"DROP KEYSPACE (IF EXISTS )?(\w+)", s, re.I):
                self.keyspaces.pop(m.group(2), None)
                return struct.pack(">i", 1)
            if m := re.match(r"DROP TABLE (IF EXISTS )?(\w+)\.(\w+)", s, re.I):
                self.keyspaces.get(m.group(2), {}).pop(m.group(3), None)
                return struct.pack(">i", 1)
            if m := re.match(r"CREATE TABLE (IF NOT EXISTS )?(?:(\w+)\.)?(\w+)\s*\((.*)\)\s*$", s, re.I | re.S):
                k, t, body = m.group(2) or ks[0], m.group(3), m.group(4)
                pkm = re.search(r"PRIMARY KEY\s*\(\(?([^)]*)\)?(?:,\s*([^)]*))?\)", body, re.I)
                parts = [p.strip() for p in re.sub(r",?\s*PRIMARY KEY\s*\(.*\)\s*$", "", body, flags=re.I | re.S)
                         .split(",") if p.strip()]
                cols = []
                for p in re.findall(r"(\w+)\s+(vector<[^>]*>|\w+)", ",".join(parts)):
                    cols.append(p)
                kinds = {}
                if pkm:
                    for c in pkm.group(1).split(","):
                        kinds[c.strip()] = "partition_key"
                    for c in (pkm.group(2) or "").split(","):
                        if c.strip():
                            kinds[c.strip()] = "clustering"
                self.keyspaces[k].setdefault(t, {"cols": cols, "kinds": kinds, "rows": {}})
                return struct.pack(">i", 1)
            if m := re.match(r"INSERT INTO (\S+) \(([^)]*)\)", s, re.I):
                tab = self._table(m.group(1), ks[0])
                row = dict(zip([c.strip() for c in m.group(2).split(",")], vals))
                key = tuple(row.get(c) for c in tab["kinds"])
                tab["rows"].setdefault(key, {}).update(row)
                return struct.pack(">i", 1)
            if m := re.match(r"DELETE FROM (\S+) WHERE (.*)", s, re.I):
                tab = self._table(m.group(1), ks[0])
                where = dict(zip(re.findall(r"(\w+)\s*=\s*\?", m.group(2)), vals))
                tab["rows"].pop(tuple(where.get(c) for c in tab["kinds"]), None)
                return struct.pack(">i", 1)
            if m := re.match(r"SELECT (.*?) FROM (\S+)(?: WHERE (.*?))?(?: ORDER BY (\w+) ANN OF \?)?"
                             r"(?: LIMIT (\d+))?$", s, re.I):
                sel, name, where_s, ann, limit = m.groups()
                wnames = re.findall(r"(\w+)\s*=\s*\?", where_s or "")
                where = dict(zip(wnames, vals))
                if name.startswith("system_schema."):
                    return self._system(name.split(".")[1], sel, where)
                tab = self._table(name, ks[0])
                rows = [r for r in tab["rows"].values() if all(r.get(k) == v for k, v in where.items())]
                if ann:
                    qv = vals[len(wnames)]
                    rows.sort(key=lambda r: -_cos(r.get(ann), qv))
                if limit:
                    rows = rows[: int(limit)]
                names = [c for c, _ in tab["cols"]] if sel.strip() == "*" else [c.strip() for c in sel.split(",")]
                colt = dict(tab["cols"])
                return self._rows([(n, _opt(colt[n])) for n in names], rows)
            raise ValueError(f"unsupported statement: {q}")

    def _system(self, which, sel, where):
        rows = []
        for k, tabs in self.keyspaces.items():
            if which == "keyspaces":
                rows.append({"keyspace_name": k})
                continue
            for t, tab in tabs.items():
                if which == "tables":
                    rows.append({"keyspace_name": k, "table_name": t})
                    continue
                order = {}
                for c, kind in tab["kinds"].items():
                    order[c] = sum(1 for x, kk in tab["kinds"].items() if kk == kind and x != c and
                                   list(tab["kinds"]).index(x) < list(tab["kinds"]).index(c))
                for c, _ in tab["cols"]:
                    rows.append({"keyspace_name": k, "table_name": t, "column_name": c,
                                 "kind": tab["kinds"].get(c, "regular"), "position": order.get(c, -1)})
        rows = [r for r in rows if all(r.get(a) == b for a, b in where.items())]
        names = [c.strip() for c in sel.split(",")]
        return self._rows([(n, (cql.T_INT,) if n == "position" else (cql.T_VARCHAR,)) for n in names], rows)

    def close(self):
        self.srv.close()


def _cos(a, b):
    if a is None:
        return -2.0
    num = sum(x * y for x, y in zip(a, b))
    return num / (math.sqrt(sum(x * x for x in a)) * math.sqrt(sum(y * y for y in b)) or 1.0)


@pytest.fixture()
def cass():
    f = FakeCassandra()
    yield f
    f.close()


def _ds(cass, **kw):
    return dict({"service": "cassandra", "contact-points": f"127.0.0.1:{cass.port}", "username": "u",
                 "password": "p", "loadBalancing-localDc": "dc1"}, **kw)


SCHEMA = ["CREATE KEYSPACE IF NOT EXISTS vsearch WITH replication = {'class': 'SimpleStrategy', "
          "'replication_factor': 1}",
          "CREATE TABLE IF NOT EXISTS vsearch.documents (filename text, chunk_id int, text text, "
          "embeddings_vector vector<float, 3>, PRIMARY KEY (filename, chunk_id))"]


def test_codecs_roundtrip():
    cases = [((cql.T_VARCHAR,), "héllo"), ((cql.T_INT,), -7), ((cql.T_BIGINT,), 1 << 40), ((cql.T_BOOLEAN,), True),
             ((cql.T_DOUBLE,), 2.5), ((cql.T_VARINT,), -(1 << 70)), ((cql.T_LIST, (cql.T_INT,)), [1, 2, 3]),
             ((cql.T_MAP, (cql.T_VARCHAR,), (cql.T_BIGINT,)), {"a": 1}),
             ((cql.T_CUSTOM, VEC.format(2)), [0.5, -1.0])]
    for t, v in cases:
        assert cql.decode_value(t, cql.encode_value(t, v)) == v
    with pytest.raises(ValueError):
        cql.encode_value((cql.T_CUSTOM, VEC.format(3)), [1.0])


def test_auth_failure(cass):
    with pytest.raises(cql.CqlError):
        cql.session_from_datasource(_ds(cass, password="wrong"))


def test_assets_writer_and_query(cass):
    from langstream_amd.agents.assets import AssetManagerRegistry
    from langstream_amd.api.model import AssetDefinition
    ks_asset = AssetDefinition(id="ks", name="vsearch", asset_type="cassandra-keyspace", creation_mode="create-if-not-exists",
                               deletion_mode="delete",
                               config={"keyspace": "vsearch", "datasource": _ds(cass), "create-statements": SCHEMA[:1]})
    t_asset = AssetDefinition(id="t", name="documents", asset_type="cassandra-table", creation_mode="create-if-not-exists",
                              deletion_mode="delete",
                              config={"keyspace": "vsearch", "table-name": "documents", "datasource": _ds(cass),
                                      "create-statements": SCHEMA[1:]})
    reg = AssetManagerRegistry
    for a in (ks_asset, t_asset):
        m = reg.create(a)
        assert not m.asset_exists()
        m.deploy_asset()
        assert m.asset_exists()

    cfg = {"datasource": _ds(cass), "table-name": "documents", "keyspace": "vsearch",
           "mapping": "filename=value.filename, chunk_id=value.chunk_id, text=value.text, "
                      "embeddings_vector=value.embeddings"}
    assert parse_cassandra_mapping(cfg["mapping"])[1] == ("chunk_id", "value.chunk_id")
    w = CassandraWriter(cfg)
    docs = [("a.pdf", 1, "one", [1.0, 0.0, 0.0]), ("a.pdf", 2, "two", [0.0, 1.0, 0.0]),
            ("b.pdf", 1, "three", [0.7, 0.7, 0.0])]
    for fn, cid, text, emb in docs:
        val = {"filename": fn, "chunk_id": cid, "text": text, "embeddings": emb}
        w.upsert(MutableRecord.from_record(SimpleRecord.of(None, json.dumps(val)))).result(5)
    rows = cass.keyspaces["vsearch"]["documents"]["rows"]
    assert len(rows) == 3 and rows[("a.pdf", 2)]["embeddings_vector"] == [0.0, 1.0, 0.0]

    # query-vector-db style ANN query through the datasource
    ds = CassandraDataSource(_ds(cass))
    out = ds.fetch_data("SELECT filename, chunk_id, text FROM vsearch.documents ORDER BY embeddings_vector "
                        "ANN OF ? LIMIT 2", [[0.9, 0.1, 0.0]])
    assert [r["text"] for r in out] == ["one", "three"]
    out = ds.fetch_data("SELECT * FROM vsearch.documents WHERE filename = ? AND chunk_id = ?", ["b.pdf", 1])
    assert out[0]["embeddings_vector"] == pytest.approx([0.7, 0.7, 0.0], abs=1e-6)

    # null value -> delete by primary key (from system_schema.columns)
    tomb = MutableRecord.from_record(SimpleRecord.of(json.dumps({"filename": "a.pdf", "chunk_id": 1}), None))
    tomb_cfg = dict(cfg, mapping="filename=key.filename, chunk_id=key.chunk_id")
    CassandraWriter(tomb_cfg).upsert(tomb).result(5)
    assert set(rows) == {("a.pdf", 2), ("b.pdf", 1)}
    assert any(q.startswith("DELETE FROM vsearch.documents WHERE filename = ? AND chunk_id = ?")
               for q, _ in cass.statements)
    w.close()
    ds.close()

    reg.create(t_asset).delete_asset_if_exists()
    assert "documents" not in cass.keyspaces["vsearch"]
    reg.create(ks_asset).delete_asset_if_exists()
    assert "vsearch" not in cass.keyspaces


def test_sink_agent_and_query_agent(cass):
    from langstream_amd.agents.vector import VectorDBSinkAgent
    from langstream_amd.agents.vector.datasources import datasource_for
    s = cql.session_from_datasource(_ds(cass))
    for st in SCHEMA:
        s.execute(st)
    s.close()
    a = VectorDBSinkAgent()
    a.init({"datasource": _ds(cass, keyspace="vsearch"), "table-name": "documents",
            "mapping": "filename=value.f, chunk_id=value.c, text=value.t, embeddings_vector=value.e"})
    a.write(SimpleRecord.of(None, json.dumps({"f": "x", "c": 3, "t": "hi", "e": [0.0, 0.0, 1.0]}))).result(5)
    a.close()
    ds = datasource_for(_ds(cass, service="astra", keyspace="vsearch"))
    assert ds.fetch_data("SELECT text FROM documents WHERE filename = ? AND chunk_id = ?", ["x", 3]) == [{"text": "hi"}]
