"""A single-node stand-in that speaks the PostgreSQL v3 wire protocol over SQLite.

For local runs and tests of the ``jdbc:postgresql://`` datasource (``pgwire.py``) without a
PostgreSQL server: ``python -m langstream_amd.cli pg-standalone --port 5432``.  It is a
protocol stand-in, not PostgreSQL: SQL runs on SQLite after a few rewrites
(``$n`` -> ``?n``, ``NOW()`` / ``CURRENT_TIMESTAMP``, ``information_schema.tables``,
ISO-8601 timestamp parameters normalised to PostgreSQL's text form), result column types
are inferred from the values.  What it does implement faithfully is the protocol the
client relies on: startup, trust / cleartext / MD5 / SCRAM-SHA-256 authentication,
ParameterStatus / BackendKeyData / ReadyForQuery, the simple-query cycle, the
extended-query cycle (Parse / Describe / Bind / Execute / Sync / Close) including error
recovery (skip to Sync), and CommandComplete tags.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import os
import re
import socket
import sqlite3
import struct
import threading
from typing import Any, Callable, Dict, List, Optional, Tuple

_TS = re.compile(r"^\d{4}-\d{2}-\d{2}[T ]\d{2}:\d{2}(:\d{2}(\.\d+)?)?(Z|[+-]\d{2}(:?\d{2})?)?$")


def _pg_now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).replace(tzinfo=None).isoformat(sep=" ")


def _norm_param(v: Optional[str]) -> Optional[str]:
    """PostgreSQL's timestamp input accepts ISO-8601 with 'T' and an offset; SQLite
    compares text, so normalise such parameters to the stored ``YYYY-MM-DD HH:MM:SS.ffffff``."""
    if v is None or not _TS.match(v):
        return v
    try:
        d = _dt.datetime.fromisoformat(v.replace("Z", "+00:00"))
    except ValueError:
        return v
    if d.tzinfo is not None:
        d = d.astimezone(_dt.timezone.utc).replace(tzinfo=None)
    return d.isoformat(sep=" ")


def _to_sqlite(sql: str) -> str:
    sql = re.sub(r"\$(\d+)", r"?\1", sql)
    sql = re.sub(r"\bNOW\s*\(\s*\)", "pg_now()", sql, flags=re.I)
    sql = re.sub(r"\binformation_schema\.tables\b",
                 "(SELECT name AS table_name, 'public' AS table_schema, 'BASE TABLE' AS table_type "
                 "FROM sqlite_master WHERE type = 'table')", sql, flags=re.I)
    return sql


def _oid_of(v: Any) -> int:
    if isinstance(v, bool):
        return 16
    if isinstance(v, int):
        return 20
    if isinstance(v, float):
        return 701
    if isinstance(v, (bytes, bytearray)):
        return 17
    return 25


def _text(v: Any) -> Optional[bytes]:
    if v is None:
        return None
    if isinstance(v, bool):
        return b"t" if v else b"f"
    if isinstance(v, float):
        return repr(v).encode()
    if isinstance(v, (bytes, bytearray)):
        return b"\\x" + bytes(v).hex().encode()
    return str(v).encode()


def _decl_oid(decl: str) -> int:
    d = decl.upper()
    if d.startswith("FLOATA") or "ARRAY" in d or d.endswith("[]"):   # HerdDB FLOATA / arrays: JSON text
        return 114
    if "INT" in d:
        return 20
    if any(x in d for x in ("REAL", "FLOA", "DOUB", "NUMERIC", "DECIMAL")):
        return 701
    if "BOOL" in d:
        return 16
    if "JSONB" in d:
        return 3802
    if "JSON" in d:
        return 114
    if "BYTEA" in d or "BLOB" in d:
        return 17
    if "TIMESTAMPTZ" in d:
        return 1184
    if "TIMESTAMP" in d:
        return 1114
    return 25


def _tag(sql: str, rowcount: int, nrows: int) -> str:
    w = sql.strip().split(None, 2)
    verb = w[0].upper() if w else ""
    if verb == "SELECT" or verb == "WITH" or verb == "VALUES":
        return f"SELECT {nrows}"
    if verb == "INSERT":
        return f"INSERT 0 {rowcount if rowcount >= 0 else nrows}"
    if verb in ("UPDATE", "DELETE"):
        return f"{verb} {rowcount if rowcount >= 0 else nrows}"
    if verb in ("CREATE", "DROP", "ALTER") and len(w) > 1:
        return f"{verb} {w[1].upper()}"
    return verb


class PgStandalone:
    """``auth``: 'trust' | 'password' | 'md5' | 'scram-sha-256'."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, users: Optional[Dict[str, str]] = None,
                 auth: str = "scram-sha-256", db_path: Optional[str] = None, db_uri: Optional[str] = None,
                 functions: Optional[Dict[str, Tuple[int, Callable[..., Any]]]] = None,
                 rewrite: Optional[Callable[[str], str]] = None, on_write: Optional[Callable[[str], None]] = None,
                 db_lock: Optional[Any] = None, server_version: str = "16.0 (langstream pg-standalone)"):
        """``db_uri`` / ``db_lock``: serve a SQLite database (and its writer lock) that this
        process shares with in-process users; ``functions``: SQL UDFs per session;
        ``rewrite``: a dialect rewrite applied before the PostgreSQL -> SQLite one;
        ``on_write``: called with every statement that is not a SELECT."""
        self.users = dict(users or {"postgres": "password"})
        self.auth = auth
        self.db_path = db_uri or (f"file:{db_path}" if db_path else f"file:pgstandalone{id(self)}?mode=memory&cache=shared")
        self._keep = sqlite3.connect(self.db_path, uri=True, check_same_thread=False)   # keeps a memory db alive
        self.db_lock = db_lock if db_lock is not None else threading.Lock()
        self.functions = dict(functions or {})
        self.rewrite = rewrite
        self.on_write = on_write
        self.server_version = server_version
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self.host, self.port = self.sock.getsockname()[:2]
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.connections = 0

    @property
    def url(self) -> str:
        return f"jdbc:postgresql://{self.host}:{self.port}/postgres"

    def start(self) -> "PgStandalone":
        t = threading.Thread(target=self._accept, daemon=True, name="pg-standalone")
        t.start()
        self._threads.append(t)
        return self

    def stop(self) -> None:
        self._stop.set()
        try:
            self.sock.close()
        except OSError:
            pass
        self._keep.close()

    def _accept(self) -> None:
        while not self._stop.is_set():
            try:
                c, _ = self.sock.accept()
            except OSError:
                return
            self.connections += 1
            threading.Thread(target=self._serve, args=(c,), daemon=True).start()

    # -- session
    def _serve(self, c: socket.socket) -> None:
        s = _Session(self, c)
        try:
            s.run()
        except (ConnectionError, OSError, struct.error):
            pass
        finally:
            s.close()


class _Session:
    def __init__(self, srv: PgStandalone, c: socket.socket):
        self.srv, self.c = srv, c
        self.buf = bytearray()
        self.db = sqlite3.connect(srv.db_path, uri=True, check_same_thread=False, isolation_level=None)
        self.db.create_function("pg_now", 0, _pg_now)
        self.db.create_function("current_timestamp_pg", 0, _pg_now)
        for fname, (nargs, fn) in srv.functions.items():
            self.db.create_function(fname, nargs, fn, deterministic=True)
        self.stmts: Dict[str, Tuple[str, int]] = {}
        self.portals: Dict[str, Tuple[str, List[Optional[str]]]] = {}
        self.skip_to_sync = False

    def close(self) -> None:
        try:
            self.c.close()
        except OSError:
            pass
        self.db.close()

    def _read(self, n: int) -> bytes:
        while len(self.buf) < n:
            chunk = self.c.recv(65536)
            if not chunk:
                raise ConnectionError("client closed")
            self.buf += chunk
        out = bytes(self.buf[:n])
        del self.buf[:n]
        return out

    def _send(self, t: bytes, body: bytes = b"") -> None:
        self.c.sendall(t + struct.pack("!i", len(body) + 4) + body)

    def _error(self, msg: str, code: str = "42601") -> None:
        self._send(b"E", b"SERROR\0VERROR\0C" + code.encode() + b"\0M" + msg.encode() + b"\0\0")

    def _ready(self) -> None:
        self._send(b"Z", b"I")

    def run(self) -> None:
        ln = struct.unpack("!i", self._read(4))[0]
        body = self._read(ln - 4)
        code = struct.unpack_from("!i", body)[0]
        if code == 80877103:                           # SSLRequest: not offered
            self.c.sendall(b"N")
            ln = struct.unpack("!i", self._read(4))[0]
            body = self._read(ln - 4)
        kv = body[4:].split(b"\0")
        params = {kv[i].decode(): kv[i + 1].decode() for i in range(0, len(kv) - 1, 2) if kv[i]}
        user = params.get("user", "")
        if not self._auth(user):
            return
        self._send(b"R", struct.pack("!i", 0))
        for k, v in (("server_version", self.srv.server_version), ("client_encoding", "UTF8"),
                     ("DateStyle", "ISO, MDY"), ("integer_datetimes", "on"), ("standard_conforming_strings", "on")):
            self._send(b"S", k.encode() + b"\0" + v.encode() + b"\0")
        self._send(b"K", struct.pack("!ii", os.getpid(), 1))
        self._ready()
        while True:
            t = self._read(1)
            ln = struct.unpack("!i", self._read(4))[0]
            body = self._read(ln - 4)
            if t == b"X":
                return
            if t == b"S":
                self.skip_to_sync = False
                self._ready()
                continue
            if self.skip_to_sync:
                continue
            try:
                self._dispatch(t, body)
            except sqlite3.Error as e:
                self._error(str(e), "42000")
                if t == b"Q":
                    self._ready()
                else:
                    self.skip_to_sync = True

    def _auth(self, user: str) -> bool:
        pw = self.srv.users.get(user)
        mode = self.srv.auth
        if mode == "trust":
            return True
        if pw is None:
            self._error(f'password authentication failed for user "{user}"', "28P01")
            return False
        if mode == "password":
            self._send(b"R", struct.pack("!i", 3))
            got = self._password_msg()[:-1].decode()
            ok = hmac.compare_digest(got, pw)
        elif mode == "md5":
            salt = os.urandom(4)
            self._send(b"R", struct.pack("!i", 5) + salt)
            got = self._password_msg()[:-1].decode()
            inner = hashlib.md5((pw + user).encode()).hexdigest()
            ok = hmac.compare_digest(got, "md5" + hashlib.md5(inner.encode() + salt).hexdigest())
        else:
            ok = self._scram(pw)
        if not ok:
            self._error(f'password authentication failed for user "{user}"', "28P01")
        return ok

    def _password_msg(self) -> bytes:
        t = self._read(1)
        ln = struct.unpack("!i", self._read(4))[0]
        body = self._read(ln - 4)
        if t != b"p":
            raise ConnectionError("expected a password message")
        return body

    def _scram(self, pw: str) -> bool:
        self._send(b"R", struct.pack("!i", 10) + b"SCRAM-SHA-256\0\0")
        body = self._password_msg()
        mech, rest = body.split(b"\0", 1)
        if mech != b"SCRAM-SHA-256":
            return False
        n = struct.unpack_from("!i", rest)[0]
        client_first = rest[4:4 + n].decode()
        bare = client_first.split(",", 2)[2]
        cnonce = dict(kv.split("=", 1) for kv in bare.split(","))["r"]
        salt, iters = os.urandom(16), 4096
        snonce = cnonce + base64.b64encode(os.urandom(18)).decode()
        server_first = f"r={snonce},s={base64.b64encode(salt).decode()},i={iters}"
        self._send(b"R", struct.pack("!i", 11) + server_first.encode())
        final = self._password_msg().decode()
        attrs = dict(kv.split("=", 1) for kv in final.split(","))
        if attrs.get("r") != snonce:
            return False
        salted = hashlib.pbkdf2_hmac("sha256", pw.encode(), salt, iters)
        client_key = hmac.new(salted, b"Client Key", hashlib.sha256).digest()
        stored = hashlib.sha256(client_key).digest()
        without_proof = final[:final.rindex(",p=")]
        auth_msg = f"{bare},{server_first},{without_proof}".encode()
        sig = hmac.new(stored, auth_msg, hashlib.sha256).digest()
        proof = base64.b64decode(attrs.get("p", ""))
        recovered = bytes(a ^ b for a, b in zip(proof, sig))
        if len(proof) != 32 or not hmac.compare_digest(hashlib.sha256(recovered).digest(), stored):
            return False
        server_key = hmac.new(salted, b"Server Key", hashlib.sha256).digest()
        server_sig = hmac.new(server_key, auth_msg, hashlib.sha256).digest()
        self._send(b"R", struct.pack("!i", 12) + b"v=" + base64.b64encode(server_sig))
        return True

    # -- queries
    def _nparams(self, sql: str) -> int:
        return max([int(x) for x in re.findall(r"\$(\d+)", sql)] or [0])

    def _sql(self, sql: str) -> str:
        return _to_sqlite(self.srv.rewrite(sql) if self.srv.rewrite else sql)

    def _run(self, sql: str, params: List[Optional[str]]):
        with self.srv.db_lock:
            cur = self.db.execute(self._sql(sql), [_norm_param(p) for p in params])
            rows = cur.fetchall() if cur.description else []
            cols = [d[0] for d in cur.description] if cur.description else None
            rc = cur.rowcount
        if self.srv.on_write is not None and cols is None:
            self.srv.on_write(sql)
        return cols, rows, rc

    def _declared_types(self) -> Dict[str, int]:
        """column name -> type OID from the tables' declared types (the stand-in's answer
        to a Describe whose NULL-parameter run returned no rows)."""
        out: Dict[str, int] = {}
        with self.srv.db_lock:
            tables = [r[0] for r in self.db.execute("SELECT name FROM sqlite_master WHERE type='table'")]
            for t in tables:
                for _cid, name, decl, *_ in self.db.execute(f'PRAGMA table_info("{t}")'):
                    out.setdefault(name.lower(), _decl_oid(decl or ""))
        return out

    def _row_desc(self, cols: List[str], rows, oids: Optional[List[int]] = None) -> bytes:
        body = struct.pack("!h", len(cols))
        for i, c in enumerate(cols):
            if oids is not None:
                oid = oids[i]
            else:
                oid = _oid_of(next((r[i] for r in rows if r[i] is not None), None))
            body += c.encode() + b"\0" + struct.pack("!ihihih", 0, 0, oid, -1, -1, 0)
        return body

    def _data_rows(self, rows) -> None:
        for r in rows:
            body = struct.pack("!h", len(r))
            for v in r:
                t = _text(v)
                body += struct.pack("!i", -1) if t is None else struct.pack("!i", len(t)) + t
            self._send(b"D", body)

    def _dispatch(self, t: bytes, body: bytes) -> None:
        if t == b"Q":
            sql = body[:-1].decode()
            for stmt in [s for s in _split_sql(sql) if s.strip()]:
                cols, rows, rc = self._run(stmt, [])
                if cols is not None:
                    self._send(b"T", self._row_desc(cols, rows))
                    self._data_rows(rows)
                self._send(b"C", _tag(stmt, rc, len(rows)).encode() + b"\0")
            self._ready()
        elif t == b"P":
            name, rest = body.split(b"\0", 1)
            sql, _ = rest.split(b"\0", 1)
            sql_s = sql.decode()
            # validate now, like the server's parse step
            with self.srv.db_lock:
                try:
                    self.db.execute("EXPLAIN " + self._sql(sql_s), [None] * self._nparams(sql_s))
                except sqlite3.Error as e:
                    raise sqlite3.OperationalError(str(e)) from e
            self.stmts[name.decode()] = (sql_s, self._nparams(sql_s))
            self._send(b"1")
        elif t == b"D":
            kind, name = body[:1], body[1:-1].decode()
            if kind == b"S":
                sql, n = self.stmts[name]
                self._send(b"t", struct.pack("!h", n) + struct.pack(f"!{n}i", *([25] * n)))
                # result shape: run on a savepoint with NULL params and roll back
                shape = self._shape(sql, n)
                if shape is None:
                    self._send(b"n")
                else:
                    self._send(b"T", self._row_desc(shape[0], [], shape[1]))
            else:
                sql, params = self.portals[name]
                shape = self._shape(sql, len(params))
                self._send(b"n" if shape is None else b"T",
                           b"" if shape is None else self._row_desc(shape[0], [], shape[1]))
        elif t == b"B":
            portal, rest = body.split(b"\0", 1)
            stmt, rest = rest.split(b"\0", 1)
            nf = struct.unpack_from("!h", rest)[0]
            i = 2 + 2 * nf
            npar = struct.unpack_from("!h", rest, i)[0]
            i += 2
            params: List[Optional[str]] = []
            for _ in range(npar):
                ln = struct.unpack_from("!i", rest, i)[0]
                i += 4
                if ln < 0:
                    params.append(None)
                else:
                    params.append(rest[i:i + ln].decode())
                    i += ln
            self.portals[portal.decode()] = (self.stmts[stmt.decode()][0], params)
            self._send(b"2")
        elif t == b"E":
            portal = body.split(b"\0", 1)[0].decode()
            sql, params = self.portals[portal]
            cols, rows, rc = self._run(sql, params)
            if cols is not None:
                self._data_rows(rows)
            self._send(b"C", _tag(sql, rc, len(rows)).encode() + b"\0")
        elif t == b"C":
            kind, name = body[:1], body[1:-1].decode()
            (self.stmts if kind == b"S" else self.portals).pop(name, None)
            self._send(b"3")
        elif t == b"H":
            pass
        else:
            self._error(f"unsupported message {t!r}", "08P01")
            self.skip_to_sync = True

    def _shape(self, sql: str, n: int) -> Optional[Tuple[List[str], List[int]]]:
        """(column names, type OIDs) of a statement's result, or None (no result)."""
        verb = sql.strip().split(None, 1)[0].upper() if sql.strip() else ""
        if verb not in ("SELECT", "WITH", "VALUES") and "RETURNING" not in sql.upper():
            return None
        rows: list = []
        with self.srv.db_lock:
            self.db.execute("SAVEPOINT pgdescribe")
            try:
                cur = self.db.execute(self._sql(sql), [None] * n)
                cols = [d[0] for d in cur.description] if cur.description else None
                rows = cur.fetchmany(16) if cols else []
            except sqlite3.Error:
                # NULL parameters can violate constraints: read a RETURNING list instead
                m = re.search(r"\bRETURNING\b(.*)$", sql, re.I | re.S)
                if not m:
                    raise
                cols = [c.strip().strip('"').split(".")[-1] for c in m.group(1).rstrip("; ").split(",")]
            finally:
                self.db.execute("ROLLBACK TO pgdescribe")
                self.db.execute("RELEASE pgdescribe")
        if cols is None:
            return None
        decl = self._declared_types()
        oids = []
        for i, c in enumerate(cols):
            v = next((r[i] for r in rows if r[i] is not None), None)
            oids.append(decl.get(c.lower(), 25) if v is None else
                        (decl[c.lower()] if c.lower() in decl and decl[c.lower()] != 25 else _oid_of(v)))
        return cols, oids


def _split_sql(sql: str) -> List[str]:
    out, cur, q = [], [], None
    for ch in sql:
        if q:
            cur.append(ch)
            if ch == q:
                q = None
        elif ch in "'\"":
            q = ch
            cur.append(ch)
        elif ch == ";":
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return out
