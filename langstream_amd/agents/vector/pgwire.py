"""PostgreSQL frontend/backend protocol v3 client (the ``jdbc:postgresql://`` datasource).

Parity: ``JdbcDataSourceProvider.java:147-160`` opens ``DriverManager.getConnection(url,
props)`` with the PostgreSQL JDBC driver the application ships
(``examples/applications/query-postgresql-chat-history/configuration.yaml:20-36``); the
``query`` step then runs ``PreparedStatement``s with ``setObject`` parameters
(``fetchData`` / ``executeStatement``), ``jdbc-table`` assets run their create / delete
statements, and ``vector-db-sink`` runs prepared UPDATE / INSERT / DELETE
(``VEC/jdbc/JdbcWriter.java:33-208``).  No PostgreSQL driver ships in this image, so this
module speaks the wire protocol itself:

* startup (protocol 3.0) with trust, cleartext, MD5 and SCRAM-SHA-256 authentication;
  optional TLS (``ssl=true`` / ``sslmode=require|verify-ca|verify-full``, certificates
  verified against the system store or ``sslrootcert``);
* prepared statements like PgJDBC's server-side ones: ``Parse`` (named, cached per query
  text) + ``Describe`` once -- the server's inferred parameter types pick each value's
  text encoding (arrays ``{...}``, json, everything else its text form) -- then ``Bind`` /
  ``Execute`` / ``Sync`` per call; JDBC ``?`` placeholders become ``$n``;
* text-format results decoded by type OID (integers, floats, numeric, bool, text, json /
  jsonb, arrays, bytea; pgvector-style ``[..]`` values become lists; date / time values
  stay in PostgreSQL's text form);
* generated keys like PgJDBC: ``RETURNING <keys>`` appended to the statement;
* the simple-query protocol for DDL scripts (asset ``create-statements``).
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import json
import os
import re
import socket
import ssl
import struct
import threading
import urllib.parse
from typing import Any, Dict, List, Optional, Sequence, Tuple

PROTOCOL_3 = 196608
SSL_REQUEST = 80877103


class PgError(Exception):
    """An ErrorResponse from the server (``fields``: severity S, code C, message M, ...)."""

    def __init__(self, fields: Dict[str, str]):
        self.fields = fields
        super().__init__(f"{fields.get('S', 'ERROR')} {fields.get('C', '')}: {fields.get('M', '')}".strip())

    @property
    def sqlstate(self) -> str:
        return self.fields.get("C", "")


# ---------------------------------------------------------------- URL
def parse_jdbc_url(url: str, props: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """``jdbc:postgresql://host[:port][,host2...]/[database][?k=v&...]`` (+ ``user`` /
    ``password`` / ``ssl`` / ``sslmode`` from the datasource properties, which the URL's
    query parameters override like PgJDBC)."""
    m = re.match(r"^jdbc:postgresql://([^/?]*)(?:/([^?]*))?(?:\?(.*))?$", url.strip())
    if not m:
        raise ValueError(f"not a PostgreSQL JDBC URL: {url!r}")
    hosts = m.group(1) or "localhost"
    host_port = hosts.split(",")[0]
    if host_port.startswith("["):                       # [ipv6]:port
        h, _, rest = host_port[1:].partition("]")
        port = int(rest[1:]) if rest.startswith(":") else 5432
    elif host_port.count(":") == 1:
        h, p = host_port.split(":")
        port = int(p) if p else 5432
    else:
        h, port = host_port, 5432
    out: Dict[str, Any] = {}
    for k, v in (props or {}).items():
        if k in ("user", "password", "ssl", "sslmode", "sslrootcert", "ApplicationName", "connectTimeout",
                 "currentSchema", "options"):
            out[k] = v
    for k, v in urllib.parse.parse_qsl(m.group(3) or ""):
        out[k] = v
    out["host"] = h or "localhost"
    out["port"] = port
    out["database"] = urllib.parse.unquote(m.group(2) or "") or out.get("user") or "postgres"
    return out


def jdbc_to_pg_sql(sql: str) -> Tuple[str, int]:
    """JDBC ``?`` placeholders -> ``$1..$n`` outside string literals, quoted identifiers
    and comments (``??`` is a literal ``?`` like PgJDBC's escape)."""
    out: List[str] = []
    i, n, k = 0, len(sql), 0
    while i < n:
        c = sql[i]
        if c == "'" or c == '"':
            j = i + 1
            while j < n:
                if sql[j] == c:
                    if j + 1 < n and sql[j + 1] == c:
                        j += 2
                        continue
                    break
                j += 1
            out.append(sql[i:j + 1])
            i = j + 1
        elif c == "-" and sql.startswith("--", i):
            j = sql.find("\n", i)
            j = n if j < 0 else j
            out.append(sql[i:j])
            i = j
        elif c == "/" and sql.startswith("/*", i):
            j = sql.find("*/", i + 2)
            j = n if j < 0 else j + 2
            out.append(sql[i:j])
            i = j
        elif c == "$" and i + 1 < n and (sql[i + 1] == "$" or sql[i + 1].isalpha() or sql[i + 1] == "_"):
            # dollar-quoted string $tag$ ... $tag$
            mm = re.match(r"\$([A-Za-z_][A-Za-z_0-9]*)?\$", sql[i:])
            if mm:
                tag = mm.group(0)
                j = sql.find(tag, i + len(tag))
                j = n if j < 0 else j + len(tag)
                out.append(sql[i:j])
                i = j
            else:
                out.append(c)
                i += 1
        elif c == "?":
            if i + 1 < n and sql[i + 1] == "?":
                out.append("?")
                i += 2
            else:
                k += 1
                out.append(f"${k}")
                i += 1
        else:
            out.append(c)
            i += 1
    return "".join(out), k


# ---------------------------------------------------------------- value codecs
_ARRAY_ELEM = {1000: 16, 1005: 21, 1007: 23, 1016: 20, 1021: 700, 1022: 701, 1231: 1700, 1009: 25, 1015: 1043,
               1014: 1042, 199: 114, 3807: 3802, 1182: 1082, 1115: 1114, 1185: 1184}
_JSON_OIDS = (114, 3802)


def _array_literal(v: Sequence[Any]) -> str:
    parts = []
    for x in v:
        if x is None:
            parts.append("NULL")
        elif isinstance(x, (list, tuple)):
            parts.append(_array_literal(x))
        elif isinstance(x, bool):
            parts.append("t" if x else "f")
        elif isinstance(x, (int, float)):
            parts.append(repr(x) if isinstance(x, float) else str(x))
        else:
            s = str(x).replace("\\", "\\\\").replace('"', '\\"')
            parts.append(f'"{s}"')
    return "{" + ",".join(parts) + "}"


def encode_param(v: Any, oid: int) -> Optional[bytes]:
    """Text-format parameter for a server-inferred type ``oid`` (``setObject``)."""
    import datetime as _dt
    if v is None:
        return None
    if isinstance(v, bool):
        return b"t" if v else b"f"
    if isinstance(v, (bytes, bytearray, memoryview)):
        return b"\\x" + bytes(v).hex().encode()
    if isinstance(v, (list, tuple)):
        if oid in _ARRAY_ELEM:
            return _array_literal(v).encode()
        return json.dumps(list(v)).encode()           # json / jsonb / pgvector '[..]'
    if isinstance(v, dict):
        return json.dumps(v).encode()
    if isinstance(v, float):
        return repr(v).encode()
    if isinstance(v, (_dt.datetime, _dt.date, _dt.time)):
        return v.isoformat(sep=" ").encode() if isinstance(v, _dt.datetime) else v.isoformat().encode()
    return str(v).encode()


def _parse_array(s: str, elem_oid: int) -> Any:
    """PostgreSQL array text ``{a,"b c",NULL,{1,2}}`` -> nested lists."""
    pos = 0

    def parse():
        nonlocal pos
        assert s[pos] == "{"
        pos += 1
        out: List[Any] = []
        if s[pos] == "}":
            pos += 1
            return out
        while True:
            if s[pos] == "{":
                out.append(parse())
            elif s[pos] == '"':
                pos += 1
                buf = []
                while s[pos] != '"':
                    if s[pos] == "\\":
                        pos += 1
                    buf.append(s[pos])
                    pos += 1
                pos += 1
                out.append(decode_value("".join(buf), elem_oid))
            else:
                j = pos
                while s[j] not in ",}":
                    j += 1
                tok = s[pos:j]
                pos = j
                out.append(None if tok == "NULL" else decode_value(tok, elem_oid))
            if s[pos] == ",":
                pos += 1
                continue
            pos += 1                               # '}'
            return out

    if s.startswith("["):                          # explicit bounds [1:3]={...}
        s = s[s.index("=") + 1:]
    return parse()


def decode_value(s: Optional[str], oid: int) -> Any:
    if s is None:
        return None
    if oid in (20, 21, 23, 26, 28):
        return int(s)
    if oid in (700, 701):
        return float(s)
    if oid == 1700:
        if s in ("NaN", "Infinity", "-Infinity"):
            return float(s)
        return int(s) if re.fullmatch(r"-?\d+", s) else float(s)
    if oid == 16:
        return s == "t"
    if oid in _JSON_OIDS:
        return json.loads(s)
    if oid == 17:
        return bytes.fromhex(s[2:]) if s.startswith("\\x") else s.encode("latin-1")
    if oid in _ARRAY_ELEM:
        return _parse_array(s, _ARRAY_ELEM[oid])
    if s[:1] == "[" and s[-1:] == "]" and oid not in (25, 1043, 1042, 19):
        try:                                       # pgvector and similar '[1,2,3]' types
            return json.loads(s)
        except ValueError:
            return s
    return s


# ---------------------------------------------------------------- SCRAM-SHA-256 (RFC 5802 / 7677)
def _scram_client_first(nonce: str) -> Tuple[str, str]:
    bare = f"n=,r={nonce}"
    return "n,," + bare, bare


def scram_client_final(password: str, client_first_bare: str, server_first: str) -> Tuple[str, bytes]:
    attrs = dict(kv.split("=", 1) for kv in server_first.split(","))
    salt = base64.b64decode(attrs["s"])
    iters = int(attrs["i"])
    salted = hashlib.pbkdf2_hmac("sha256", password.encode(), salt, iters)
    client_key = hmac.new(salted, b"Client Key", hashlib.sha256).digest()
    stored = hashlib.sha256(client_key).digest()
    without_proof = f"c=biws,r={attrs['r']}"
    auth_msg = f"{client_first_bare},{server_first},{without_proof}".encode()
    sig = hmac.new(stored, auth_msg, hashlib.sha256).digest()
    proof = bytes(a ^ b for a, b in zip(client_key, sig))
    server_key = hmac.new(salted, b"Server Key", hashlib.sha256).digest()
    server_sig = hmac.new(server_key, auth_msg, hashlib.sha256).digest()
    return f"{without_proof},p={base64.b64encode(proof).decode()}", server_sig


# ---------------------------------------------------------------- connection
class _Stmt:
    __slots__ = ("name", "param_oids", "columns")

    def __init__(self, name: str, param_oids: List[int], columns: Optional[List[Tuple[str, int]]]):
        self.name, self.param_oids, self.columns = name, param_oids, columns


class PgConnection:
    """One backend connection; thread-safe (calls serialise on a lock); autocommit."""

    def __init__(self, host: str, port: int, user: str, password: Optional[str], database: str,
                 timeout: float = 30.0, ssl_mode: str = "disable", ssl_root_cert: Optional[str] = None,
                 application_name: str = "langstream", options: Optional[Dict[str, str]] = None):
        self.host, self.port, self.user, self.password, self.database = host, port, user, password, database
        self.params: Dict[str, str] = {}
        self.backend_key: Optional[Tuple[int, int]] = None
        self.lock = threading.RLock()
        self._stmts: Dict[str, _Stmt] = {}
        self._nstmt = 0
        self._buf = bytearray()
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if ssl_mode in ("require", "verify-ca", "verify-full"):
            self._start_tls(ssl_mode, ssl_root_cert)
        startup = {"user": user, "database": database, "application_name": application_name,
                   "client_encoding": "UTF8", "DateStyle": "ISO"}
        startup.update(options or {})
        body = struct.pack("!i", PROTOCOL_3) + b"".join(
            k.encode() + b"\0" + str(v).encode() + b"\0" for k, v in startup.items()) + b"\0"
        self.sock.sendall(struct.pack("!i", len(body) + 4) + body)
        self._authenticate()

    @classmethod
    def from_jdbc(cls, url: str, props: Optional[Dict[str, Any]] = None) -> "PgConnection":
        c = parse_jdbc_url(url, props)
        mode = str(c.get("sslmode") or "").lower()
        if not mode:
            mode = "verify-full" if str(c.get("ssl", "false")).lower() == "true" else "disable"
        if mode not in ("disable", "allow", "prefer", "require", "verify-ca", "verify-full"):
            raise ValueError(f"unsupported sslmode {mode}")
        if mode in ("allow", "prefer"):
            mode = "disable"
        opts = {}
        if c.get("currentSchema"):
            opts["search_path"] = str(c["currentSchema"])
        return cls(c["host"], int(c["port"]), str(c.get("user") or os.environ.get("USER", "postgres")),
                   None if c.get("password") is None else str(c["password"]), c["database"],
                   timeout=float(c.get("connectTimeout") or 30), ssl_mode=mode, ssl_root_cert=c.get("sslrootcert"),
                   application_name=str(c.get("ApplicationName") or "langstream"), options=opts)

    def _start_tls(self, mode: str, root_cert: Optional[str]) -> None:
        self.sock.sendall(struct.pack("!ii", 8, SSL_REQUEST))
        ans = self.sock.recv(1)
        if ans != b"S":
            raise PgError({"M": "server does not support TLS but sslmode requires it"})
        ctx = ssl.create_default_context(cafile=root_cert) if root_cert else ssl.create_default_context()
        # verify-ca: the chain, not the host name; require / verify-full: both
        ctx.check_hostname = mode != "verify-ca"
        self.sock = ctx.wrap_socket(self.sock, server_hostname=self.host)

    # -- framing
    def _send(self, msgs: List[bytes]) -> None:
        self.sock.sendall(b"".join(msgs))

    @staticmethod
    def _msg(t: bytes, body: bytes) -> bytes:
        return t + struct.pack("!i", len(body) + 4) + body

    def _recv(self) -> Tuple[bytes, bytes]:
        while True:
            if len(self._buf) >= 5:
                ln = struct.unpack_from("!i", self._buf, 1)[0]
                if len(self._buf) >= ln + 1:
                    t = bytes(self._buf[:1])
                    body = bytes(self._buf[5:ln + 1])
                    del self._buf[:ln + 1]
                    if t == b"N":                       # NoticeResponse: ignore
                        continue
                    if t == b"S":                       # ParameterStatus (any time)
                        k, v = body[:-1].split(b"\0")[:2]
                        self.params[k.decode()] = v.decode()
                        continue
                    if t == b"A":                       # NotificationResponse
                        continue
                    return t, body
            chunk = self.sock.recv(65536)
            if not chunk:
                raise ConnectionError("PostgreSQL server closed the connection")
            self._buf += chunk

    @staticmethod
    def _error_fields(body: bytes) -> Dict[str, str]:
        out: Dict[str, str] = {}
        i = 0
        while i < len(body) and body[i] != 0:
            k = chr(body[i])
            j = body.index(b"\0", i + 1)
            out[k] = body[i + 1:j].decode("utf-8", "replace")
            i = j + 1
        return out

    def _authenticate(self) -> None:
        scram: Optional[Tuple[str, str]] = None
        server_sig = b""
        while True:
            t, body = self._recv()
            if t == b"E":
                raise PgError(self._error_fields(body))
            if t == b"R":
                code = struct.unpack_from("!i", body)[0]
                if code == 0:
                    continue
                if self.password is None:
                    raise PgError({"M": "the server requested a password but none was configured"})
                if code == 3:
                    self._send([self._msg(b"p", self.password.encode() + b"\0")])
                elif code == 5:
                    salt = body[4:8]
                    inner = hashlib.md5((self.password + self.user).encode()).hexdigest()
                    outer = hashlib.md5(inner.encode() + salt).hexdigest()
                    self._send([self._msg(b"p", b"md5" + outer.encode() + b"\0")])
                elif code == 10:
                    mechs = [m.decode() for m in body[4:].split(b"\0") if m]
                    if "SCRAM-SHA-256" not in mechs:
                        raise PgError({"M": f"no supported SASL mechanism in {mechs}"})
                    nonce = base64.b64encode(os.urandom(18)).decode()
                    first, bare = _scram_client_first(nonce)
                    scram = (bare, nonce)
                    fb = first.encode()
                    self._send([self._msg(b"p", b"SCRAM-SHA-256\0" + struct.pack("!i", len(fb)) + fb)])
                elif code == 11:
                    server_first = body[4:].decode()
                    if scram is None or not dict(kv.split("=", 1) for kv in server_first.split(","))["r"] \
                            .startswith(scram[1]):
                        raise PgError({"M": "SCRAM: server nonce does not extend the client nonce"})
                    final, server_sig = scram_client_final(self.password, scram[0], server_first)
                    self._send([self._msg(b"p", final.encode())])
                elif code == 12:
                    attrs = dict(kv.split("=", 1) for kv in body[4:].decode().split(","))
                    if not hmac.compare_digest(base64.b64decode(attrs.get("v", "")), server_sig):
                        raise PgError({"M": "SCRAM: the server's signature does not verify"})
                else:
                    raise PgError({"M": f"unsupported authentication method {code}"})
            elif t == b"K":
                self.backend_key = struct.unpack("!ii", body[:8])
            elif t == b"Z":
                return
            # anything else during startup is ignored

    def _drain_error(self, first: Optional[Dict[str, str]]) -> None:
        """After an ErrorResponse the backend skips to the Sync: read to ReadyForQuery."""
        while True:
            t, body = self._recv()
            if t == b"Z":
                break
        if first is not None:
            raise PgError(first)

    # -- prepared statements
    def _prepare(self, sql: str) -> _Stmt:
        st = self._stmts.get(sql)
        if st is not None:
            return st
        self._nstmt += 1
        name = f"ls_{self._nstmt}"
        self._send([self._msg(b"P", name.encode() + b"\0" + sql.encode() + b"\0" + struct.pack("!h", 0)),
                    self._msg(b"D", b"S" + name.encode() + b"\0"),
                    self._msg(b"S", b"")])
        oids: List[int] = []
        cols: Optional[List[Tuple[str, int]]] = None
        err = None
        while True:
            t, body = self._recv()
            if t == b"E":
                err = self._error_fields(body)
            elif t == b"t":
                n = struct.unpack_from("!h", body)[0]
                oids = list(struct.unpack_from(f"!{n}i", body, 2))
            elif t == b"T":
                cols = self._row_description(body)
            elif t == b"n":
                cols = None
            elif t == b"Z":
                break
        if err is not None:
            raise PgError(err)
        st = _Stmt(name, oids, cols)
        if len(self._stmts) >= 256:                 # bounded cache: close the oldest
            old_sql, old = next(iter(self._stmts.items()))
            del self._stmts[old_sql]
            self._send([self._msg(b"C", b"S" + old.name.encode() + b"\0"), self._msg(b"S", b"")])
            while self._recv()[0] != b"Z":
                pass
        self._stmts[sql] = st
        return st

    @staticmethod
    def _row_description(body: bytes) -> List[Tuple[str, int]]:
        n = struct.unpack_from("!h", body)[0]
        cols, i = [], 2
        for _ in range(n):
            j = body.index(b"\0", i)
            name = body[i:j].decode()
            i = j + 1
            _tbl, _att, oid, _len, _mod, _fmt = struct.unpack_from("!ihihih", body, i)
            i += 18
            cols.append((name, oid))
        return cols

    def execute(self, sql: str, params: Sequence[Any] = ()) -> Tuple[List[Dict[str, Any]], int, str]:
        """Run one PostgreSQL statement (``$n`` placeholders); returns (rows, rowcount, tag)."""
        with self.lock:
            st = self._prepare(sql)
            if len(params) != len(st.param_oids):
                raise PgError({"M": f"statement has {len(st.param_oids)} parameters, {len(params)} given"})
            vals = [encode_param(v, o) for v, o in zip(params, st.param_oids)]
            bind = bytearray(b"\0" + st.name.encode() + b"\0" + struct.pack("!hh", 0, len(vals)))
            for v in vals:
                if v is None:
                    bind += struct.pack("!i", -1)
                else:
                    bind += struct.pack("!i", len(v)) + v
            bind += struct.pack("!h", 0)
            self._send([self._msg(b"B", bytes(bind)), self._msg(b"E", b"\0" + struct.pack("!i", 0)),
                        self._msg(b"S", b"")])
            rows: List[Dict[str, Any]] = []
            count, tag, err = 0, "", None
            cols = st.columns or []
            while True:
                t, body = self._recv()
                if t == b"D":
                    n = struct.unpack_from("!h", body)[0]
                    i, row = 2, {}
                    for c in range(n):
                        ln = struct.unpack_from("!i", body, i)[0]
                        i += 4
                        raw = None
                        if ln >= 0:
                            raw = body[i:i + ln].decode("utf-8")
                            i += ln
                        name, oid = cols[c] if c < len(cols) else (f"column{c + 1}", 25)
                        row[name] = decode_value(raw, oid)
                    rows.append(row)
                elif t == b"C":
                    tag = body[:-1].decode()
                    parts = tag.split()
                    count = int(parts[-1]) if parts and parts[-1].isdigit() else 0
                elif t == b"E":
                    err = self._error_fields(body)
                elif t == b"Z":
                    break
            if err is not None:
                if err.get("C") in ("26000", "0A000"):    # statement gone (e.g. DDL changed it)
                    self._stmts.pop(sql, None)
                raise PgError(err)
            return rows, count, tag

    def simple_query(self, sql: str) -> List[Tuple[List[Dict[str, Any]], str]]:
        """The simple-query protocol (several ';'-separated statements, no parameters)."""
        with self.lock:
            self._send([self._msg(b"Q", sql.encode() + b"\0")])
            out: List[Tuple[List[Dict[str, Any]], str]] = []
            cols: List[Tuple[str, int]] = []
            rows: List[Dict[str, Any]] = []
            err = None
            while True:
                t, body = self._recv()
                if t == b"T":
                    cols, rows = self._row_description(body), []
                elif t == b"D":
                    n = struct.unpack_from("!h", body)[0]
                    i, row = 2, {}
                    for c in range(n):
                        ln = struct.unpack_from("!i", body, i)[0]
                        i += 4
                        raw = body[i:i + ln].decode() if ln >= 0 else None
                        i += max(ln, 0)
                        row[cols[c][0]] = decode_value(raw, cols[c][1])
                    rows.append(row)
                elif t == b"C":
                    out.append((rows, body[:-1].decode()))
                    rows = []
                elif t == b"E":
                    err = self._error_fields(body)
                elif t == b"Z":
                    break
            if err is not None:
                raise PgError(err)
            # DDL may invalidate cached plans: drop them
            self._stmts.clear()
            return out

    def close(self) -> None:
        try:
            self._send([self._msg(b"X", b"")])
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass


# ---------------------------------------------------------------- datasource
class PostgresDataSource:
    """``query`` / ``vector-db-sink`` / ``jdbc-table`` over a PostgreSQL server."""

    def __init__(self, cfg: Dict[str, Any]):
        self.url = str(cfg.get("url"))
        props = {k: v for k, v in cfg.items() if k not in ("url", "service", "driverClass")}
        self.props = props
        self._conn: Optional[PgConnection] = None
        self._lock = threading.Lock()
        self.conn()      # connect at init: a wrong URL / credentials fail the agent's start

    def conn(self) -> PgConnection:
        with self._lock:
            if self._conn is None:
                self._conn = PgConnection.from_jdbc(self.url, self.props)
            return self._conn

    def _run(self, sql: str, params: Sequence[Any]):
        try:
            return self.conn().execute(sql, params)
        except (ConnectionError, OSError):
            with self._lock:                            # one reconnect on a dropped socket
                self._conn = None
            return self.conn().execute(sql, params)

    def fetch_data(self, query: str, params: List[Any]) -> List[Dict[str, Any]]:
        sql, _ = jdbc_to_pg_sql(query)
        return self._run(sql, params)[0]

    def execute_statement(self, query: str, generated_keys: Sequence[str], params: List[Any]) -> Dict[str, Any]:
        sql, _ = jdbc_to_pg_sql(query)
        if generated_keys:
            # PgJDBC's prepareStatement(sql, String[] keys): RETURNING the key columns
            sql = sql.rstrip().rstrip(";") + " RETURNING " + ", ".join(f'"{k}"' for k in generated_keys)
        rows, count, _ = self._run(sql, params)
        out: Dict[str, Any] = {"count": count}
        if generated_keys:
            keys: Dict[str, Any] = {}
            for r in rows:
                keys.update(r)
            out["generatedKeys"] = keys
        return out

    def script(self, statements: Sequence[str]) -> None:
        for s in statements:
            self.conn().simple_query(s)

    def table_exists(self, table: str) -> bool:
        # DatabaseMetaData.getTables(name), then upper / lower case (JdbcAssetsManagerProvider)
        rows = self.fetch_data("SELECT table_name FROM information_schema.tables WHERE table_name = ? "
                               "OR table_name = ? OR table_name = ?", [table, table.upper(), table.lower()])
        return any(str(r.get("table_name", "")).lower() == table.lower() for r in rows)

    def close(self) -> None:
        with self._lock:
            if self._conn is not None:
                self._conn.close()
                self._conn = None
