"""Cassandra / Astra DB over the CQL native protocol v4 (§2.2 B8).

The reference uses the DataStax Java driver (``AIA/.../datasource/CassandraDataSource.java``)
and the DataStax Kafka-Connect sink (``VEC/cassandra/CassandraWriter.java``).  This is a
small synchronous client speaking protocol v4 directly:
* STARTUP, SASL PLAIN authentication (username/password, or ``token`` as Astra's
  "token" user with the AstraCS token as password), optional TLS;
* PREPARE + EXECUTE with typed bind values (the prepared metadata says each column's
  type, so Python ints become int/bigint/smallint/... exactly as the column needs),
  QUERY for unprepared statements;
* RESULT decoding for the CQL types LangStream apps use: ascii/text/varchar, int,
  bigint, counter, smallint, tinyint, boolean, float, double, decimal, varint, blob,
  timestamp, date, time, uuid/timeuuid, inet, list/set/map/tuple/udt and the Cassandra 5
  ``VectorType(FloatType, n)`` custom type (decoded to a list of floats).
"""
from __future__ import annotations

import decimal
import ipaddress
import socket
import ssl
import struct
import threading
import uuid
from datetime import date, datetime, timezone
from typing import Any, Dict, List, Optional, Tuple

OP_ERROR, OP_STARTUP, OP_READY, OP_AUTHENTICATE, OP_OPTIONS, OP_SUPPORTED = 0x00, 0x01, 0x02, 0x03, 0x05, 0x06
OP_QUERY, OP_RESULT, OP_PREPARE, OP_EXECUTE = 0x07, 0x08, 0x09, 0x0A
OP_AUTH_CHALLENGE, OP_AUTH_RESPONSE, OP_AUTH_SUCCESS = 0x0E, 0x0F, 0x10

CONSISTENCY = {"ANY": 0, "ONE": 1, "TWO": 2, "THREE": 3, "QUORUM": 4, "ALL": 5, "LOCAL_QUORUM": 6,
               "EACH_QUORUM": 7, "SERIAL": 8, "LOCAL_SERIAL": 9, "LOCAL_ONE": 10}

T_CUSTOM, T_ASCII, T_BIGINT, T_BLOB, T_BOOLEAN, T_COUNTER, T_DECIMAL, T_DOUBLE, T_FLOAT, T_INT = range(10)
T_TIMESTAMP, T_UUID, T_VARCHAR, T_VARINT, T_TIMEUUID, T_INET, T_DATE, T_TIME, T_SMALLINT, T_TINYINT = \
    0x0B, 0x0C, 0x0D, 0x0E, 0x0F, 0x10, 0x11, 0x12, 0x13, 0x14
T_TEXT = 0x0A
T_LIST, T_MAP, T_SET, T_UDT, T_TUPLE = 0x20, 0x21, 0x22, 0x30, 0x31

_EPOCH_DATE = 1 << 31


class CqlError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"CQL error 0x{code:04x}: {message}")
        self.code = code


# ------------------------------------------------------------------ primitive codecs
def _string(s: str) -> bytes:
    b = s.encode()
    return struct.pack(">H", len(b)) + b


def _long_string(s: str) -> bytes:
    b = s.encode()
    return struct.pack(">i", len(b)) + b


def _string_map(m: Dict[str, str]) -> bytes:
    return struct.pack(">H", len(m)) + b"".join(_string(k) + _string(v) for k, v in m.items())


def _bytes(b: Optional[bytes]) -> bytes:
    return struct.pack(">i", -1) if b is None else struct.pack(">i", len(b)) + b


class _Reader:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def take(self, n: int) -> bytes:
        b = self.d[self.p:self.p + n]
        self.p += n
        return b

    def byte(self) -> int:
        return self.take(1)[0]

    def short(self) -> int:
        return struct.unpack(">H", self.take(2))[0]

    def int(self) -> int:
        return struct.unpack(">i", self.take(4))[0]

    def string(self) -> str:
        return self.take(self.short()).decode()

    def long_string(self) -> str:
        return self.take(self.int()).decode()

    def bytes(self) -> Optional[bytes]:
        n = self.int()
        return None if n < 0 else self.take(n)

    def short_bytes(self) -> bytes:
        return self.take(self.short())

    def option(self) -> Tuple:
        t = self.short()
        if t == T_CUSTOM:
            return (t, self.string())
        if t in (T_LIST, T_SET):
            return (t, self.option())
        if t == T_MAP:
            return (t, self.option(), self.option())
        if t == T_UDT:
            ks, name = self.string(), self.string()
            fields = [(self.string(), self.option()) for _ in range(self.short())]
            return (t, ks, name, fields)
        if t == T_TUPLE:
            return (t, [self.option() for _ in range(self.short())])
        return (t,)


def _vector_dim(custom: str) -> Optional[int]:
    if "VectorType" not in custom:
        return None
    try:
        return int(custom.rsplit(",", 1)[1].strip(" )"))
    except (IndexError, ValueError):
        return None


def decode_value(typ: Tuple, b: Optional[bytes]) -> Any:
    if b is None:
        return None
    t = typ[0]
    if t in (T_ASCII, T_VARCHAR, T_TEXT):
        return b.decode()
    if t in (T_BIGINT, T_COUNTER):
        return struct.unpack(">q", b)[0]
    if t == T_INT:
        return struct.unpack(">i", b)[0]
    if t == T_SMALLINT:
        return struct.unpack(">h", b)[0]
    if t == T_TINYINT:
        return struct.unpack(">b", b)[0]
    if t == T_BOOLEAN:
        return b != b"\x00"
    if t == T_FLOAT:
        return struct.unpack(">f", b)[0]
    if t == T_DOUBLE:
        return struct.unpack(">d", b)[0]
    if t == T_VARINT:
        return int.from_bytes(b, "big", signed=True)
    if t == T_DECIMAL:
        scale = struct.unpack(">i", b[:4])[0]
        return decimal.Decimal(int.from_bytes(b[4:], "big", signed=True)).scaleb(-scale)
    if t == T_BLOB:
        return b
    if t == T_TIMESTAMP:
        return datetime.fromtimestamp(struct.unpack(">q", b)[0] / 1000, tz=timezone.utc)
    if t == T_DATE:
        return date.fromordinal(date(1970, 1, 1).toordinal() + struct.unpack(">I", b)[0] - _EPOCH_DATE)
    if t == T_TIME:
        return struct.unpack(">q", b)[0]
    if t in (T_UUID, T_TIMEUUID):
        return uuid.UUID(bytes=b)
    if t == T_INET:
        return str(ipaddress.ip_address(b))
    if t in (T_LIST, T_SET):
        r = _Reader(b)
        out = [decode_value(typ[1], r.bytes()) for _ in range(r.int())]
        return out
    if t == T_MAP:
        r = _Reader(b)
        return {decode_value(typ[1], r.bytes()): decode_value(typ[2], r.bytes()) for _ in range(r.int())}
    if t == T_TUPLE:
        r = _Reader(b)
        return [decode_value(ft, r.bytes()) for ft in typ[1]]
    if t == T_UDT:
        r = _Reader(b)
        out = {}
        for name, ft in typ[3]:
            if r.p >= len(b):
                break
            out[name] = decode_value(ft, r.bytes())
        return out
    if t == T_CUSTOM:
        dim = _vector_dim(typ[1])
        if dim is not None and len(b) == 4 * dim:
            return list(struct.unpack(f">{dim}f", b))
        return b
    return b


def encode_value(typ: Tuple, v: Any) -> Optional[bytes]:
    if v is None:
        return None
    t = typ[0]
    if t in (T_ASCII, T_VARCHAR, T_TEXT):
        return str(v).encode()
    if t in (T_BIGINT, T_COUNTER, T_TIME):
        return struct.pack(">q", int(v))
    if t == T_INT:
        return struct.pack(">i", int(v))
    if t == T_SMALLINT:
        return struct.pack(">h", int(v))
    if t == T_TINYINT:
        return struct.pack(">b", int(v))
    if t == T_BOOLEAN:
        return b"\x01" if (v if not isinstance(v, str) else v.lower() == "true") else b"\x00"
    if t == T_FLOAT:
        return struct.pack(">f", float(v))
    if t == T_DOUBLE:
        return struct.pack(">d", float(v))
    if t == T_VARINT:
        i = int(v)
        return i.to_bytes(max(1, (i.bit_length() + 8) // 8), "big", signed=True)
    if t == T_DECIMAL:
        d = decimal.Decimal(str(v))
        sign, digits, exp = d.as_tuple()
        unscaled = int("".join(map(str, digits)) or "0") * (-1 if sign else 1)
        return struct.pack(">i", -exp) + unscaled.to_bytes(max(1, (unscaled.bit_length() + 8) // 8), "big",
                                                            signed=True)
    if t == T_BLOB:
        return bytes(v) if not isinstance(v, str) else v.encode()
    if t == T_TIMESTAMP:
        ms = int(v.timestamp() * 1000) if isinstance(v, datetime) else int(v)
        return struct.pack(">q", ms)
    if t == T_DATE:
        d = v if isinstance(v, date) else date.fromisoformat(str(v))
        return struct.pack(">I", d.toordinal() - date(1970, 1, 1).toordinal() + _EPOCH_DATE)
    if t in (T_UUID, T_TIMEUUID):
        return (v if isinstance(v, uuid.UUID) else uuid.UUID(str(v))).bytes
    if t == T_INET:
        return ipaddress.ip_address(v).packed
    if t in (T_LIST, T_SET):
        items = list(v)
        return struct.pack(">i", len(items)) + b"".join(_bytes(encode_value(typ[1], x)) for x in items)
    if t == T_MAP:
        return struct.pack(">i", len(v)) + b"".join(_bytes(encode_value(typ[1], k)) + _bytes(encode_value(typ[2], x))
                                                   for k, x in v.items())
    if t == T_TUPLE:
        return b"".join(_bytes(encode_value(ft, x)) for ft, x in zip(typ[1], v))
    if t == T_UDT:
        return b"".join(_bytes(encode_value(ft, (v or {}).get(name))) for name, ft in typ[3])
    if t == T_CUSTOM:
        dim = _vector_dim(typ[1])
        if dim is not None:
            vals = [float(x) for x in v]
            if len(vals) != dim:
                raise ValueError(f"vector of {len(vals)} values for a {dim}-dimension column")
            return struct.pack(f">{dim}f", *vals)
    if isinstance(v, bytes):
        return v
    raise ValueError(f"cannot encode {v!r} as CQL type {typ}")


# ------------------------------------------------------------------ connection
class Prepared:
    def __init__(self, query_id: bytes, bind_types: List[Tuple], bind_names: List[str]):
        self.query_id, self.bind_types, self.bind_names = query_id, bind_types, bind_names


class CqlSession:
    def __init__(self, contact_points: List[str], port: int = 9042, username: Optional[str] = None,
                 password: Optional[str] = None, keyspace: Optional[str] = None, use_tls: bool = False,
                 consistency: str = "LOCAL_QUORUM", timeout: float = 30.0, ssl_context=None):
        last: Optional[Exception] = None
        for cp in contact_points:
            host, _, p = cp.partition(":")
            try:
                s = socket.create_connection((host, int(p or port)), timeout=timeout)
                if use_tls or ssl_context is not None:
                    s = (ssl_context or ssl.create_default_context()).wrap_socket(s, server_hostname=host)
                self.sock = s
                break
            except OSError as e:
                last = e
        else:
            raise ConnectionError(f"no Cassandra contact point reachable: {contact_points}: {last}")
        self.lock = threading.Lock()
        self.stream = 0
        self.consistency = CONSISTENCY.get(consistency.upper(), 6)
        self.prepared: Dict[str, Prepared] = {}
        op, body = self._request(OP_STARTUP, _string_map({"CQL_VERSION": "3.0.0"}))
        if op == OP_AUTHENTICATE:
            token = b"\x00" + (username or "").encode() + b"\x00" + (password or "").encode()
            op, body = self._request(OP_AUTH_RESPONSE, _bytes(token))
            if op != OP_AUTH_SUCCESS:
                raise CqlError(0x0100, "authentication failed")
        elif op != OP_READY:
            raise CqlError(0, f"unexpected startup response opcode {op}")
        if keyspace:
            self.execute(f'USE "{keyspace}"')

    def _recv_exact(self, n: int) -> bytes:
        buf = b""
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("CQL connection closed")
            buf += chunk
        return buf

    def _request(self, opcode: int, body: bytes) -> Tuple[int, bytes]:
        with self.lock:
            self.stream = (self.stream + 1) % 32768
            self.sock.sendall(struct.pack(">BBhBi", 0x04, 0, self.stream, opcode, len(body)) + body)
            while True:
                _ver, _flags, stream, op, n = struct.unpack(">BBhBi", self._recv_exact(9))
                payload = self._recv_exact(n)
                if stream == self.stream or stream < 0:
                    break
        if op == OP_ERROR:
            r = _Reader(payload)
            raise CqlError(r.int(), r.string())
        return op, payload

    def _params(self, values: bytes, n: int) -> bytes:
        flags = 0x01 if n else 0x00
        out = struct.pack(">HB", self.consistency, flags)
        if n:
            out += struct.pack(">H", n) + values
        return out

    def prepare(self, query: str) -> Prepared:
        p = self.prepared.get(query)
        if p is not None:
            return p
        op, body = self._request(OP_PREPARE, _long_string(query))
        r = _Reader(body)
        kind = r.int()
        if kind != 0x0004:
            raise CqlError(0, f"unexpected PREPARE result kind {kind}")
        qid = r.short_bytes()
        flags, ncols = r.int(), r.int()
        pk_count = r.int()
        for _ in range(pk_count):
            r.short()
        glob = bool(flags & 0x0001)
        if glob:
            r.string(), r.string()
        types, names = [], []
        for _ in range(ncols):
            if not glob:
                r.string(), r.string()
            names.append(r.string())
            types.append(r.option())
        p = Prepared(qid, types, names)
        self.prepared[query] = p
        return p

    def execute(self, query: str, params: Optional[List[Any]] = None) -> List[Dict[str, Any]]:
        params = list(params or [])
        if params or query.lstrip().upper().startswith(("SELECT", "INSERT", "UPDATE", "DELETE")):
            p = self.prepare(query)
            if len(params) != len(p.bind_types):
                raise ValueError(f"statement needs {len(p.bind_types)} parameters, got {len(params)}")
            vals = b"".join(_bytes(encode_value(t, v)) for t, v in zip(p.bind_types, params))
            op, body = self._request(OP_EXECUTE, struct.pack(">H", len(p.query_id)) + p.query_id +
                                     self._params(vals, len(params)))
        else:
            op, body = self._request(OP_QUERY, _long_string(query) + self._params(b"", 0))
        return self._result(body)

    @staticmethod
    def _result(body: bytes) -> List[Dict[str, Any]]:
        r = _Reader(body)
        kind = r.int()
        if kind != 0x0002:
            return []
        flags, ncols = r.int(), r.int()
        if flags & 0x0002:
            r.bytes()  # paging state
        glob = bool(flags & 0x0001)
        if glob:
            r.string(), r.string()
        cols = []
        if not flags & 0x0004:
            for _ in range(ncols):
                if not glob:
                    r.string(), r.string()
                cols.append((r.string(), r.option()))
        rows = []
        for _ in range(r.int()):
            rows.append({name: decode_value(t, r.bytes()) for name, t in cols})
        return rows

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


def session_from_datasource(cfg: Dict[str, Any]) -> CqlSession:
    """datasource keys as the reference: contact-points, port, username/password (or
    clientId/secret), token (Astra: user "token"), keyspace, loadBalancing-localDc, tls."""
    cps = cfg.get("contact-points") or cfg.get("contactPoints") or ["localhost"]
    if isinstance(cps, str):
        cps = [c.strip() for c in cps.split(",") if c.strip()]
    token = cfg.get("token") or ""
    user = cfg.get("username") or cfg.get("clientId") or ("token" if token else None)
    pwd = cfg.get("password") or cfg.get("secret") or token or None
    return CqlSession(cps, int(cfg.get("port") or 9042), user, pwd, cfg.get("keyspace") or None,
                      bool(cfg.get("tls") or cfg.get("secureBundle")), str(cfg.get("consistency", "LOCAL_QUORUM")))
