"""Kafka wire protocol (the subset LangStream uses), encode + decode for both sides.

Non-flexible (pre-KIP-482) API versions only, so every message is fixed-layout:

    ApiVersions v0, Metadata v1, Produce v3, Fetch v4, ListOffsets v1,
    FindCoordinator v0, JoinGroup v1, SyncGroup v0, Heartbeat v0, LeaveGroup v0,
    OffsetCommit v2, OffsetFetch v1, CreateTopics v0, DeleteTopics v0

Records use the v2 RecordBatch format (magic 2, CRC-32C, varint records).  Schemas are
declared once as nested tuples and interpreted by one generic encoder/decoder, so
request and response layouts are data, not code.  The default partitioner is Kafka's
murmur2 (``Utils.toPositive(murmur2(key)) % partitions``), so keyed records land on the
same partitions as with the Java client.
"""
from __future__ import annotations

import struct
from typing import Any, Dict, List, Optional, Tuple

# ---------------------------------------------------------------- api keys
PRODUCE, FETCH, LIST_OFFSETS, METADATA = 0, 1, 2, 3
OFFSET_COMMIT, OFFSET_FETCH, FIND_COORDINATOR = 8, 9, 10
JOIN_GROUP, HEARTBEAT, LEAVE_GROUP, SYNC_GROUP = 11, 12, 13, 14
API_VERSIONS, CREATE_TOPICS, DELETE_TOPICS = 18, 19, 20
SASL_HANDSHAKE, SASL_AUTHENTICATE = 17, 36
DESCRIBE_CONFIGS = 32
RESOURCE_TOPIC = 2

VERSIONS = {PRODUCE: 3, FETCH: 4, LIST_OFFSETS: 1, METADATA: 1, OFFSET_COMMIT: 2, OFFSET_FETCH: 1,
            FIND_COORDINATOR: 0, JOIN_GROUP: 1, HEARTBEAT: 0, LEAVE_GROUP: 0, SYNC_GROUP: 0, API_VERSIONS: 0,
            CREATE_TOPICS: 0, DELETE_TOPICS: 0, SASL_HANDSHAKE: 1, SASL_AUTHENTICATE: 0, DESCRIBE_CONFIGS: 0}

# error codes
NONE, OFFSET_OUT_OF_RANGE, UNKNOWN_TOPIC_OR_PARTITION = 0, 1, 3
COORDINATOR_NOT_AVAILABLE, NOT_COORDINATOR = 15, 16
ILLEGAL_GENERATION, UNKNOWN_MEMBER_ID, REBALANCE_IN_PROGRESS = 22, 25, 27
TOPIC_ALREADY_EXISTS, UNSUPPORTED_VERSION = 36, 35
UNSUPPORTED_SASL_MECHANISM, ILLEGAL_SASL_STATE, SASL_AUTHENTICATION_FAILED = 33, 34, 58

# ---------------------------------------------------------------- schemas
# a schema is a list of (name, type); type is a primitive name, ("array", schema|primitive)
I8, I16, I32, I64, STR, NSTR, BYTES, NBYTES, BOOL = "i8", "i16", "i32", "i64", "str", "nstr", "bytes", "nbytes", "bool"


def A(t):
    return ("array", t)


REQ = {
    API_VERSIONS: [],
    SASL_HANDSHAKE: [("mechanism", STR)],
    SASL_AUTHENTICATE: [("auth_bytes", BYTES)],
    METADATA: [("topics", A(STR))],  # null array = all topics
    PRODUCE: [("transactional_id", NSTR), ("acks", I16), ("timeout", I32),
              ("topics", A([("name", STR), ("partitions", A([("partition", I32), ("records", NBYTES)]))]))],
    FETCH: [("replica_id", I32), ("max_wait", I32), ("min_bytes", I32), ("max_bytes", I32), ("isolation", I8),
            ("topics", A([("name", STR), ("partitions", A([("partition", I32), ("offset", I64),
                                                           ("max_bytes", I32)]))]))],
    LIST_OFFSETS: [("replica_id", I32),
                   ("topics", A([("name", STR), ("partitions", A([("partition", I32), ("timestamp", I64)]))]))],
    FIND_COORDINATOR: [("key", STR)],
    JOIN_GROUP: [("group_id", STR), ("session_timeout", I32), ("rebalance_timeout", I32), ("member_id", STR),
                 ("protocol_type", STR), ("protocols", A([("name", STR), ("metadata", BYTES)]))],
    SYNC_GROUP: [("group_id", STR), ("generation", I32), ("member_id", STR),
                 ("assignments", A([("member_id", STR), ("assignment", BYTES)]))],
    HEARTBEAT: [("group_id", STR), ("generation", I32), ("member_id", STR)],
    LEAVE_GROUP: [("group_id", STR), ("member_id", STR)],
    OFFSET_COMMIT: [("group_id", STR), ("generation", I32), ("member_id", STR), ("retention", I64),
                    ("topics", A([("name", STR), ("partitions", A([("partition", I32), ("offset", I64),
                                                                   ("metadata", NSTR)]))]))],
    OFFSET_FETCH: [("group_id", STR), ("topics", A([("name", STR), ("partitions", A(I32))]))],
    CREATE_TOPICS: [("topics", A([("name", STR), ("num_partitions", I32), ("replication_factor", I16),
                                  ("assignments", A([("partition", I32), ("brokers", A(I32))])),
                                  ("configs", A([("name", STR), ("value", NSTR)]))])), ("timeout", I32)],
    DELETE_TOPICS: [("topics", A(STR)), ("timeout", I32)],
    DESCRIBE_CONFIGS: [("resources", A([("type", I8), ("name", STR), ("config_names", A(STR))]))],
}

RESP = {
    API_VERSIONS: [("error", I16), ("apis", A([("key", I16), ("min", I16), ("max", I16)]))],
    SASL_HANDSHAKE: [("error", I16), ("mechanisms", A(STR))],
    SASL_AUTHENTICATE: [("error", I16), ("error_message", NSTR), ("auth_bytes", BYTES)],
    METADATA: [("brokers", A([("node_id", I32), ("host", STR), ("port", I32), ("rack", NSTR)])),
               ("controller_id", I32),
               ("topics", A([("error", I16), ("name", STR), ("internal", BOOL),
                             ("partitions", A([("error", I16), ("partition", I32), ("leader", I32),
                                               ("replicas", A(I32)), ("isr", A(I32))]))]))],
    PRODUCE: [("topics", A([("name", STR), ("partitions", A([("partition", I32), ("error", I16),
                                                             ("base_offset", I64), ("log_append_time", I64)]))])),
              ("throttle", I32)],
    FETCH: [("throttle", I32),
            ("topics", A([("name", STR), ("partitions", A([("partition", I32), ("error", I16), ("hw", I64),
                                                           ("lso", I64),
                                                           ("aborted", A([("pid", I64), ("first", I64)])),
                                                           ("records", NBYTES)]))]))],
    LIST_OFFSETS: [("topics", A([("name", STR), ("partitions", A([("partition", I32), ("error", I16),
                                                                  ("timestamp", I64), ("offset", I64)]))]))],
    FIND_COORDINATOR: [("error", I16), ("node_id", I32), ("host", STR), ("port", I32)],
    JOIN_GROUP: [("error", I16), ("generation", I32), ("protocol", STR), ("leader", STR), ("member_id", STR),
                 ("members", A([("member_id", STR), ("metadata", BYTES)]))],
    SYNC_GROUP: [("error", I16), ("assignment", BYTES)],
    HEARTBEAT: [("error", I16)],
    LEAVE_GROUP: [("error", I16)],
    OFFSET_COMMIT: [("topics", A([("name", STR), ("partitions", A([("partition", I32), ("error", I16)]))]))],
    OFFSET_FETCH: [("topics", A([("name", STR), ("partitions", A([("partition", I32), ("offset", I64),
                                                                  ("metadata", NSTR), ("error", I16)]))]))],
    CREATE_TOPICS: [("topics", A([("name", STR), ("error", I16)]))],
    DELETE_TOPICS: [("topics", A([("name", STR), ("error", I16)]))],
    DESCRIBE_CONFIGS: [("throttle", I32),
                       ("resources", A([("error", I16), ("error_message", NSTR), ("type", I8), ("name", STR),
                                        ("configs", A([("name", STR), ("value", NSTR), ("read_only", BOOL),
                                                       ("is_default", BOOL), ("sensitive", BOOL)]))]))],
}

# embedded consumer-protocol blobs (JoinGroup metadata / SyncGroup assignment)
SUBSCRIPTION = [("version", I16), ("topics", A(STR)), ("user_data", NBYTES)]
ASSIGNMENT = [("version", I16), ("partitions", A([("topic", STR), ("partitions", A(I32))])), ("user_data", NBYTES)]

_FMT = {I8: ">b", I16: ">h", I32: ">i", I64: ">q"}


class Writer:
    def __init__(self):
        self.parts: List[bytes] = []

    def prim(self, t, v):
        if t in _FMT:
            self.parts.append(struct.pack(_FMT[t], v))
        elif t == BOOL:
            self.parts.append(b"\x01" if v else b"\x00")
        elif t in (STR, NSTR):
            if v is None:
                self.parts.append(struct.pack(">h", -1))
            else:
                b = v.encode()
                self.parts.append(struct.pack(">h", len(b)) + b)
        elif t in (BYTES, NBYTES):
            if v is None:
                self.parts.append(struct.pack(">i", -1))
            else:
                self.parts.append(struct.pack(">i", len(v)) + bytes(v))
        else:
            raise ValueError(t)

    def write(self, schema, obj):
        if isinstance(schema, str):
            self.prim(schema, obj)
        elif isinstance(schema, tuple):  # array
            if obj is None:
                self.parts.append(struct.pack(">i", -1))
                return
            self.parts.append(struct.pack(">i", len(obj)))
            for it in obj:
                self.write(schema[1], it)
        else:
            for name, t in schema:
                self.write(t, obj.get(name) if isinstance(obj, dict) else obj[name])

    def bytes(self) -> bytes:
        return b"".join(self.parts)


class Reader:
    def __init__(self, b: bytes, pos: int = 0):
        self.b = memoryview(b)
        self.pos = pos

    def prim(self, t):
        if t in _FMT:
            f = _FMT[t]
            n = struct.calcsize(f)
            v = struct.unpack_from(f, self.b, self.pos)[0]
            self.pos += n
            return v
        if t == BOOL:
            v = self.b[self.pos] != 0
            self.pos += 1
            return v
        if t in (STR, NSTR):
            n = struct.unpack_from(">h", self.b, self.pos)[0]
            self.pos += 2
            if n < 0:
                return None
            v = bytes(self.b[self.pos: self.pos + n]).decode()
            self.pos += n
            return v
        if t in (BYTES, NBYTES):
            n = struct.unpack_from(">i", self.b, self.pos)[0]
            self.pos += 4
            if n < 0:
                return None
            v = bytes(self.b[self.pos: self.pos + n])
            self.pos += n
            return v
        raise ValueError(t)

    def read(self, schema):
        if isinstance(schema, str):
            return self.prim(schema)
        if isinstance(schema, tuple):
            n = struct.unpack_from(">i", self.b, self.pos)[0]
            self.pos += 4
            if n < 0:
                return None
            return [self.read(schema[1]) for _ in range(n)]
        return {name: self.read(t) for name, t in schema}


def encode(schema, obj) -> bytes:
    w = Writer()
    w.write(schema, obj)
    return w.bytes()


def decode(schema, b: bytes) -> Any:
    return Reader(b).read(schema)


def request_frame(api_key: int, correlation_id: int, client_id: str, body: Dict[str, Any]) -> bytes:
    payload = struct.pack(">hhi", api_key, VERSIONS[api_key], correlation_id) + encode(NSTR, client_id) + \
        encode(REQ[api_key], body)
    return struct.pack(">i", len(payload)) + payload


def response_frame(correlation_id: int, api_key: int, body: Dict[str, Any]) -> bytes:
    payload = struct.pack(">i", correlation_id) + encode(RESP[api_key], body)
    return struct.pack(">i", len(payload)) + payload


def parse_request(payload: bytes):
    api_key, version, corr = struct.unpack_from(">hhi", payload, 0)
    r = Reader(payload, 8)
    client_id = r.prim(NSTR)
    body = r.read(REQ[api_key]) if api_key in REQ and version == VERSIONS.get(api_key) else None
    return api_key, version, corr, client_id, body


# ---------------------------------------------------------------- varints / crc32c / murmur2
def zigzag_varint(v: int) -> bytes:
    z = (v << 1) ^ (v >> 63)
    z &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = z & 0x7F
        z >>= 7
        if z:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def read_varint(b, pos: int) -> Tuple[int, int]:
    shift = z = 0
    while True:
        c = b[pos]
        pos += 1
        z |= (c & 0x7F) << shift
        if not c & 0x80:
            break
        shift += 7
    return (z >> 1) ^ -(z & 1), pos


def _crc32c_table():
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        t.append(c)
    return t


_CRC = _crc32c_table()


def _crc32c_py(data: bytes) -> int:
    c = 0xFFFFFFFF
    t = _CRC
    for x in data:
        c = t[(c ^ x) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _murmur2_py(data: bytes) -> int:
    length = len(data)
    seed, m, r = 0x9747B28C, 0x5BD1E995, 24
    h = (seed ^ length) & 0xFFFFFFFF
    n4 = length // 4
    for i in range(n4):
        k = int.from_bytes(data[i * 4: i * 4 + 4], "little")
        k = (k * m) & 0xFFFFFFFF
        k ^= k >> r
        k = (k * m) & 0xFFFFFFFF
        h = (h * m) & 0xFFFFFFFF
        h ^= k
    rem = length & 3
    if rem == 3:
        h ^= data[(length & ~3) + 2] << 16
    if rem >= 2:
        h ^= data[(length & ~3) + 1] << 8
    if rem >= 1:
        h ^= data[length & ~3]
        h = (h * m) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return h - (1 << 32) if h >= 1 << 31 else h


def _native():
    try:
        from ...native import lib
        m = lib()
        return m if hasattr(m, "crc32c") else None
    except Exception:  # noqa: BLE001  (no toolchain: the Python loops below)
        return None


_NATIVE = _native()
# record-batch checksums and the partitioner hash run per batch / per keyed record on
# every produce and fetch: native (SSE4.2 crc32) when the host runtime is built
crc32c = _NATIVE.crc32c if _NATIVE is not None else _crc32c_py
murmur2 = _NATIVE.murmur2 if _NATIVE is not None else _murmur2_py
# records sections of every produced / fetched batch (native/kafka_records.cpp)
_ENC = getattr(_NATIVE, "kafka_encode_records", None)
_DEC = getattr(_NATIVE, "kafka_decode_records", None)


def partition_for_key(key: bytes, num_partitions: int) -> int:
    return (murmur2(key) & 0x7FFFFFFF) % num_partitions


# ---------------------------------------------------------------- record batches (v2)
def encode_batch(base_offset: int, records: List[Tuple[Optional[bytes], Optional[bytes], List[Tuple[str, bytes]],
                                                         int]], codec: int = 0) -> bytes:
    """records: (key, value, headers, timestamp_ms); codec: attributes compression bits
    (topics/kafka/codecs.py) applied to the records section."""
    first_ts = records[0][3] if records else 0
    max_ts = max((r[3] for r in records), default=0)
    if _ENC is not None:
        body = _ENC(records, first_ts)
    else:
        body = _encode_records_py(records, first_ts)
    if codec:
        from . import codecs
        body = codecs.compress(codec, bytes(body))
    tail = struct.pack(">hiqqqhii", codec & 0x07, len(records) - 1, first_ts, max_ts, -1, -1, -1,
                       len(records)) + bytes(body)
    crc = crc32c(tail)
    head = struct.pack(">ib", -1, 2) + struct.pack(">I", crc)  # partitionLeaderEpoch, magic, crc
    batch_len = len(head) + len(tail)
    return struct.pack(">qi", base_offset, batch_len) + head + tail


def _encode_records_py(records, first_ts: int) -> bytearray:
    body = bytearray()
    for i, (k, v, hs, ts) in enumerate(records):
        rec = bytearray(b"\x00")
        rec += zigzag_varint(ts - first_ts)
        rec += zigzag_varint(i)
        for x in (k, v):
            if x is None:
                rec += zigzag_varint(-1)
            else:
                rec += zigzag_varint(len(x)) + x
        rec += zigzag_varint(len(hs))
        for hk, hv in hs:
            kb = hk.encode()
            rec += zigzag_varint(len(kb)) + kb
            if hv is None:
                rec += zigzag_varint(-1)
            else:
                rec += zigzag_varint(len(hv)) + hv
        body += zigzag_varint(len(rec)) + rec
    return body


def decode_batches(data: Optional[bytes], verify_crc: bool = False):
    """Yields (offset, timestamp, key, value, headers[(k, v)]) from concatenated batches;
    a truncated trailing batch (partial fetch) is ignored."""
    if not data:
        return
    pos, n = 0, len(data)
    while pos + 12 <= n:
        base, blen = struct.unpack_from(">qi", data, pos)
        end = pos + 12 + blen
        if end > n:
            return
        magic = data[pos + 16]
        if magic != 2:
            raise ValueError(f"unsupported record batch magic {magic}")
        crc = struct.unpack_from(">I", data, pos + 17)[0]
        if verify_crc and crc32c(data[pos + 21: end]) != crc:
            raise ValueError("record batch CRC mismatch")
        attrs, _lod, first_ts, _max_ts, _pid, _pe, _bs, count = struct.unpack_from(">hiqqqhii", data, pos + 21)
        p = pos + 21 + 2 + 4 + 8 + 8 + 8 + 2 + 4 + 4
        if attrs & 0x07:   # compressed records section: decode it, then parse the records from it
            from . import codecs
            rdata = codecs.decompress(attrs & 0x07, bytes(data[p:end]))
            yield from _records(rdata, 0, count, base, first_ts)
            pos = end
            continue
        yield from _records(data, p, count, base, first_ts)
        pos = end


def _records(data, p: int, count: int, base: int, first_ts: int):
    """Records of one (decompressed) batch starting at byte ``p``."""
    if _DEC is not None:
        return _DEC(data, p, count, base, first_ts)
    return _records_py(data, p, count, base, first_ts)


def _records_py(data, p: int, count: int, base: int, first_ts: int):
    for _ in range(count):
        _ln, p = read_varint(data, p)
        p += 1  # attributes
        tsd, p = read_varint(data, p)
        od, p = read_varint(data, p)
        kl, p = read_varint(data, p)
        key = None if kl < 0 else bytes(data[p: p + kl])
        p += max(kl, 0)
        vl, p = read_varint(data, p)
        val = None if vl < 0 else bytes(data[p: p + vl])
        p += max(vl, 0)
        nh, p = read_varint(data, p)
        hs = []
        for _h in range(nh):
            hkl, p = read_varint(data, p)
            hk = bytes(data[p: p + hkl]).decode()
            p += hkl
            hvl, p = read_varint(data, p)
            hv = None if hvl < 0 else bytes(data[p: p + hvl])
            p += max(hvl, 0)
            hs.append((hk, hv))
        yield base + od, first_ts + tsd, key, val, hs
