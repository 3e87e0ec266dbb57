"""Framed segment protocol shared by the ``pravega`` client and the in-tree standalone.

Frame layout (big-endian, like Pravega's WireCommands framing of an int32 type code
followed by an int32 payload length):

    int32 type | int32 length | int32 meta_len | meta (UTF-8 JSON) | blob

``meta`` carries the command fields and ``blob`` the event payloads (a list of
length-prefixed byte strings), so event bytes are never JSON-escaped.  Every request
carries ``rid`` (request id) and the reply echoes it with ``ok`` or ``error``.

Command set (the subset of Pravega's controller + segment-store surface that
LangStream's adapter uses, ``langstream-pravega-runtime/.../PravegaTopicConnectionsRuntimeProvider.java``
and ``PravegaClientUtils.java``): scopes, fixed-segment streams, seal/delete, keyed
appends routed over the key space, reader groups with online/offline readers and
segment rebalancing, and direct segment reads for position-addressed readers.
"""
from __future__ import annotations

import json
import socket
import struct
from typing import Any, Dict, List, Optional, Tuple

HELLO = -127
CREATE_SCOPE = 1
SCOPE_EXISTS = 2
CREATE_STREAM = 3
STREAM_INFO = 4
SEAL_STREAM = 5
DELETE_STREAM = 6
APPEND = 7
CREATE_READER_GROUP = 8
DELETE_READER_GROUP = 9
READER_ONLINE = 10
READER_OFFLINE = 11
READ_NEXT = 12
READ_SEGMENT = 13
REPLY = 100

PROTOCOL_VERSION = 1
_HDR = struct.Struct(">iii")
_LEN = struct.Struct(">i")
MAX_FRAME = 64 << 20


def pack_blob(items: List[bytes]) -> bytes:
    return b"".join(_LEN.pack(len(b)) + b for b in items)


def unpack_blob(blob: bytes) -> List[bytes]:
    out, i, n = [], 0, len(blob)
    while i < n:
        (ln,) = _LEN.unpack_from(blob, i)
        i += 4
        out.append(blob[i:i + ln])
        i += ln
    return out


def encode(kind: int, meta: Dict[str, Any], items: Optional[List[bytes]] = None) -> bytes:
    m = json.dumps(meta, separators=(",", ":")).encode()
    blob = pack_blob(items) if items else b""
    return _HDR.pack(kind, 4 + len(m) + len(blob), len(m)) + m + blob


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("pravega connection closed")
        buf += chunk
    return bytes(buf)


def read_frame(sock: socket.socket) -> Tuple[int, Dict[str, Any], List[bytes]]:
    kind, length, mlen = _HDR.unpack(_recv_exact(sock, 12))
    if length < 4 or length > MAX_FRAME or mlen > length - 4:
        raise ConnectionError(f"bad pravega frame (type {kind}, length {length})")
    body = _recv_exact(sock, length - 4)
    meta = json.loads(body[:mlen]) if mlen else {}
    return kind, meta, unpack_blob(body[mlen:])


def key_position(routing_key: str) -> float:
    """Routing key -> position in the [0, 1) key space (FNV-1a 64 + splitmix64 finaliser,
    top 53 bits)."""
    m = 0xFFFFFFFFFFFFFFFF
    h = 0xCBF29CE484222325
    for b in routing_key.encode():
        h = ((h ^ b) * 0x100000001B3) & m
    h = ((h ^ (h >> 30)) * 0xBF58476D1CE4E5B9) & m
    h = ((h ^ (h >> 27)) * 0x94D049BB133111EB) & m
    h ^= h >> 31
    return (h >> 11) / float(1 << 53)


def segment_for_key(routing_key: str, n_segments: int) -> int:
    """Fixed scaling policy: segment i owns key range [i/n, (i+1)/n)."""
    return min(n_segments - 1, int(key_position(routing_key) * n_segments))


def parse_uri(uri: str, default_port: int = 9090) -> Tuple[str, int]:
    u = uri.split("://", 1)[-1].rstrip("/")
    host, _, port = u.rpartition(":")
    if not host:
        return port or "localhost", default_port
    return host, int(port)
