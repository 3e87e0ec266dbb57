"""Minimal synchronous WebSocket client (RFC 6455) for thread-based runtime code.

Used by the Pulsar adapter (Pulsar's WebSocket producer/consumer/reader API) where the
agent runtime is thread-per-replica and an asyncio client would need its own loop.
Supports ws:// and wss://, text and binary frames, fragmentation, ping/pong and close.
"""
from __future__ import annotations

import base64
import hashlib
import os
import socket
import ssl
import struct
import threading
from typing import Dict, Optional, Tuple
from urllib.parse import urlsplit

_GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"

OP_CONT, OP_TEXT, OP_BIN, OP_CLOSE, OP_PING, OP_PONG = 0x0, 0x1, 0x2, 0x8, 0x9, 0xA


class WebSocketClosed(ConnectionError):
    pass


class WebSocket:
    def __init__(self, url: str, headers: Optional[Dict[str, str]] = None, timeout: float = 10.0):
        u = urlsplit(url)
        if u.scheme not in ("ws", "wss"):
            raise ValueError(f"not a websocket url: {url}")
        self.url = url
        port = u.port or (443 if u.scheme == "wss" else 80)
        sock = socket.create_connection((u.hostname, port), timeout=timeout)
        if u.scheme == "wss":
            sock = ssl.create_default_context().wrap_socket(sock, server_hostname=u.hostname)
        self.sock = sock
        self._send_lock = threading.Lock()
        self._buf = b""
        self.closed = False
        key = base64.b64encode(os.urandom(16)).decode()
        path = (u.path or "/") + (f"?{u.query}" if u.query else "")
        lines = [f"GET {path} HTTP/1.1", f"Host: {u.hostname}:{port}", "Upgrade: websocket",
                 "Connection: Upgrade", f"Sec-WebSocket-Key: {key}", "Sec-WebSocket-Version: 13"]
        for k, v in (headers or {}).items():
            lines.append(f"{k}: {v}")
        sock.sendall(("\r\n".join(lines) + "\r\n\r\n").encode())
        head = self._read_until(b"\r\n\r\n")
        status = head.split(b"\r\n", 1)[0].decode(errors="replace")
        if " 101 " not in status + " ":
            raise ConnectionError(f"websocket upgrade to {url} failed: {status}")
        hdrs = {}
        for ln in head.split(b"\r\n")[1:]:
            if b":" in ln:
                k, v = ln.split(b":", 1)
                hdrs[k.strip().lower()] = v.strip()
        want = base64.b64encode(hashlib.sha1(key.encode() + _GUID).digest())
        if hdrs.get(b"sec-websocket-accept") != want:
            raise ConnectionError("bad Sec-WebSocket-Accept")
        sock.settimeout(None)

    # ------------------------------------------------------------------ io
    def _read_until(self, sep: bytes) -> bytes:
        while sep not in self._buf:
            chunk = self.sock.recv(65536)
            if not chunk:
                raise WebSocketClosed("connection closed during handshake")
            self._buf += chunk
        head, self._buf = self._buf.split(sep, 1)
        return head

    def _read_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self.sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                self.closed = True
                raise WebSocketClosed("connection closed")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def _send_frame(self, op: int, payload: bytes) -> None:
        if self.closed:
            raise WebSocketClosed("send on closed websocket")
        n = len(payload)
        hdr = bytes([0x80 | op])
        if n < 126:
            hdr += bytes([0x80 | n])
        elif n < 65536:
            hdr += bytes([0x80 | 126]) + struct.pack(">H", n)
        else:
            hdr += bytes([0x80 | 127]) + struct.pack(">Q", n)
        mask = os.urandom(4)
        if n:
            m = (mask * (n // 4 + 1))[:n]
            payload = (int.from_bytes(payload, "big") ^ int.from_bytes(m, "big")).to_bytes(n, "big")
        with self._send_lock:
            self.sock.sendall(hdr + mask + payload)

    def send_text(self, s: str) -> None:
        self._send_frame(OP_TEXT, s.encode())

    def send_bytes(self, b: bytes) -> None:
        self._send_frame(OP_BIN, b)

    def recv(self, timeout: Optional[float] = None) -> Optional[Tuple[int, bytes]]:
        """Next data message as (opcode, payload); None on timeout.  Control frames are
        handled here (ping -> pong, close -> WebSocketClosed)."""
        self.sock.settimeout(timeout)
        try:
            parts, first_op = [], None
            while True:
                if not self._buf:
                    try:
                        chunk = self.sock.recv(65536)
                    except socket.timeout:
                        if parts:
                            self.sock.settimeout(None)
                            continue
                        return None
                    if not chunk:
                        self.closed = True
                        raise WebSocketClosed("connection closed")
                    self._buf += chunk
                self.sock.settimeout(None)
                b0, b1 = self._read_exact(2)
                fin, op = b0 & 0x80, b0 & 0x0F
                n = b1 & 0x7F
                if n == 126:
                    n = struct.unpack(">H", self._read_exact(2))[0]
                elif n == 127:
                    n = struct.unpack(">Q", self._read_exact(8))[0]
                mask = self._read_exact(4) if b1 & 0x80 else None
                data = self._read_exact(n)
                if mask:
                    m = (mask * (n // 4 + 1))[:n]
                    data = (int.from_bytes(data, "big") ^ int.from_bytes(m, "big")).to_bytes(n, "big")
                if op == OP_PING:
                    self._send_frame(OP_PONG, data)
                    continue
                if op == OP_PONG:
                    continue
                if op == OP_CLOSE:
                    self.closed = True
                    try:
                        self._send_frame(OP_CLOSE, data[:2])
                    except OSError:
                        pass
                    raise WebSocketClosed(f"closed by peer {data[:2].hex()}")
                if op != OP_CONT:
                    first_op = op
                parts.append(data)
                if fin:
                    return first_op, b"".join(parts)
        finally:
            if not self.closed:
                try:
                    self.sock.settimeout(None)
                except OSError:
                    pass

    def close(self) -> None:
        if not self.closed:
            try:
                self._send_frame(OP_CLOSE, struct.pack(">H", 1000))
            except OSError:
                pass
            self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass
