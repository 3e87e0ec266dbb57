"""Single-node Pravega-style server (controller + segment store in one process).

Serves the framed protocol of ``wire.py`` so the ``pravega`` streaming cluster runs
offline (``langstream pravega-standalone``), the way ``topics/pulsar/standalone.py``
stands in for a Pulsar standalone.  Semantics follow Pravega's client-visible model:

* scopes contain streams; a stream has a fixed number of segments (``ScalingPolicy.fixed``)
  that split the routing-key space evenly; keyless events go to a random segment;
* a sealed stream refuses appends; only sealed streams can be deleted;
* a reader group tracks one read offset per segment and hands the segments out evenly
  to its online readers (rebalanced whenever a reader comes online or goes offline);
  a reader's reads advance the group's offsets for the segments it owns, so a reader
  that goes offline leaves its segments, positioned after its last read event, to the
  remaining readers (Pravega's ``readerOffline(reader, lastPosition)``);
* direct segment reads (offset addressed) serve position-resumable topic readers.

State is in memory (the Pravega standalone default).
"""
from __future__ import annotations

import argparse
import logging
import random
import socket
import socketserver
import threading
import time
from typing import Any, Dict, List, Optional

from . import wire

log = logging.getLogger(__name__)


class PravegaError(Exception):
    pass


class _Stream:
    def __init__(self, n: int):
        self.segments: List[List[bytes]] = [[] for _ in range(max(1, n))]
        self.sealed = False


class _ReaderGroup:
    def __init__(self, stream: str, offsets: List[int]):
        self.stream = stream
        self.offsets = offsets
        self.readers: List[str] = []

    def assignment(self, reader: str) -> List[int]:
        if reader not in self.readers:
            return []
        rs = sorted(self.readers)
        i, n = rs.index(reader), len(rs)
        return [s for s in range(len(self.offsets)) if s % n == i]


class PravegaState:
    def __init__(self):
        self.cond = threading.Condition()
        self.scopes: Dict[str, Dict[str, _Stream]] = {}
        self.groups: Dict[str, Dict[str, _ReaderGroup]] = {}

    def _stream(self, scope: str, stream: str) -> _Stream:
        try:
            return self.scopes[scope][stream]
        except KeyError:
            raise PravegaError(f"stream {scope}/{stream} does not exist") from None

    def _group(self, scope: str, group: str) -> _ReaderGroup:
        try:
            return self.groups[scope][group]
        except KeyError:
            raise PravegaError(f"reader group {scope}/{group} does not exist") from None

    # -- handlers: meta, items -> (reply meta, reply items) --------------------------
    def handle(self, kind: int, m: Dict[str, Any], items: List[bytes]):
        with self.cond:
            if kind == wire.HELLO:
                return {"version": wire.PROTOCOL_VERSION}, None
            if kind == wire.CREATE_SCOPE:
                created = m["scope"] not in self.scopes
                self.scopes.setdefault(m["scope"], {})
                self.groups.setdefault(m["scope"], {})
                return {"created": created}, None
            if kind == wire.SCOPE_EXISTS:
                return {"exists": m["scope"] in self.scopes}, None
            if kind == wire.CREATE_STREAM:
                if m["scope"] not in self.scopes:
                    raise PravegaError(f"scope {m['scope']} does not exist")
                streams = self.scopes[m["scope"]]
                created = m["stream"] not in streams
                if created:
                    streams[m["stream"]] = _Stream(int(m.get("segments", 1)))
                return {"created": created}, None
            if kind == wire.STREAM_INFO:
                s = self.scopes.get(m["scope"], {}).get(m["stream"])
                if s is None:
                    return {"exists": False}, None
                return {"exists": True, "segments": len(s.segments), "sealed": s.sealed,
                        "tails": [len(x) for x in s.segments]}, None
            if kind == wire.SEAL_STREAM:
                self._stream(m["scope"], m["stream"]).sealed = True
                self.cond.notify_all()
                return {}, None
            if kind == wire.DELETE_STREAM:
                s = self._stream(m["scope"], m["stream"])
                if not s.sealed:
                    raise PravegaError(f"stream {m['scope']}/{m['stream']} must be sealed before deletion")
                del self.scopes[m["scope"]][m["stream"]]
                return {}, None
            if kind == wire.APPEND:
                s = self._stream(m["scope"], m["stream"])
                if s.sealed:
                    raise PravegaError(f"stream {m['scope']}/{m['stream']} is sealed")
                n = len(s.segments)
                placed = []
                for key, data in zip(m["keys"], items):
                    seg = wire.segment_for_key(key, n) if key is not None else random.randrange(n)
                    s.segments[seg].append(data)
                    placed.append([seg, len(s.segments[seg]) - 1])
                self.cond.notify_all()
                return {"placed": placed}, None
            if kind == wire.CREATE_READER_GROUP:
                groups = self.groups.setdefault(m["scope"], {})
                if m["group"] in groups:
                    return {"created": False}, None
                s = self._stream(m["scope"], m["stream"])
                start = m.get("start", "head")
                if start == "tail":
                    offsets = [len(x) for x in s.segments]
                elif isinstance(start, dict):
                    offsets = [int(start.get(str(i), 0)) for i in range(len(s.segments))]
                else:
                    offsets = [0] * len(s.segments)
                groups[m["group"]] = _ReaderGroup(m["stream"], offsets)
                return {"created": True}, None
            if kind == wire.DELETE_READER_GROUP:
                self.groups.get(m["scope"], {}).pop(m["group"], None)
                self.cond.notify_all()
                return {}, None
            if kind == wire.READER_ONLINE:
                g = self._group(m["scope"], m["group"])
                if m["reader"] not in g.readers:
                    g.readers.append(m["reader"])
                return {"segments": g.assignment(m["reader"])}, None
            if kind == wire.READER_OFFLINE:
                g = self.groups.get(m["scope"], {}).get(m["group"])
                if g is not None and m["reader"] in g.readers:
                    g.readers.remove(m["reader"])
                    self.cond.notify_all()
                return {}, None
            if kind == wire.READ_NEXT:
                return self._read_next(m)
            if kind == wire.READ_SEGMENT:
                s = self._stream(m["scope"], m["stream"])
                seg, off, mx = int(m["segment"]), int(m["offset"]), int(m.get("max", 500))
                data = s.segments[seg][off:off + mx]
                return {"offset": off, "count": len(data), "tail": len(s.segments[seg])}, data
            raise PravegaError(f"unknown command {kind}")

    def _read_next(self, m):
        deadline = time.monotonic() + max(0, int(m.get("timeout_ms", 1000))) / 1000.0
        mx = int(m.get("max", 500))
        while True:
            g = self._group(m["scope"], m["group"])
            s = self._stream(m["scope"], g.stream)
            owned = g.assignment(m["reader"])
            events, data = [], []
            for seg in owned:
                off = g.offsets[seg]
                take = s.segments[seg][off:off + mx - len(data)]
                for i, d in enumerate(take):
                    events.append([seg, off + i])
                    data.append(d)
                g.offsets[seg] = off + len(take)
                if len(data) >= mx:
                    break
            left = deadline - time.monotonic()
            if data or left <= 0:
                return {"events": events, "segments": owned,
                        "end": s.sealed and all(g.offsets[i] >= len(s.segments[i]) for i in owned)}, data
            self.cond.wait(left)


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        state: PravegaState = self.server.state  # type: ignore[attr-defined]
        sock: socket.socket = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        while True:
            try:
                kind, meta, items = wire.read_frame(sock)
            except (ConnectionError, OSError):
                return
            rid = meta.get("rid")
            try:
                reply, data = state.handle(kind, meta, items)
                reply.update(rid=rid, ok=True)
            except (PravegaError, KeyError, ValueError, TypeError) as e:
                reply, data = {"rid": rid, "ok": False, "error": str(e)}, None
            try:
                sock.sendall(wire.encode(wire.REPLY, reply, data))
            except OSError:
                return


class _Server(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True


class PravegaStandalone:
    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.state = PravegaState()
        self.server = _Server((host, port), _Handler)
        self.server.state = self.state  # type: ignore[attr-defined]
        self.thread: Optional[threading.Thread] = None

    @property
    def controller_uri(self) -> str:
        h, p = self.server.server_address[:2]
        return f"tcp://{h}:{p}"

    def start(self) -> "PravegaStandalone":
        self.thread = threading.Thread(target=self.server.serve_forever, name="pravega-standalone", daemon=True)
        self.thread.start()
        return self

    def stop(self) -> None:
        self.server.shutdown()
        self.server.server_close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser("pravega-standalone")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=9090)
    a = ap.parse_args(argv)
    s = PravegaStandalone(a.host, a.port).start()
    print(f"pravega standalone listening on {s.controller_uri}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        s.stop()
    return 0
