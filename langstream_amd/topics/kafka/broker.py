"""Single-node Kafka-protocol broker (asyncio) for development, tests and single-host
multi-process deployments (the "docker run" mode of the reference starts a real
single-node Kafka -- SURVEY §2.3 C9; this is the in-tree equivalent).

Speaks the same API subset as ``client.py`` (``protocol.VERSIONS``) and implements:
topics/partitions with offsets, long-poll Fetch (``max_wait`` / ``min_bytes``),
ListOffsets, Create/DeleteTopics (+ auto-create on Metadata/Produce when enabled),
and a group coordinator: JoinGroup (new members wait for the rebalance barrier:
every known member rejoins or its rebalance timeout expires), SyncGroup (followers wait
for the leader's assignment), Heartbeat (REBALANCE_IN_PROGRESS while rebalancing),
LeaveGroup, session expiry, OffsetCommit/OffsetFetch.  Storage is in memory.
"""
from __future__ import annotations

import asyncio
import logging
import struct
import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

from . import protocol as P
from .security import SCRAM_MECHANISMS, ScramServer

log = logging.getLogger(__name__)


class _Partition:
    def __init__(self):
        self.records: List[Tuple[Optional[bytes], Optional[bytes], list, int]] = []


class _Group:
    def __init__(self, gid: str):
        self.id = gid
        self.members: Dict[str, Dict[str, Any]] = {}
        self.generation = 0
        self.leader: Optional[str] = None
        self.protocol: Optional[str] = None
        self.state = "Empty"  # Empty | PreparingRebalance | CompletingRebalance | Stable
        self.pending_joins: Dict[str, asyncio.Future] = {}
        self.pending_syncs: Dict[str, asyncio.Future] = {}
        self.assignments: Dict[str, bytes] = {}
        self.rebalance_task: Optional[asyncio.Task] = None


# what DescribeConfigs reports for a topic setting the creator did not pass (Kafka defaults)
TOPIC_CONFIG_DEFAULTS = {"cleanup.policy": "delete", "retention.ms": "604800000", "retention.bytes": "-1",
                         "max.message.bytes": "1048588", "segment.bytes": "1073741824"}


class KafkaBroker:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, auto_create_topics: bool = True,
                 default_partitions: int = 1, node_id: int = 0, ssl_context=None,
                 sasl_users: Optional[Dict[str, str]] = None):
        """``ssl_context``: a server-side SSLContext -> TLS listener (SSL / SASL_SSL);
        ``sasl_users``: {username: password} -> SASL (PLAIN or SCRAM-SHA-256/512) required
        before any other API
        (an unauthenticated request closes the connection, as a Kafka broker does)."""
        self.host, self.port = host, port
        self.ssl_context = ssl_context
        self.sasl_users = sasl_users
        self.node_id = node_id
        self.auto_create = auto_create_topics
        self.default_partitions = default_partitions
        self.topics: Dict[str, List[_Partition]] = {}
        self.topic_configs: Dict[str, Dict[str, Optional[str]]] = {}   # CreateTopics configs (DescribeConfigs)
        self.groups: Dict[str, _Group] = {}
        self.offsets: Dict[Tuple[str, str, int], int] = {}
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread: Optional[threading.Thread] = None
        self._server = None
        self._data_cv: Optional[asyncio.Condition] = None
        self._started = threading.Event()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "KafkaBroker":
        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._data_cv = asyncio.Condition()
            self._server = self._loop.run_until_complete(
                asyncio.start_server(self._handle, self.host, self.port, ssl=self.ssl_context))
            self.port = self._server.sockets[0].getsockname()[1]
            self._loop.create_task(self._expire_sessions())
            self._started.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, daemon=True, name="kafka-broker")
        self._thread.start()
        self._started.wait(10)
        return self

    def stop(self) -> None:
        if self._loop is None:
            return

        async def shut():
            self._server.close()
            me = asyncio.current_task()
            tasks = [t for t in asyncio.all_tasks() if t is not me]
            for t in tasks:
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
        try:
            asyncio.run_coroutine_threadsafe(shut(), self._loop).result(5)
        except Exception:  # noqa: BLE001
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(5)

    @property
    def bootstrap(self) -> str:
        return f"{self.host}:{self.port}"

    # ------------------------------------------------------------------ connection
    async def _handle(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter) -> None:
        authed = not self.sasl_users
        scram = None
        try:
            while True:
                hdr = await reader.readexactly(4)
                n = struct.unpack(">i", hdr)[0]
                payload = await reader.readexactly(n)
                api, ver, corr, client_id, body = P.parse_request(payload)
                if body is None:
                    if api == P.API_VERSIONS:
                        body = {}
                    else:
                        log.warning("unsupported api %s v%s", api, ver)
                        writer.close()
                        return
                if api == P.SASL_HANDSHAKE:
                    offered = (["PLAIN"] + list(SCRAM_MECHANISMS)) if self.sasl_users else []
                    mech = body["mechanism"]
                    ok = mech in offered
                    scram = ScramServer(mech, self.sasl_users) if ok and mech in SCRAM_MECHANISMS else None
                    resp = {"error": P.NONE if ok else P.UNSUPPORTED_SASL_MECHANISM, "mechanisms": offered}
                elif api == P.SASL_AUTHENTICATE and scram is not None:
                    reply, done = scram.step(bytes(body["auth_bytes"]))
                    authed = bool(done)
                    failed = done is False
                    resp = {"error": P.SASL_AUTHENTICATION_FAILED if failed else P.NONE,
                            "error_message": "Authentication failed: SCRAM " + reply.decode() if failed else None,
                            "auth_bytes": b"" if failed else reply}
                elif api == P.SASL_AUTHENTICATE:
                    parts = bytes(body["auth_bytes"]).split(b"\0")
                    user, pw = (parts[1].decode(), parts[2].decode()) if len(parts) == 3 else (None, None)
                    authed = user is not None and self.sasl_users.get(user) == pw
                    resp = {"error": P.NONE if authed else P.SASL_AUTHENTICATION_FAILED,
                            "error_message": None if authed else "Authentication failed: invalid credentials",
                            "auth_bytes": b""}
                elif not authed and api != P.API_VERSIONS:
                    log.warning("unauthenticated request %s from %s: closing", api, client_id)
                    return
                else:
                    resp = await self._dispatch(api, body, client_id or "client")
                writer.write(P.response_frame(corr, api, resp))
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError):
            pass
        finally:
            try:
                writer.close()
            except Exception:  # noqa: BLE001
                pass

    async def _dispatch(self, api: int, b: Dict[str, Any], client_id: str) -> Dict[str, Any]:
        if api == P.API_VERSIONS:
            return {"error": 0, "apis": [{"key": k, "min": v, "max": v} for k, v in sorted(P.VERSIONS.items())]}
        if api == P.METADATA:
            return self._metadata(b["topics"])
        if api == P.CREATE_TOPICS:
            out = []
            for t in b["topics"]:
                if t["name"] in self.topics:
                    out.append({"name": t["name"], "error": P.TOPIC_ALREADY_EXISTS})
                else:
                    self.topics[t["name"]] = [_Partition() for _ in range(max(1, t["num_partitions"]))]
                    self.topic_configs[t["name"]] = {c["name"]: c["value"] for c in t.get("configs") or []}
                    out.append({"name": t["name"], "error": P.NONE})
            return {"topics": out}
        if api == P.DESCRIBE_CONFIGS:
            res = []
            for r in b["resources"]:
                if r["type"] != P.RESOURCE_TOPIC or r["name"] not in self.topics:
                    res.append({"error": P.UNKNOWN_TOPIC_OR_PARTITION, "error_message": f"unknown {r['name']}",
                                "type": r["type"], "name": r["name"], "configs": []})
                    continue
                conf = dict(TOPIC_CONFIG_DEFAULTS)
                conf.update(self.topic_configs.get(r["name"], {}))
                want = r.get("config_names")
                res.append({"error": P.NONE, "error_message": None, "type": r["type"], "name": r["name"],
                            "configs": [{"name": k, "value": v, "read_only": False,
                                         "is_default": k not in self.topic_configs.get(r["name"], {}),
                                         "sensitive": False} for k, v in sorted(conf.items())
                                        if not want or k in want]})
            return {"throttle": 0, "resources": res}
        if api == P.DELETE_TOPICS:
            out = []
            for name in b["topics"]:
                ok = self.topics.pop(name, None) is not None
                self.topic_configs.pop(name, None)
                out.append({"name": name, "error": P.NONE if ok else P.UNKNOWN_TOPIC_OR_PARTITION})
            return {"topics": out}
        if api == P.PRODUCE:
            return await self._produce(b)
        if api == P.FETCH:
            return await self._fetch(b)
        if api == P.LIST_OFFSETS:
            out = []
            for t in b["topics"]:
                parts = []
                for p in t["partitions"]:
                    tp = self.topics.get(t["name"])
                    if tp is None or p["partition"] >= len(tp):
                        parts.append({"partition": p["partition"], "error": P.UNKNOWN_TOPIC_OR_PARTITION,
                                      "timestamp": -1, "offset": -1})
                        continue
                    off = 0 if p["timestamp"] == -2 else len(tp[p["partition"]].records)
                    parts.append({"partition": p["partition"], "error": 0, "timestamp": -1, "offset": off})
                out.append({"name": t["name"], "partitions": parts})
            return {"topics": out}
        if api == P.FIND_COORDINATOR:
            return {"error": 0, "node_id": self.node_id, "host": self.host, "port": self.port}
        if api == P.JOIN_GROUP:
            return await self._join(b, client_id)
        if api == P.SYNC_GROUP:
            return await self._sync(b)
        if api == P.HEARTBEAT:
            g = self.groups.get(b["group_id"])
            if g is None or b["member_id"] not in g.members:
                return {"error": P.UNKNOWN_MEMBER_ID}
            g.members[b["member_id"]]["last_hb"] = time.monotonic()
            if b["generation"] != g.generation:
                return {"error": P.ILLEGAL_GENERATION}
            if g.state == "PreparingRebalance":
                return {"error": P.REBALANCE_IN_PROGRESS}
            return {"error": 0}
        if api == P.LEAVE_GROUP:
            g = self.groups.get(b["group_id"])
            if g is not None and b["member_id"] in g.members:
                del g.members[b["member_id"]]
                self._start_rebalance(g)
            return {"error": 0}
        if api == P.OFFSET_COMMIT:
            g = self.groups.get(b["group_id"])
            out = []
            for t in b["topics"]:
                parts = []
                for p in t["partitions"]:
                    err = 0
                    if g is not None and b["generation"] >= 0 and (b["member_id"] not in g.members):
                        err = P.UNKNOWN_MEMBER_ID
                    elif g is not None and b["generation"] >= 0 and b["generation"] != g.generation:
                        err = P.ILLEGAL_GENERATION
                    else:
                        self.offsets[(b["group_id"], t["name"], p["partition"])] = p["offset"]
                    parts.append({"partition": p["partition"], "error": err})
                out.append({"name": t["name"], "partitions": parts})
            return {"topics": out}
        if api == P.OFFSET_FETCH:
            out = []
            for t in b["topics"]:
                out.append({"name": t["name"], "partitions": [
                    {"partition": p, "offset": self.offsets.get((b["group_id"], t["name"], p), -1), "metadata": None,
                     "error": 0} for p in t["partitions"]]})
            return {"topics": out}
        raise ValueError(f"api {api} not handled")

    # ------------------------------------------------------------------ data path
    def _ensure(self, name: str) -> Optional[List[_Partition]]:
        t = self.topics.get(name)
        if t is None and self.auto_create:
            t = self.topics[name] = [_Partition() for _ in range(self.default_partitions)]
        return t

    def _metadata(self, names: Optional[List[str]]) -> Dict[str, Any]:
        names = list(self.topics) if names is None else names
        topics = []
        for n in names:
            t = self._ensure(n)
            if t is None:
                topics.append({"error": P.UNKNOWN_TOPIC_OR_PARTITION, "name": n, "internal": False, "partitions": []})
                continue
            topics.append({"error": 0, "name": n, "internal": False, "partitions": [
                {"error": 0, "partition": i, "leader": self.node_id, "replicas": [self.node_id],
                 "isr": [self.node_id]} for i in range(len(t))]})
        return {"brokers": [{"node_id": self.node_id, "host": self.host, "port": self.port, "rack": None}],
                "controller_id": self.node_id, "topics": topics}

    async def _produce(self, b) -> Dict[str, Any]:
        out = []
        now = int(time.time() * 1000)
        for t in b["topics"]:
            parts = []
            tp = self._ensure(t["name"])
            for p in t["partitions"]:
                if tp is None or p["partition"] >= len(tp):
                    parts.append({"partition": p["partition"], "error": P.UNKNOWN_TOPIC_OR_PARTITION,
                                  "base_offset": -1, "log_append_time": -1})
                    continue
                part = tp[p["partition"]]
                base = len(part.records)
                for _off, ts, k, v, hs in P.decode_batches(p["records"], verify_crc=True):
                    part.records.append((k, v, hs, ts if ts > 0 else now))
                parts.append({"partition": p["partition"], "error": 0, "base_offset": base, "log_append_time": -1})
            out.append({"name": t["name"], "partitions": parts})
        async with self._data_cv:
            self._data_cv.notify_all()
        return {"topics": out, "throttle": 0}

    def _collect(self, b) -> Tuple[Dict[str, Any], int]:
        total = 0
        topics = []
        for t in b["topics"]:
            tp = self.topics.get(t["name"])
            parts = []
            for p in t["partitions"]:
                if tp is None or p["partition"] >= len(tp):
                    parts.append({"partition": p["partition"], "error": P.UNKNOWN_TOPIC_OR_PARTITION, "hw": -1,
                                  "lso": -1, "aborted": None, "records": None})
                    continue
                recs = tp[p["partition"]].records
                off = p["offset"]
                hw = len(recs)
                if off > hw:
                    parts.append({"partition": p["partition"], "error": P.OFFSET_OUT_OF_RANGE, "hw": hw, "lso": hw,
                                  "aborted": None, "records": None})
                    continue
                chunk, size = [], 0
                for r in recs[off:]:
                    size += (len(r[0] or b"") + len(r[1] or b"") + 32)
                    chunk.append(r)
                    if size >= p["max_bytes"] or len(chunk) >= 1000:
                        break
                data = P.encode_batch(off, chunk) if chunk else None
                total += len(chunk)
                parts.append({"partition": p["partition"], "error": 0, "hw": hw, "lso": hw, "aborted": None,
                              "records": data})
            topics.append({"name": t["name"], "partitions": parts})
        return {"throttle": 0, "topics": topics}, total

    async def _fetch(self, b) -> Dict[str, Any]:
        resp, n = self._collect(b)
        if n >= max(1, b["min_bytes"]) or b["max_wait"] <= 0:
            return resp
        deadline = time.monotonic() + b["max_wait"] / 1000.0
        async with self._data_cv:
            while True:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    await asyncio.wait_for(self._data_cv.wait(), timeout=left)
                except asyncio.TimeoutError:
                    break
                resp, n = self._collect(b)
                if n:
                    return resp
        resp, _ = self._collect(b)
        return resp

    # ------------------------------------------------------------------ group coordinator
    async def _join(self, b, client_id: str) -> Dict[str, Any]:
        g = self.groups.setdefault(b["group_id"], _Group(b["group_id"]))
        mid = b["member_id"]
        if mid and mid not in g.members:
            return {"error": P.UNKNOWN_MEMBER_ID, "generation": -1, "protocol": "", "leader": "",
                    "member_id": mid, "members": []}
        if not mid:
            mid = f"{client_id}-{uuid.uuid4()}"
        meta = b["protocols"][0]["metadata"] if b["protocols"] else b""
        g.protocol = b["protocols"][0]["name"] if b["protocols"] else "range"
        g.members[mid] = {"metadata": meta, "last_hb": time.monotonic(), "session": b["session_timeout"],
                          "rebalance": b["rebalance_timeout"]}
        fut = self._loop.create_future()
        old = g.pending_joins.get(mid)
        if old is not None and not old.done():
            old.cancel()
        g.pending_joins[mid] = fut
        self._start_rebalance(g)
        self._maybe_complete(g)
        return await fut

    def _start_rebalance(self, g: _Group) -> None:
        if g.state != "PreparingRebalance":
            g.state = "PreparingRebalance" if g.members else "Empty"
            for f in g.pending_syncs.values():
                if not f.done():
                    f.set_result({"error": P.REBALANCE_IN_PROGRESS, "assignment": b""})
            g.pending_syncs.clear()
            if g.members:
                timeout = max((m["rebalance"] for m in g.members.values()), default=3000) / 1000.0
                initial = 0.3 if g.generation == 0 else timeout
                g.rebalance_task = self._loop.create_task(self._rebalance_deadline(g, initial))
        self._maybe_complete(g)

    async def _rebalance_deadline(self, g: _Group, delay: float) -> None:
        await asyncio.sleep(delay)
        if g.state != "PreparingRebalance":
            return
        for m in [m for m in g.members if m not in g.pending_joins]:
            del g.members[m]  # did not rejoin in time
        self._complete(g)

    def _maybe_complete(self, g: _Group) -> None:
        if g.state == "PreparingRebalance" and g.members and all(m in g.pending_joins for m in g.members) \
                and g.generation > 0:
            self._complete(g)

    def _complete(self, g: _Group) -> None:
        if not g.members:
            g.state = "Empty"
            return
        g.generation += 1
        g.leader = sorted(g.members)[0]
        g.state = "CompletingRebalance"
        g.assignments = {}
        members = [{"member_id": m, "metadata": g.members[m]["metadata"]} for m in sorted(g.members)]
        for mid, fut in list(g.pending_joins.items()):
            if fut.done():
                continue
            fut.set_result({"error": 0, "generation": g.generation, "protocol": g.protocol or "range",
                            "leader": g.leader, "member_id": mid, "members": members if mid == g.leader else []})
        g.pending_joins.clear()
        if g.rebalance_task is not None:
            g.rebalance_task.cancel()
            g.rebalance_task = None

    async def _sync(self, b) -> Dict[str, Any]:
        g = self.groups.get(b["group_id"])
        if g is None or b["member_id"] not in g.members:
            return {"error": P.UNKNOWN_MEMBER_ID, "assignment": b""}
        if b["generation"] != g.generation:
            return {"error": P.ILLEGAL_GENERATION, "assignment": b""}
        if g.state == "PreparingRebalance":
            return {"error": P.REBALANCE_IN_PROGRESS, "assignment": b""}
        if b["member_id"] == g.leader and b["assignments"]:
            g.assignments = {a["member_id"]: a["assignment"] for a in b["assignments"]}
            g.state = "Stable"
            for mid, f in list(g.pending_syncs.items()):
                if not f.done():
                    f.set_result({"error": 0, "assignment": g.assignments.get(mid, b"")})
            g.pending_syncs.clear()
        if g.state == "Stable":
            return {"error": 0, "assignment": g.assignments.get(b["member_id"], b"")}
        fut = self._loop.create_future()
        g.pending_syncs[b["member_id"]] = fut
        return await fut

    async def _expire_sessions(self) -> None:
        while True:
            await asyncio.sleep(0.5)
            now = time.monotonic()
            for g in list(self.groups.values()):
                dead = [m for m, d in g.members.items()
                        if m not in g.pending_joins and now - d["last_hb"] > d["session"] / 1000.0]
                if dead:
                    for m in dead:
                        del g.members[m]
                    self._start_rebalance(g)


def main(argv=None) -> int:
    """Standalone broker process (``python -m langstream_amd.topics.kafka.broker``): the
    single-node Kafka of the reference's docker mode in its own interpreter, so broker
    work never contends for the agents' GIL.  Prints ``bootstrap=<host:port>`` once
    listening and serves until stdin closes or SIGTERM."""
    import argparse
    import signal
    import sys
    ap = argparse.ArgumentParser(prog="langstream_amd.topics.kafka.broker")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--partitions", type=int, default=1, help="partitions of auto-created topics")
    ap.add_argument("--no-auto-create", action="store_true")
    a = ap.parse_args(argv)
    b = KafkaBroker(a.host, a.port, auto_create_topics=not a.no_auto_create,
                    default_partitions=a.partitions).start()
    done = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    print(f"bootstrap={b.bootstrap}", flush=True)

    def watch_stdin():
        try:
            sys.stdin.read()
        except Exception:  # noqa: BLE001
            pass
        done.set()
    threading.Thread(target=watch_stdin, daemon=True).start()
    done.wait()
    b.stop()
    return 0


class BrokerProcess:
    """A broker in a child interpreter; the parent holds its stdin, so the broker also
    ends when the parent dies."""

    def __init__(self, partitions: int = 1, host: str = "127.0.0.1"):
        from ...utils.procs import read_tagged, spawn_module
        self.proc = spawn_module("langstream_amd.topics.kafka.broker",
                                 ["--host", host, "--partitions", str(partitions)])
        self.bootstrap = read_tagged(self.proc, "bootstrap=", "broker process")

    def stop(self) -> None:
        from ...utils.procs import close_stdin_and_wait
        close_stdin_and_wait(self.proc)


if __name__ == "__main__":
    raise SystemExit(main())
