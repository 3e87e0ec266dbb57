"""Single-process Pulsar-compatible broker speaking the Pulsar **WebSocket API** and the
admin REST subset LangStream uses -- the ``pulsar`` analogue of the in-tree Kafka broker
(``topics/kafka/broker.py``), for ``docker run``-style local runs and the CPU tests
(the reference's Pulsar tests start a Pulsar container: PulsarClusterRuntimeDockerTest).

Endpoints (same paths and JSON bodies as a Pulsar broker with the WebSocket service on):
* ``/ws/v2/producer/persistent/{tenant}/{ns}/{topic}``: ``{"payload": b64, "properties",
  "key", "context"}`` -> ``{"result": "ok", "messageId", "context"}``.  Keyed messages go
  to ``hash(key) % partitions``, unkeyed round-robin.
* ``/ws/v2/consumer/persistent/{tenant}/{ns}/{topic}/{subscription}?subscriptionType=``
  ``Exclusive|Failover|Shared`` (+ ``subscriptionInitialPosition=Earliest|Latest``,
  ``receiverQueueSize``): pushes ``{"messageId", "payload", "properties", "publishTime",
  "key", "redeliveryCount"}``; the client acks with ``{"messageId"}``.  Failover: each
  partition has ONE active consumer (partition i -> i-th of the subscription's consumers
  in connect order); unacked messages are redelivered when their consumer disconnects.
* ``/ws/v2/reader/persistent/...?messageId=earliest|latest|<b64 id>`` (starts AFTER an
  explicit id, like ``Reader.startMessageId``).
* admin ``/admin/v2/persistent/{t}/{ns}/{topic}`` PUT/DELETE, ``.../partitions`` PUT (body =
  count) / GET / DELETE, ``/admin/v2/persistent/{t}/{ns}`` GET (topic list).
* schema registry ``/admin/v2/schemas/{t}/{ns}/{topic}/schema`` GET (``{"version", "type",
  "timestamp", "data", "properties"}``, 404 without one) / POST (``{"type", "schema",
  "properties"}``) / DELETE.  With ``schema_enforced`` (the namespace policy
  ``schemaValidationEnforced``) a produced message must decode under the topic's schema
  (a KeyValue message: its key too), else the send fails -- what a broker does for a
  producer whose schema does not match.
Topics are auto-created on first produce/subscribe (``allowAutoTopicCreation``).
Message ids are opaque base64 tokens (``partition:entry``).
"""
from __future__ import annotations

import asyncio
import base64
import json
import threading
import time
import zlib
from dataclasses import dataclass, field
from datetime import datetime, timezone
from typing import Dict, List, Optional, Set

from aiohttp import WSMsgType, web


@dataclass
class _Msg:
    entry: int
    payload: bytes
    properties: Dict[str, str]
    key: Optional[str]
    publish_ms: int


@dataclass
class _Partition:
    name: str
    log: List[_Msg] = field(default_factory=list)
    cond: Optional[asyncio.Condition] = None


@dataclass
class _Topic:
    name: str                    # persistent://t/ns/topic
    partitions: int              # 0 = non-partitioned
    parts: List[_Partition] = field(default_factory=list)
    rr: int = 0


@dataclass
class _Consumer:
    ws: web.WebSocketResponse
    name: str
    queue: int
    unacked: Set[tuple] = field(default_factory=set)


@dataclass
class _Sub:
    mode: str
    consumers: List[_Consumer] = field(default_factory=list)
    cursor: Dict[int, int] = field(default_factory=dict)      # next entry to deliver, per partition
    acked: Dict[int, Set[int]] = field(default_factory=dict)
    redeliver: Dict[int, int] = field(default_factory=dict)   # entry -> redelivery count (flat key p<<40|e)
    wake: Optional[asyncio.Event] = None


def _mid(p: int, e: int) -> str:
    return base64.b64encode(f"{p}:{e}".encode()).decode()


def _parse_mid(s: str):
    p, e = base64.b64decode(s).decode().split(":")
    return int(p), int(e)


class PulsarStandalone:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, schema_enforced: bool = False):
        self.host, self.port = host, port
        self.schema_enforced = schema_enforced
        self.schemas: Dict[str, List[dict]] = {}     # base topic -> versions (GetSchemaResponse)
        self.topics: Dict[str, _Topic] = {}
        self.subs: Dict[tuple, _Sub] = {}
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._runner: Optional[web.AppRunner] = None
        self._thread: Optional[threading.Thread] = None
        self._ready = threading.Event()
        self._sockets: Set[web.WebSocketResponse] = set()

    # ------------------------------------------------------------------ lifecycle
    @property
    def web_url(self) -> str:
        return f"http://{self.host}:{self.port}"

    @property
    def service_url(self) -> str:
        return f"pulsar://{self.host}:{self.port}"

    def start(self) -> "PulsarStandalone":
        self._thread = threading.Thread(target=self._run, name="pulsar-standalone", daemon=True)
        self._thread.start()
        if not self._ready.wait(15):
            raise RuntimeError("pulsar standalone did not start")
        return self

    def stop(self) -> None:
        if self._loop is not None:
            fut = asyncio.run_coroutine_threadsafe(self._shutdown(), self._loop)
            try:
                fut.result(10)
            except Exception:  # noqa: BLE001
                pass
            self._loop.call_soon_threadsafe(self._loop.stop)
        if self._thread is not None:
            self._thread.join(10)

    async def _shutdown(self):
        for ws in list(self._sockets):        # every producer / consumer / reader socket
            try:
                await asyncio.wait_for(ws.close(), 2)
            except Exception:  # noqa: BLE001
                pass
        if self._runner is not None:
            await self._runner.cleanup()

    def _run(self):
        self._loop = asyncio.new_event_loop()
        asyncio.set_event_loop(self._loop)
        app = web.Application()
        base = "/admin/v2/persistent/{tenant}/{ns}"
        app.router.add_get(base, self._list_topics)
        app.router.add_get(base + "/partitioned", self._list_partitioned)
        app.router.add_put(base + "/{topic}", self._create_topic)
        app.router.add_delete(base + "/{topic}", self._delete_topic)
        app.router.add_put(base + "/{topic}/partitions", self._create_partitioned)
        app.router.add_get(base + "/{topic}/partitions", self._get_partitions)
        app.router.add_delete(base + "/{topic}/partitions", self._delete_topic)
        sch = "/admin/v2/schemas/{tenant}/{ns}/{topic}/schema"
        app.router.add_get(sch, self._get_schema)
        app.router.add_post(sch, self._post_schema)
        app.router.add_delete(sch, self._delete_schema)
        ws = "/ws/v2/{kind}/persistent/{tenant}/{ns}/{topic}"
        app.router.add_get(ws, self._ws)
        app.router.add_get(ws + "/{sub}", self._ws)
        self._runner = web.AppRunner(app)
        self._loop.run_until_complete(self._runner.setup())
        site = web.TCPSite(self._runner, self.host, self.port)
        self._loop.run_until_complete(site.start())
        self.port = site._server.sockets[0].getsockname()[1]
        self._ready.set()
        self._loop.run_forever()

    # ------------------------------------------------------------------ topics
    @staticmethod
    def _full(req) -> str:
        m = req.match_info
        return f"persistent://{m['tenant']}/{m['ns']}/{m['topic']}"

    def _make(self, name: str, partitions: int) -> _Topic:
        t = _Topic(name, partitions)
        n = max(1, partitions)
        for i in range(n):
            pn = f"{name}-partition-{i}" if partitions > 0 else name
            t.parts.append(_Partition(pn, cond=asyncio.Condition()))
        self.topics[name] = t
        return t

    def _get_or_create(self, name: str):
        """-> (topic, partition indices addressed by `name`)."""
        t = self.topics.get(name)
        if t is None:
            base, _, idx = name.rpartition("-partition-")
            bt = self.topics.get(base)
            if idx.isdigit() and bt is not None and int(idx) < len(bt.parts):
                return bt, [int(idx)]  # one partition of a partitioned topic
            t = self._make(name, 0)
        return t, list(range(len(t.parts)))

    async def _create_topic(self, req):
        name = self._full(req)
        if name in self.topics:
            return web.json_response({"reason": "This topic already exists"}, status=409)
        self._make(name, 0)
        return web.Response(status=204)

    async def _create_partitioned(self, req):
        name = self._full(req)
        try:
            n = int((await req.text()).strip() or "0")
        except ValueError:
            return web.json_response({"reason": "partitions must be an integer"}, status=400)
        if n <= 0:
            return web.json_response({"reason": "Number of partitions should be more than 0"}, status=412)
        if name in self.topics:
            return web.json_response({"reason": "This topic already exists"}, status=409)
        self._make(name, n)
        return web.Response(status=204)

    async def _get_partitions(self, req):
        t = self.topics.get(self._full(req))
        return web.json_response({"partitions": t.partitions if t else 0})

    async def _delete_topic(self, req):
        name = self._full(req)
        if self.topics.pop(name, None) is None:
            return web.json_response({"reason": "Topic not found"}, status=404)
        for k in [k for k in self.subs if k[0] == name]:
            for c in self.subs[k].consumers:
                await c.ws.close()
            del self.subs[k]
        return web.Response(status=204)

    async def _list_topics(self, req):
        m = req.match_info
        pre = f"persistent://{m['tenant']}/{m['ns']}/"
        out = []
        for t in self.topics.values():
            if t.name.startswith(pre):
                out += [p.name for p in t.parts]
        return web.json_response(sorted(out))

    async def _list_partitioned(self, req):
        m = req.match_info
        pre = f"persistent://{m['tenant']}/{m['ns']}/"
        return web.json_response(sorted(t.name for t in self.topics.values()
                                        if t.name.startswith(pre) and t.partitions > 0))

    # ------------------------------------------------------------------ schemas
    async def _get_schema(self, req):
        v = self.schemas.get(self._full(req))
        if not v:
            return web.json_response({"reason": "Schema not found"}, status=404)
        return web.json_response(v[-1])

    async def _post_schema(self, req):
        from .schema import SchemaError, TopicSchema
        body = await req.json()
        name = self._full(req)
        doc = {"version": len(self.schemas.get(name, [])), "type": str(body.get("type", "BYTES")).upper(),
               "timestamp": int(time.time() * 1000), "data": body.get("schema") or "",
               "properties": body.get("properties") or {}}
        try:
            ts = TopicSchema.from_rest(doc)
        except (SchemaError, ValueError) as e:
            return web.json_response({"reason": f"Invalid schema definition: {e}"}, status=422)
        cur = self.schemas.get(name)
        if cur and TopicSchema.from_rest(cur[-1]) == ts:
            return web.json_response({"version": cur[-1]["version"]})
        if cur and self.schema_enforced:
            return web.json_response({"reason": "Schema not compatible with the existing one"}, status=409)
        self.schemas.setdefault(name, []).append(doc)
        return web.json_response({"version": doc["version"]})

    async def _delete_schema(self, req):
        if self.schemas.pop(self._full(req), None) is None:
            return web.json_response({"reason": "Schema not found"}, status=404)
        return web.json_response({"version": 0})

    def _validate(self, topic: _Topic, key: Optional[str], payload: bytes) -> Optional[str]:
        """None when the message decodes under the topic's schema (enforcement on)."""
        if not self.schema_enforced:
            return None
        v = self.schemas.get(topic.name)
        if not v:
            return None
        from .schema import TopicSchema
        try:
            ts = TopicSchema.from_rest(v[-1])
            if payload or ts.value.type not in ("STRING", "BYTES", "NONE"):
                ts.value.decode(payload)
            if ts.is_kv and key is not None and ts.key.type != "STRING":
                ts.key.decode(base64.b64decode(key))
            if ts.value.type == "AVRO" and payload:
                # the whole payload must be one Avro datum
                from ...api import avro
                if avro.encode(ts.value._avro, ts.value.decode(payload)) != payload:
                    return "payload is not exactly one Avro datum of the topic's schema"
        except Exception as e:  # noqa: BLE001
            return f"message does not match the topic's {v[-1]['type']} schema: {e}"
        return None

    # ------------------------------------------------------------------ websocket
    async def _ws(self, req):
        kind = req.match_info["kind"]
        if kind not in ("producer", "consumer", "reader"):
            return web.Response(status=404)
        ws = web.WebSocketResponse(heartbeat=30)
        await ws.prepare(req)
        self._sockets.add(ws)
        topic, pids = self._get_or_create(self._full(req))
        try:
            if kind == "producer":
                await self._producer(ws, topic, pids)
            elif kind == "consumer":
                await self._consumer(ws, topic, pids, req.match_info.get("sub") or "sub", req.query)
            else:
                await self._reader(ws, topic, pids, req.query)
        finally:
            self._sockets.discard(ws)
            await ws.close()
        return ws

    async def _producer(self, ws, topic: _Topic, pids: List[int]):
        async for msg in ws:
            if msg.type != WSMsgType.TEXT:
                continue
            try:
                d = json.loads(msg.data)
                payload = base64.b64decode(d.get("payload") or "")
            except (ValueError, TypeError) as e:
                await ws.send_json({"result": "send-error:1", "errorMsg": str(e)})
                continue
            key = d.get("key")
            bad = self._validate(topic, key, payload)
            if bad is not None:
                await ws.send_json({"result": "send-error:2", "errorMsg": bad, "context": d.get("context")})
                continue
            n = len(pids)
            if key is not None:
                p = pids[zlib.crc32(str(key).encode()) % n]
            else:
                p = pids[topic.rr % n]
                topic.rr += 1
            part = topic.parts[p]
            e = len(part.log)
            part.log.append(_Msg(e, payload, {str(k): str(v) for k, v in (d.get("properties") or {}).items()},
                                 key, int(time.time() * 1000)))
            async with part.cond:
                part.cond.notify_all()
            for s in self.subs.values():
                if s.wake is not None:
                    s.wake.set()
            await ws.send_json({"result": "ok", "messageId": _mid(p, e), "context": d.get("context")})

    @staticmethod
    def _wire(p: int, m: _Msg, redelivery: int = 0) -> dict:
        ts = datetime.fromtimestamp(m.publish_ms / 1000, tz=timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%f")[:-3] + "Z"
        d = {"messageId": _mid(p, m.entry), "payload": base64.b64encode(m.payload).decode(),
             "properties": m.properties, "publishTime": ts, "redeliveryCount": redelivery}
        if m.key is not None:
            d["key"] = m.key
        return d

    @staticmethod
    def _owned(sub: _Sub, c: _Consumer, pids: List[int]) -> List[int]:
        if sub.mode == "Shared":
            return pids
        if not sub.consumers:
            return []
        if sub.mode == "Exclusive" or len(pids) == 1:
            return pids if sub.consumers[0] is c else []
        idx = sub.consumers.index(c)
        return [p for p in pids if p % len(sub.consumers) == idx]

    async def _consumer(self, ws, topic: _Topic, pids: List[int], sub_name: str, q):
        mode = q.get("subscriptionType", "Exclusive")
        key = (topic.name, tuple(pids), sub_name)
        sub = self.subs.get(key)
        latest = q.get("subscriptionInitialPosition", "Latest").lower() == "latest"
        if sub is None:
            sub = _Sub(mode, wake=asyncio.Event())
            for p, part in enumerate(topic.parts):
                sub.cursor[p] = len(part.log) if latest else 0
                sub.acked[p] = set()
            self.subs[key] = sub
        elif mode == "Exclusive" and sub.consumers:
            await ws.send_json({"result": "error", "errorMsg": "Exclusive consumer is already connected"})
            return
        c = _Consumer(ws, f"c{id(ws)}", int(q.get("receiverQueueSize", 1000)))
        sub.consumers.append(c)
        sub.wake.set()
        sender = asyncio.ensure_future(self._deliver(ws, topic, pids, sub, c))
        try:
            async for msg in ws:
                if msg.type != WSMsgType.TEXT:
                    continue
                try:
                    d = json.loads(msg.data)
                    p, e = _parse_mid(d["messageId"])
                except (ValueError, KeyError, TypeError):
                    continue
                if d.get("type") == "negativeAcknowledge":
                    c.unacked.discard((p, e))
                    sub.cursor[p] = min(sub.cursor.get(p, 0), e)
                    sub.redeliver[(p << 40) | e] = sub.redeliver.get((p << 40) | e, 0) + 1
                else:
                    c.unacked.discard((p, e))
                    sub.acked.setdefault(p, set()).add(e)
                sub.wake.set()
        finally:
            sender.cancel()
            sub.consumers.remove(c)
            for p, e in c.unacked:  # redeliver what this consumer never acked
                sub.cursor[p] = min(sub.cursor.get(p, 0), e)
                sub.redeliver[(p << 40) | e] = sub.redeliver.get((p << 40) | e, 0) + 1
            sub.wake.set()

    async def _deliver(self, ws, topic: _Topic, pids: List[int], sub: _Sub, c: _Consumer):
        while not ws.closed:
            sent = 0
            for p in self._owned(sub, c, pids):
                log = topic.parts[p].log
                cur = sub.cursor.get(p, 0)
                acked = sub.acked.setdefault(p, set())
                while cur < len(log) and len(c.unacked) < c.queue:
                    if cur not in acked and not any((p, cur) in o.unacked for o in sub.consumers):
                        c.unacked.add((p, cur))
                        await ws.send_json(self._wire(p, log[cur], sub.redeliver.get((p << 40) | cur, 0)))
                        sent += 1
                    cur += 1
                sub.cursor[p] = cur
            if not sent:
                sub.wake.clear()
                try:
                    await asyncio.wait_for(sub.wake.wait(), 0.5)
                except asyncio.TimeoutError:
                    pass

    async def _reader(self, ws, topic: _Topic, pids: List[int], q):
        if len(pids) != 1:
            await ws.send_json({"result": "error", "errorMsg": "reader needs a non-partitioned topic or a partition"})
            return
        pid = pids[0]
        part = topic.parts[pid]
        start = q.get("messageId", "latest")
        if start == "earliest":
            cur = 0
        elif start == "latest":
            cur = len(part.log)
        else:
            cur = _parse_mid(start)[1] + 1
        acker = asyncio.ensure_future(self._drain(ws))
        try:
            while not ws.closed:
                while cur < len(part.log):
                    await ws.send_json(self._wire(pid, part.log[cur]))
                    cur += 1
                async with part.cond:
                    try:
                        await asyncio.wait_for(part.cond.wait(), 0.5)
                    except asyncio.TimeoutError:
                        pass
        finally:
            acker.cancel()

    @staticmethod
    async def _drain(ws):
        async for _ in ws:  # reader acks are flow-control only here
            pass


def main(argv=None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="Pulsar-compatible single-node broker (WebSocket API + admin)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--schema-enforced", action="store_true",
                    help="reject messages that do not decode under the topic's schema")
    a = ap.parse_args(argv)
    b = PulsarStandalone(a.host, a.port, schema_enforced=a.schema_enforced).start()
    print(f"pulsar standalone on {b.web_url}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        b.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
