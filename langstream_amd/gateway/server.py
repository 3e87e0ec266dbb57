"""API gateway: WebSocket produce / consume / chat and HTTP produce / service
(SURVEY §2.7 G2-G4).

Parity:
* paths ``/v1/{produce,consume,chat}/{tenant}/{application}/{gateway}`` (WebSocket) and
  ``/api/gateways/produce/...`` (HTTP POST), ``/api/gateways/service/.../**``
  (``WebSocketConfig.java:47-99``, ``GatewayResource.java:95-400``);
* query string: ``param:<name>`` (gateway parameters; required ones enforced, unknown
  ones rejected), ``option:<name>`` (``position`` = latest | earliest | base64 offset),
  ``credentials`` / ``test-credentials`` (``GatewayRequestHandler.java:60-298``);
* produce: client sends ``{"key","value","headers"}``, gets
  ``{"status": OK|BAD_REQUEST|PRODUCER_ERROR, "reason"}``; configured produce headers
  (value / value-from-parameters / value-from-authentication) are added and may not be
  overridden by the client (``ProduceGateway.java``); producers are cached per
  (tenant, app, gateway, topic) in an LRU of 100 (``LRUTopicProducerCache``);
* consume: pushes ``{"record": {"key","value","headers"}, "offset": <base64>}`` for
  every record passing the header filters (``ConsumeGateway.java``);
* chat: reader on ``answers-topic`` filtered by ``chat-options.headers`` + producer to
  ``questions-topic`` with the same headers (``ChatHandler.java``);
* service: with ``agent-id`` the request is proxied to that service agent's HTTP
  endpoint; otherwise request/response over topics correlated by the
  ``langstream-service-request-id`` header (first matching record on the output topic
  completes the HTTP response);
* ``events-topic``: ClientConnected / ClientDisconnected event records.

The gateway runs on aiohttp in its own event-loop thread; topic IO (blocking reads on
the native in-memory log or Kafka) runs in worker threads and is bridged to the
WebSocket with ``call_soon_threadsafe``.
"""
from __future__ import annotations

import asyncio
import base64
import json
import logging
import threading
import time
import uuid
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api.model import Application, ComputeCluster, Gateway, Instance, KeyValueComparison, StreamingCluster
from ..api.record import Header, Record, SimpleRecord
from ..api.topics import TopicConnectionsRuntimeRegistry, TopicOffsetPosition
from ..core.placeholders import resolve_placeholders
from ..core.store import ApplicationStore
from .auth import PROVIDER_CACHE, AuthResult, load_provider, test_principal_values

log = logging.getLogger(__name__)
SERVICE_REQUEST_ID_HEADER = "langstream-service-request-id"


class GatewayError(Exception):
    def __init__(self, msg: str, status: int = 400):
        super().__init__(msg)
        self.status = status


@dataclass
class RequestContext:
    tenant: str
    application_id: str
    application: Application
    gateway: Gateway
    credentials: Optional[str] = None
    test_credentials: Optional[str] = None
    http_headers: Dict[str, str] = field(default_factory=dict)
    options: Dict[str, str] = field(default_factory=dict)
    user_parameters: Dict[str, str] = field(default_factory=dict)
    principal_values: Dict[str, str] = field(default_factory=dict)

    @property
    def is_test_mode(self) -> bool:
        return self.test_credentials is not None

    @property
    def streaming_cluster(self) -> StreamingCluster:
        inst = self.application.instance
        if inst is None or inst.streaming_cluster is None:
            return StreamingCluster("memory", {})
        return inst.streaming_cluster


def _required_params(gw: Gateway) -> List[str]:
    params = list(gw.parameters or [])
    kvs: List[KeyValueComparison] = []
    if gw.type == "produce":
        kvs = gw.produce_options or []
    elif gw.type == "consume":
        kvs = gw.consume_options or []
    elif gw.type == "chat" and gw.chat_options:
        kvs = gw.chat_options.headers or []
    elif gw.type == "service" and gw.service_options:
        kvs = gw.service_options.headers or []
    for kv in kvs:
        if kv.value_from_parameters and kv.value_from_parameters not in params:
            params.append(kv.value_from_parameters)
    return params


def _kv_value(kv: KeyValueComparison, ctx: RequestContext) -> Optional[str]:
    if kv.value is not None:
        return kv.value
    if kv.value_from_parameters is not None:
        return ctx.user_parameters.get(kv.value_from_parameters)
    if kv.value_from_authentication is not None:
        return ctx.principal_values.get(kv.value_from_authentication)
    return None


def message_filters(kvs: Optional[List[KeyValueComparison]], ctx: RequestContext) -> List[Callable[[Record], bool]]:
    out = []
    for kv in kvs or []:
        if kv.key is None:
            raise GatewayError("Key cannot be null")

        def f(rec: Record, kv=kv) -> bool:
            h = rec.get_header(kv.key)
            if h is None or h.value_as_string() is None:
                return False
            want = _kv_value(kv, ctx)
            return want is not None and h.value_as_string() == want
        out.append(f)
    return out


def common_headers(kvs: Optional[List[KeyValueComparison]], ctx: RequestContext) -> List[Header]:
    """ProduceGateway.getProducerCommonHeaders: every mapping needs a key and a value."""
    out = []
    for kv in kvs or []:
        if not kv.key:
            raise GatewayError("Header key cannot be empty")
        v = _kv_value(kv, ctx)
        if v is None:
            raise GatewayError(f"header {kv.key} cannot be empty")
        out.append(Header(kv.key, v))
    return out


class _SharedProducer:
    """A cached topic producer that sessions keep using after the cache evicts it
    (``LRUTopicProducerCache``'s reference-counted handles, LRUTopicProducerCacheTest):
    an evicted producer closes once its in-flight writes finish, and a session that writes
    through it later reopens it for that write instead of failing on a closed producer."""

    def __init__(self, factory):
        self._factory = factory
        self._lock = threading.Lock()
        self._p = factory()
        self._inflight = 0
        self._evicted = False

    def write(self, record):
        with self._lock:
            if self._p is None:
                self._p = self._factory()
            self._inflight += 1
            p = self._p
        try:
            fut = p.write(record)
        except BaseException:
            self._done(None)
            raise
        fut.add_done_callback(self._done)
        return fut

    def _done(self, _f) -> None:
        close = None
        with self._lock:
            self._inflight -= 1
            if self._evicted and self._inflight == 0 and self._p is not None:
                close, self._p = self._p, None
        if close is not None:
            _close_quietly(close)

    def evict(self) -> None:
        close = None
        with self._lock:
            self._evicted = True
            if self._inflight == 0 and self._p is not None:
                close, self._p = self._p, None
        if close is not None:
            _close_quietly(close)

    @property
    def closed(self) -> bool:
        return self._p is None

    def __getattr__(self, name):
        return getattr(self._p, name)


def _close_quietly(p) -> None:
    try:
        p.close()
    except Exception:  # noqa: BLE001
        pass


class _ProducerCache:
    def __init__(self, size: int = 100):
        self.size = size
        self._d: "OrderedDict[tuple, _SharedProducer]" = OrderedDict()
        self._lock = threading.Lock()

    def get_or_create(self, key: tuple, factory) -> _SharedProducer:
        with self._lock:
            p = self._d.get(key)
            if p is not None:
                self._d.move_to_end(key)
                return p
            p = _SharedProducer(factory)
            self._d[key] = p
            while len(self._d) > self.size:
                _, old = self._d.popitem(last=False)
                old.evict()
            return p


class GatewayService:
    """Request validation, authentication and topic plumbing shared by WS and HTTP."""

    def __init__(self, store: ApplicationStore, test_auth: Optional[tuple] = None,
                 service_url_resolver: Optional[Callable[[str, str, str], str]] = None):
        self.store = store
        self.test_provider = load_provider(test_auth[0], test_auth[1]) if test_auth else None
        self.producers = _ProducerCache()
        self.service_url_resolver = service_url_resolver or (lambda t, a, agent: "http://127.0.0.1:8000")

    # -- validation / auth
    def validate(self, tenant: str, app_id: str, gw_id: str, gtype: str, query: Dict[str, str],
                 headers: Dict[str, str]) -> RequestContext:
        stored = self.store.get(tenant, app_id)
        if stored is None:
            raise GatewayError(f"application {app_id} not found", 404)
        app = resolve_placeholders(stored.application)
        gw = next((g for g in app.gateways or [] if g.id == gw_id and g.type == gtype), None)
        if gw is None:
            raise GatewayError(f"gateway {gw_id} of type {gtype} is not defined in the application", 404)
        q = dict(query)
        creds, test_creds = q.pop("credentials", None), q.pop("test-credentials", None)
        options, params = {}, {}
        check = not (gtype == "service" and gw.service_options and gw.service_options.agent_id)
        if check:
            for k, v in q.items():
                if k.startswith("option:"):
                    options[k[len("option:"):]] = v
                elif k.startswith("param:"):
                    params[k[len("param:"):]] = v
                else:
                    raise GatewayError(f"invalid query parameter {k}. To specify a gateway parameter, use the format "
                                       f"param:<parameter_name>.To specify a option, use the format "
                                       f"option:<option_name>.")
        err = lambda m: GatewayError(f"Error for gateway {gw.id} (tenant: {tenant}, appId: {app_id}): {m}")  # noqa
        required = _required_params(gw)
        leftover = set(params)
        for p in required:
            if not (params.get(p) or "").strip():
                raise err(f"missing required parameter {p}. Required parameters: [{', '.join(required)}]")
            leftover.discard(p)
        if leftover:
            raise err(f"unknown parameters: [{', '.join(sorted(leftover))}]")
        for k, v in options.items():
            if gtype in ("consume", "chat") and k == "position":
                if not v.strip():
                    raise GatewayError("'position' cannot be blank")
            elif gtype != "service" or not check:
                raise GatewayError(f"Unknown option {k}")
        if creds is not None and test_creds is not None:
            raise err("credentials and test-credentials cannot be used together")
        return RequestContext(tenant, app_id, app, gw, creds, test_creds, dict(headers), options, params)

    def authenticate(self, ctx: RequestContext) -> None:
        auth = ctx.gateway.authentication
        if auth is None or auth.provider is None:
            return
        if ctx.is_test_mode:
            if not auth.allow_test_mode:
                raise GatewayError(f"Gateway {ctx.gateway.id} of tenant {ctx.tenant} does not allow test mode.", 401)
            if self.test_provider is None:
                raise GatewayError("No test auth provider specified", 401)
            res = self.test_provider.authenticate(_CredView(ctx, ctx.test_credentials))
            if res is None or not res.authenticated:
                raise GatewayError(res.reason if res else "Authentication provider returned null", 401)
            ctx.principal_values = test_principal_values(ctx.test_credentials)
            return
        res: AuthResult = PROVIDER_CACHE.get(auth.provider, auth.configuration).authenticate(ctx)
        if res is None:
            raise GatewayError("Authentication provider returned null", 401)
        if not res.authenticated:
            raise GatewayError(res.reason or "authentication failed", 401)
        ctx.principal_values = dict(res.principal_values or {})

    # -- topic plumbing
    def _runtime(self, ctx: RequestContext):
        return TopicConnectionsRuntimeRegistry.get(ctx.streaming_cluster)

    def producer(self, ctx: RequestContext, topic: str):
        sc = ctx.streaming_cluster
        key = (ctx.tenant, ctx.application_id, ctx.gateway.id, topic, sc.type, json.dumps(sc.configuration,
                                                                                          sort_keys=True, default=str))

        def make():
            p = self._runtime(ctx).create_producer(None, sc, {"topic": topic})
            p.start()
            return p
        return self.producers.get_or_create(key, make)

    def reader(self, ctx: RequestContext, topic: str):
        pos = TopicOffsetPosition.parse(ctx.options.get("position", "latest"))
        r = self._runtime(ctx).create_reader(ctx.streaming_cluster, {"topic": topic}, pos)
        r.start()
        return r

    @staticmethod
    def produce(producer, headers: List[Header], payload: Any) -> Dict[str, Any]:
        if isinstance(payload, (str, bytes)):
            try:
                req = json.loads(payload)
                if not isinstance(req, dict):
                    raise ValueError("not an object")
            except ValueError as e:
                return {"status": "BAD_REQUEST", "reason": f"Error while parsing JSON payload: {e}"}
        else:
            req = payload
        if req.get("value") is None and req.get("key") is None:
            return {"status": "BAD_REQUEST", "reason": "Either key or value must be set."}
        hs = list(headers)
        configured = {h.key for h in hs}
        for k, v in (req.get("headers") or {}).items():
            if k in configured:
                return {"status": "BAD_REQUEST", "reason": f"Header {k} is configured as parameter-level header."}
            hs.append(Header(k, v))
        try:
            producer.write(SimpleRecord.of(req.get("key"), req.get("value"), hs)).result(30)
        except Exception as e:  # noqa: BLE001
            return {"status": "PRODUCER_ERROR", "reason": str(e)}
        return {"status": "OK", "reason": None}

    @staticmethod
    def push_message(rec: Record, offset: Optional[bytes]) -> str:
        hs = {h.key: h.value_as_string() for h in rec.headers()}
        v = rec.value()
        if isinstance(v, bytes):
            v = v.decode("utf-8", errors="replace")
        k = rec.key()
        if isinstance(k, bytes):
            k = k.decode("utf-8", errors="replace")
        return json.dumps({"record": {"key": k, "value": v, "headers": hs},
                           "offset": base64.b64encode(offset).decode() if offset else None}, default=str)

    def send_event(self, ctx: RequestContext, typ: str) -> None:
        topic = ctx.gateway.events_topic
        if not topic:
            return
        ev = {"category": "Gateway", "type": typ, "timestamp": int(time.time() * 1000),
              "source": {"tenant": ctx.tenant, "applicationId": ctx.application_id,
                         "gateway": {"id": ctx.gateway.id, "type": ctx.gateway.type, "topic": ctx.gateway.topic,
                                     "parameters": list(ctx.gateway.parameters or []),
                                     "events-topic": ctx.gateway.events_topic}},
              "data": {"userParameters": ctx.user_parameters, "options": ctx.options,
                       "httpRequestHeaders": {k.lower(): v for k, v in (ctx.http_headers or {}).items()}}}
        try:
            self.producer(ctx, topic).write(SimpleRecord.of(None, json.dumps(ev))).result(10)
        except Exception as e:  # noqa: BLE001
            log.warning("cannot write gateway event: %s", e)


class _CredView:
    def __init__(self, ctx: RequestContext, creds: Optional[str]):
        self.tenant = ctx.tenant
        self.credentials = creds
        self.application_id = ctx.application_id


class _ReaderPump:
    """Blocking topic reader in a thread -> asyncio queue of JSON messages."""

    def __init__(self, loop, reader, filters, on_msg: Callable[[str], None]):
        self.loop, self.reader, self.filters, self.on_msg = loop, reader, filters, on_msg
        self.stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True, name="gateway-reader")
        self.t.start()

    def _run(self) -> None:
        try:
            while not self.stop.is_set():
                res = self.reader.read()
                for rec in res.records:
                    if all(f(rec) for f in self.filters):
                        msg = GatewayService.push_message(rec, res.offset)
                        self.loop.call_soon_threadsafe(self.on_msg, msg)
        except Exception as e:  # noqa: BLE001
            log.info("gateway reader stopped: %s", e)
        finally:
            try:
                self.reader.close()
            except Exception:  # noqa: BLE001
                pass

    def close(self) -> None:
        self.stop.set()


class _ReaderHub:
    """One topic reader shared by every ``latest``-positioned consume/chat session of a
    gateway whose filters are header equalities (the chat case: one answers topic, a
    ``session``-like header per client).

    The reference gives every WebSocket its own reader that scans the whole topic and
    drops records for other sessions (``GW/gateways/ConsumeGateway.java:40-270``), so N
    sessions cost O(N) filter evaluations per record -- with per-token chunk streaming
    that is the gateway's bottleneck well before the GPU's.  Here a record is read
    once and routed by a dict lookup on its filter-header values: O(1) per record."""

    def __init__(self, reader, keys: Tuple[str, ...], on_empty: Callable[["_ReaderHub"], None]):
        self.reader, self.keys, self.on_empty = reader, keys, on_empty
        self.subs: Dict[tuple, List[tuple]] = {}
        self.lock = threading.Lock()
        self.stop = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True, name="gateway-hub")
        self.t.start()

    def subscribe(self, want: tuple, loop, on_msg) -> "_HubSubscription":
        entry = (loop, on_msg)
        with self.lock:
            self.subs.setdefault(want, []).append(entry)
        return _HubSubscription(self, want, entry)

    def unsubscribe(self, want: tuple, entry) -> None:
        with self.lock:
            lst = self.subs.get(want)
            if lst and entry in lst:
                lst.remove(entry)
                if not lst:
                    del self.subs[want]
            empty = not self.subs
        if empty:
            self.on_empty(self)

    def _run(self) -> None:
        keys = self.keys
        try:
            while not self.stop.is_set():
                res = self.reader.read()
                for rec in res.records:
                    vals = []
                    for k in keys:
                        h = rec.get_header(k)
                        v = h.value_as_string() if h is not None else None
                        if v is None:
                            break
                        vals.append(v)
                    else:
                        with self.lock:
                            targets = list(self.subs.get(tuple(vals), ()))
                        if targets:
                            msg = GatewayService.push_message(rec, res.offset)
                            for loop, on_msg in targets:
                                loop.call_soon_threadsafe(on_msg, msg)
        except Exception as e:  # noqa: BLE001
            log.info("gateway hub reader stopped: %s", e)
        finally:
            try:
                self.reader.close()
            except Exception:  # noqa: BLE001
                pass


class _HubSubscription:
    def __init__(self, hub: _ReaderHub, want: tuple, entry):
        self.hub, self.want, self.entry = hub, want, entry

    def close(self) -> None:
        self.hub.unsubscribe(self.want, self.entry)


class GatewayServer:
    def __init__(self, service: GatewayService, host: str = "127.0.0.1", port: int = 8091):
        self.service = service
        self.host, self.port = host, port
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread: Optional[threading.Thread] = None
        self._runner = None
        self._started = threading.Event()
        self._hubs: Dict[tuple, _ReaderHub] = {}
        self._hubs_lock = threading.Lock()

    # ------------------------------------------------------------------ app
    def make_app(self):
        from aiohttp import web
        app = web.Application(client_max_size=64 * 1024 * 1024)
        app.router.add_get("/v1/produce/{tenant}/{application}/{gateway}", self._ws_produce)
        app.router.add_get("/v1/consume/{tenant}/{application}/{gateway}", self._ws_consume)
        app.router.add_get("/v1/chat/{tenant}/{application}/{gateway}", self._ws_chat)
        app.router.add_post("/api/gateways/produce/{tenant}/{application}/{gateway}", self._http_produce)
        app.router.add_route("*", "/api/gateways/service/{tenant}/{application}/{gateway}", self._http_service)
        app.router.add_route("*", "/api/gateways/service/{tenant}/{application}/{gateway}/{tail:.*}",
                             self._http_service)
        app.router.add_get("/management/health", lambda r: web.json_response({"status": "UP"}))
        return app

    def _ctx(self, request, gtype: str) -> RequestContext:
        m = request.match_info
        ctx = self.service.validate(m["tenant"], m["application"], m["gateway"], gtype, dict(request.query),
                                    dict(request.headers))
        self.service.authenticate(ctx)
        return ctx

    async def _prepare(self, request, gtype):
        from aiohttp import web
        try:
            ctx = await asyncio.get_running_loop().run_in_executor(None, self._ctx, request, gtype)
        except GatewayError as e:
            raise _http_error(e)
        ws = web.WebSocketResponse(heartbeat=30)
        await ws.prepare(request)
        return ctx, ws

    async def _produce_loop(self, ws, ctx, producer, headers):
        from aiohttp import WSMsgType
        loop = asyncio.get_running_loop()
        async for msg in ws:
            if msg.type == WSMsgType.TEXT:
                resp = await loop.run_in_executor(None, self.service.produce, producer, headers, msg.data)
                await ws.send_str(json.dumps(resp))
            elif msg.type in (WSMsgType.ERROR, WSMsgType.CLOSE):
                break

    async def _ws_produce(self, request):
        ctx, ws = await self._prepare(request, "produce")
        loop = asyncio.get_running_loop()
        producer = await loop.run_in_executor(None, self.service.producer, ctx, ctx.gateway.topic)
        await loop.run_in_executor(None, self.service.send_event, ctx, "ClientConnected")
        try:
            await self._produce_loop(ws, ctx, producer, common_headers(ctx.gateway.produce_options, ctx))
        finally:
            await loop.run_in_executor(None, self.service.send_event, ctx, "ClientDisconnected")
        return ws

    async def _pump_to_ws(self, ws, ctx, topic, kvs):
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        pump = None
        if kvs and str(ctx.options.get("position", "latest")).lower() == "latest":
            pump = await loop.run_in_executor(None, self._hub_subscribe, ctx, topic, kvs, loop, q.put_nowait)
        if pump is None:
            reader = await loop.run_in_executor(None, self.service.reader, ctx, topic)
            pump = _ReaderPump(loop, reader, message_filters(kvs, ctx), q.put_nowait)

        async def sender():
            while True:
                m = await q.get()
                if ws.closed:
                    return
                await ws.send_str(m)
        return pump, asyncio.ensure_future(sender())

    def _hub_subscribe(self, ctx: RequestContext, topic: str, kvs, loop, on_msg):
        message_filters(kvs, ctx)   # same validation as the per-session path
        want = tuple(_kv_value(kv, ctx) for kv in kvs)
        if any(w is None for w in want):
            return None             # a filter that can never match: per-session semantics
        keys = tuple(kv.key for kv in kvs)
        hk = (ctx.tenant, ctx.application_id, topic, keys)
        with self._hubs_lock:
            hub = self._hubs.get(hk)
            if hub is None or hub.stop.is_set():
                hub = _ReaderHub(self.service.reader(ctx, topic), keys, lambda h, hk=hk: self._hub_empty(hk, h))
                self._hubs[hk] = hub
            return hub.subscribe(tuple(str(w) for w in want), loop, on_msg)

    def _hub_empty(self, hk: tuple, hub: _ReaderHub) -> None:
        with self._hubs_lock:
            with hub.lock:
                if hub.subs:
                    return          # re-subscribed meanwhile
            hub.stop.set()
            if self._hubs.get(hk) is hub:
                del self._hubs[hk]

    async def _ws_consume(self, request):
        from aiohttp import WSMsgType
        ctx, ws = await self._prepare(request, "consume")
        loop = asyncio.get_running_loop()
        # the reader is positioned first: a consumer of its own gateway's events topic sees
        # its ClientConnected event (ProduceConsumeHandlerTest.testSendEvents)
        pump, task = await self._pump_to_ws(ws, ctx, ctx.gateway.topic, ctx.gateway.consume_options)
        await loop.run_in_executor(None, self.service.send_event, ctx, "ClientConnected")
        try:
            async for msg in ws:
                if msg.type in (WSMsgType.ERROR, WSMsgType.CLOSE):
                    break
        finally:
            pump.close()
            task.cancel()
            await loop.run_in_executor(None, self.service.send_event, ctx, "ClientDisconnected")
        return ws

    async def _ws_chat(self, request):
        ctx, ws = await self._prepare(request, "chat")
        loop = asyncio.get_running_loop()
        co = ctx.gateway.chat_options
        pump, task = await self._pump_to_ws(ws, ctx, co.answers_topic, co.headers)
        producer = await loop.run_in_executor(None, self.service.producer, ctx, co.questions_topic)
        await loop.run_in_executor(None, self.service.send_event, ctx, "ClientConnected")
        try:
            await self._produce_loop(ws, ctx, producer, common_headers(co.headers, ctx))
        finally:
            pump.close()
            task.cancel()
            await loop.run_in_executor(None, self.service.send_event, ctx, "ClientDisconnected")
        return ws

    async def _http_produce(self, request):
        from aiohttp import web
        loop = asyncio.get_running_loop()
        try:
            ctx = await loop.run_in_executor(None, self._ctx, request, "produce")
        except GatewayError as e:
            raise _http_error(e)
        body = await request.text()
        payload: Any = body
        if not (request.content_type or "").startswith("application/json"):
            payload = {"value": body}
        producer = await loop.run_in_executor(None, self.service.producer, ctx, ctx.gateway.topic)
        resp = await loop.run_in_executor(None, self.service.produce, producer,
                                          common_headers(ctx.gateway.produce_options, ctx), payload)
        return web.json_response(resp, status=200 if resp["status"] == "OK" else 400)

    async def _http_service(self, request):
        from aiohttp import web
        loop = asyncio.get_running_loop()
        try:
            ctx = await loop.run_in_executor(None, self._ctx, request, "service")
        except GatewayError as e:
            raise _http_error(e)
        so = ctx.gateway.service_options
        if so.agent_id:
            return await self._proxy(request, ctx, so.agent_id)
        if request.method != "POST":
            raise web.HTTPMethodNotAllowed(request.method, ["POST"])
        body = await request.text()
        payload = json.loads(body) if (request.content_type or "").startswith("application/json") and body else \
            {"value": body}
        req_id = str(uuid.uuid4())
        fut: asyncio.Future = loop.create_future()
        reader = await loop.run_in_executor(None, self.service.reader, ctx, so.output_topic)
        filters = message_filters(so.headers, ctx) + [
            lambda r: (r.get_header(SERVICE_REQUEST_ID_HEADER) is not None
                       and r.get_header(SERVICE_REQUEST_ID_HEADER).value_as_string() == req_id)]
        pump = _ReaderPump(loop, reader, filters, lambda m: fut.done() or fut.set_result(m))
        try:
            producer = await loop.run_in_executor(None, self.service.producer, ctx, so.input_topic)
            payload = dict(payload)
            payload["headers"] = dict(payload.get("headers") or {}, **{SERVICE_REQUEST_ID_HEADER: req_id})
            resp = await loop.run_in_executor(None, self.service.produce, producer,
                                              common_headers(so.headers, ctx), payload)
            if resp["status"] != "OK":
                return web.json_response(resp, status=400)
            msg = await asyncio.wait_for(fut, timeout=float(ctx.options.get("timeout", 120)))
            return web.Response(text=msg, content_type="application/json")
        except asyncio.TimeoutError:
            raise web.HTTPGatewayTimeout(text="no response from the service pipeline")
        finally:
            pump.close()

    async def _proxy(self, request, ctx, agent_id):
        import aiohttp
        from aiohttp import web
        base = self.service.service_url_resolver(ctx.tenant, ctx.application_id, agent_id)
        tail = request.match_info.get("tail", "")
        url = base.rstrip("/") + "/" + tail
        if request.query_string:
            url += "?" + request.query_string
        hdrs = {k: v for k, v in request.headers.items()
                if k.lower() not in ("connection", "content-length", "expect", "host", "upgrade")}
        async with aiohttp.ClientSession() as s:
            async with s.request(request.method, url, data=await request.read(), headers=hdrs) as r:
                body = await r.read()
                return web.Response(body=body, status=r.status,
                                    headers={k: v for k, v in r.headers.items()
                                             if k.lower() not in ("content-length", "transfer-encoding",
                                                                  "content-encoding", "connection")})

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "GatewayServer":
        def run():
            from aiohttp import web
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._runner = web.AppRunner(self.make_app())
            self._loop.run_until_complete(self._runner.setup())
            site = web.TCPSite(self._runner, self.host, self.port)
            try:
                self._loop.run_until_complete(site.start())
            except OSError as e:      # e.g. the port is taken: start() raises it
                self._start_error = e
                self._started.set()
                return
            if self.port == 0:
                self.port = site._server.sockets[0].getsockname()[1]
            self._started.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, daemon=True, name="api-gateway")
        self._start_error = None
        self._thread.start()
        self._started.wait(30)
        if self._start_error is not None:
            self._loop = None
            raise self._start_error
        return self

    def stop(self) -> None:
        if self._loop is None:
            return

        async def shutdown():
            await self._runner.cleanup()
        fut = asyncio.run_coroutine_threadsafe(shutdown(), self._loop)
        try:
            fut.result(10)
        except Exception:  # noqa: BLE001
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(10)

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"


def _http_error(e: GatewayError):
    """An RFC 7807 problem body, as the reference's HTTP gateway answers
    (GatewayResourceTest.produceJsonAndExpectBadRequest reads ``detail``)."""
    from aiohttp import web
    cls = {401: web.HTTPUnauthorized, 404: web.HTTPNotFound}.get(e.status, web.HTTPBadRequest)
    import http
    code = cls.status_code
    body = json.dumps({"type": "about:blank", "title": http.HTTPStatus(code).phrase, "status": code, "detail": str(e)})
    return cls(text=body, content_type="application/problem+json")
