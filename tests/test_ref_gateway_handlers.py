"""The reference's gateway handler tests, ported (``langstream-api-gateway/src/test/java/ai/
langstream/apigateway/``: ``websocket/handlers/ProduceConsumeHandlerTest`` and
``http/GatewayResourceTest``), on the memory streaming cluster, the in-tree Kafka broker and the Pulsar stand-in (the Java
suite's Kafka and Pulsar subclasses).  Each case builds the
application the Java test builds (one module, the case's topics, the case's gateways) and
talks to the gateway over WebSockets / HTTP.

Deliberate difference: a WebSocket handshake the gateway refuses (bad parameters) answers
HTTP 400 with the reason, where the reference's servlet container answers 500."""
import asyncio
import json
import uuid

import pytest
import requests
import yaml

from ref_runtime_harness import instance_yaml
from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.parser import build_application_instance
from langstream_amd.core.store import InMemoryApplicationStore, StoredApplication
from langstream_amd.gateway.server import GatewayServer, GatewayService
from langstream_amd.topics.kafka.broker import KafkaBroker
from langstream_amd.topics.memory import reset_memlogs

class GW:
    def __init__(self, topics, gateways, streaming="memory", bootstrap=None, test_auth=None, resolver=None):
        reset_memlogs()
        module = {"module": "mod1", "id": "p",
                  "topics": [{"name": t, "creation-mode": "create-if-not-exists"} for t in topics]}
        files = {"module.yaml": yaml.safe_dump(module), "gateways.yaml": yaml.safe_dump({"gateways": gateways})}
        app = self.app = build_application_instance(files, instance_yaml(streaming, bootstrap), None).application
        # prepareTopicsForTest: the topics exist before any client connects
        dep = ApplicationDeployer()
        dep.setup("tenant1", dep.create_implementation("application1", app))
        store = InMemoryApplicationStore()
        store.put(StoredApplication("application1", "tenant1", app, files))
        self.srv = GatewayServer(GatewayService(store, test_auth=test_auth, service_url_resolver=resolver),
                                 port=0).start()
        self.ws = self.srv.url.replace("http", "ws")
        self.http = self.srv.url

    def close(self):
        self.srv.stop()
        reset_memlogs()


@pytest.fixture(scope="module")
def kafka():
    b = KafkaBroker(default_partitions=1).start()
    yield b
    b.stop()


@pytest.fixture(scope="module")
def pulsar():
    from langstream_amd.topics.pulsar.standalone import PulsarStandalone
    b = PulsarStandalone().start()
    yield b
    b.stop()


@pytest.fixture(params=["memory", "kafka", "pulsar"])
def gw(request, kafka, pulsar):
    """Every case on the memory streaming cluster, the in-tree Kafka broker and the Pulsar
    stand-in (the Java suite's Kafka* / Pulsar* ProduceConsumeHandlerTest and
    GatewayResourceTest subclasses)."""
    made = []

    def make(topics, gateways, test_auth=None):
        boot = {"kafka": kafka.bootstrap, "pulsar": (pulsar.web_url, pulsar.service_url, "public", "default")}
        g = GW(topics, gateways, request.param, boot.get(request.param), test_auth)
        made.append(g)
        return g
    yield make
    for g in made:
        g.close()


def _topic():
    return "topic" + uuid.uuid4().hex[:8]


def _run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


async def _produce(s, url, req):
    ws = await s.ws_connect(url)
    await ws.send_str(req if isinstance(req, str) else json.dumps(req))
    resp = json.loads((await ws.receive(timeout=10)).data)
    await ws.close()
    return resp


class _Collector:
    def __init__(self):
        self.msgs = []

    async def start(self, s, url, settle=True):
        self.ws = await s.ws_connect(url)
        self.task = asyncio.ensure_future(self._loop())
        if settle:
            await asyncio.sleep(0.3)     # the reader is positioned before anything is produced
        return self

    async def _loop(self):
        async for m in self.ws:
            self.msgs.append(json.loads(m.data))

    def records(self):
        return [(m["record"]["key"], m["record"]["value"], m["record"]["headers"]) for m in self.msgs]

    async def wait(self, n, timeout=10.0):
        for _ in range(int(timeout / 0.05)):
            if len(self.msgs) >= n:
                return
            await asyncio.sleep(0.05)

    async def close(self):
        await self.ws.close()
        self.task.cancel()


def test_simple_produce_consume(gw):
    """ProduceConsumeHandlerTest.testSimpleProduceConsume"""
    import aiohttp
    t = _topic()
    g = gw([t], [{"id": "produce", "type": "produce", "topic": t}, {"id": "consume", "type": "consume", "topic": t}])

    async def go():
        async with aiohttp.ClientSession() as s:
            c = await _Collector().start(s, f"{g.ws}/v1/consume/tenant1/application1/consume")
            r = await _produce(s, f"{g.ws}/v1/produce/tenant1/application1/produce", {"value": "this is a message"})
            assert r["status"] == "OK"
            await c.wait(1)
            assert c.records() == [(None, "this is a message", {})]
            await c.close()
    _run(go())


@pytest.mark.parametrize("kind", ["consume", "produce"])
def test_parameters_required(gw, kind):
    """ProduceConsumeHandlerTest.testParametersRequired"""
    import aiohttp
    t = _topic()
    g = gw([t], [{"id": "gw", "type": kind, "topic": t, "parameters": ["session-id"]}])

    async def go():
        async with aiohttp.ClientSession() as s:
            base = f"{g.ws}/v1/{kind}/tenant1/application1/gw"
            for q in ("", "?param:otherparam=1", "?param:session-id=", "?param:session-id=ok&param:another-non-declared=y"):
                with pytest.raises(aiohttp.WSServerHandshakeError) as e:
                    await s.ws_connect(base + q)
                assert e.value.status == 400
            for q in ("?param:session-id=1", "?param:session-id=string-value"):
                ws = await s.ws_connect(base + q)
                await ws.close()
    _run(go())


def test_filter_out_messages_by_fixed_value(gw):
    """ProduceConsumeHandlerTest.testFilterOutMessagesByFixedValue"""
    import aiohttp
    t = _topic()
    g = gw([t], [
        {"id": "produce", "type": "produce", "topic": t, "parameters": ["session-id"],
         "produce-options": {"headers": [{"key": "header1", "value": "langstream"}]}},
        {"id": "produce-non-langstream", "type": "produce", "topic": t, "parameters": ["session-id"]},
        {"id": "consume", "type": "consume", "topic": t, "parameters": ["session-id"],
         "consume-options": {"filters": {"headers": [{"key": "header1", "value": "langstream"}]}}}])

    async def go():
        async with aiohttp.ClientSession() as s:
            base = f"{g.ws}/v1/consume/tenant1/application1/consume?param:session-id="
            u1 = await _Collector().start(s, base + "user1")
            u2 = await _Collector().start(s, base + "user2")
            await _produce(s, f"{g.ws}/v1/produce/tenant1/application1/produce-non-langstream?param:session-id=user1",
                           {"value": "this is a message non from langstream"})
            await _produce(s, f"{g.ws}/v1/produce/tenant1/application1/produce?param:session-id=user1",
                           {"value": "this is a message for everyone"})
            await u1.wait(1)
            await u2.wait(1)
            await asyncio.sleep(0.3)
            for c in (u1, u2):
                assert c.records() == [(None, "this is a message for everyone", {"header1": "langstream"})]
                await c.close()
    _run(go())


def test_produce(gw):
    """ProduceConsumeHandlerTest.testProduce: reasons for a parameter-level header set by
    the client, an empty request and bad JSON (the parser's own message follows the
    prefix: Python's here, Jackson's there)."""
    import aiohttp
    t = _topic()
    g = gw([t], [{"id": "gw", "type": "produce", "topic": t, "parameters": ["session-id"],
                  "produce-options": {"headers": [{"key": "header1", "value-from-parameters": "session-id"}]}}])

    async def go():
        async with aiohttp.ClientSession() as s:
            url = f"{g.ws}/v1/produce/tenant1/application1/gw?param:session-id=s"
            r = await _produce(s, url, {"value": "hello", "headers": {"header0": "value0", "header2": "value2"}})
            assert r["status"] == "OK"
            r = await _produce(s, url, {"value": "hello", "headers": {"header1": "value1"}})
            assert (r["status"], r["reason"]) == ("BAD_REQUEST", "Header header1 is configured as parameter-level header.")
            r = await _produce(s, url, "{}")
            assert (r["status"], r["reason"]) == ("BAD_REQUEST", "Either key or value must be set.")
            r = await _produce(s, url, "invalid-json")
            assert r["status"] == "BAD_REQUEST" and r["reason"].startswith("Error while parsing JSON payload: ")
    _run(go())


def test_start_from_offsets(gw):
    """ProduceConsumeHandlerTest.testStartFromOffsets: ``option:position`` = an offset a
    consumer was handed (resume after it), ``earliest`` or ``latest``."""
    import aiohttp
    t = _topic()
    g = gw([t], [{"id": "produce", "type": "produce", "topic": t}, {"id": "consume", "type": "consume", "topic": t}])

    async def go():
        async with aiohttp.ClientSession() as s:
            cons = f"{g.ws}/v1/consume/tenant1/application1/consume"
            prod = f"{g.ws}/v1/produce/tenant1/application1/produce"
            c1 = await _Collector().start(s, cons)
            await _produce(s, prod, {"value": "msg1"})
            await c1.wait(1)
            assert c1.records() == [(None, "msg1", {})]
            off1 = c1.msgs[0]["offset"]
            await _produce(s, prod, {"value": "msg2"})
            c_off = await _Collector().start(s, f"{cons}?option:position={off1}")
            await c_off.wait(1)
            assert c_off.records() == [(None, "msg2", {})]
            c_early = await _Collector().start(s, f"{cons}?option:position=earliest")
            await c_early.wait(2)
            assert [v for _, v, _ in c_early.records()] == ["msg1", "msg2"]
            c_late = await _Collector().start(s, f"{cons}?option:position=latest")
            await _produce(s, prod, {"value": "msg3"})
            for c, want in ((c1, ["msg1", "msg2", "msg3"]), (c_off, ["msg2", "msg3"]),
                            (c_early, ["msg1", "msg2", "msg3"]), (c_late, ["msg3"])):
                await c.wait(len(want))
                assert [v for _, v, _ in c.records()] == want
            for c in (c1, c_off, c_early, c_late):
                await c.close()
    _run(go())


def test_http_parameters_required(gw):
    """GatewayResourceTest.testParametersRequired: problem-detail 400s naming the parameter."""
    t = _topic()
    g = gw([t], [{"id": "gw", "type": "produce", "topic": t, "parameters": ["session-id"]}])
    base = f"{g.http}/api/gateways/produce/tenant1/application1/gw"
    body = '{"value": "my-value"}'
    hdr = {"Content-Type": "application/json"}
    for q, msg in (("", "missing required parameter session-id"),
                   ("?param:otherparam=1", "missing required parameter session-id"),
                   ("?param:session-id=", "missing required parameter session-id"),
                   ("?param:session-id=ok&param:another-non-declared=y", "unknown parameters: [another-non-declared]")):
        r = requests.post(base + q, data=body, headers=hdr, timeout=30)
        assert r.status_code == 400 and msg in r.json()["detail"]
    for q in ("?param:session-id=1", "?param:session-id=string-value"):
        r = requests.post(base + q, data=body, headers=hdr, timeout=30)
        assert r.status_code == 200 and r.json()["status"] == "OK"


def test_http_simple_produce(gw):
    """GatewayResourceTest.testSimpleProduce: JSON bodies as produce requests, other
    content types as the record value."""
    t = _topic()
    g = gw([t], [{"id": "produce", "type": "produce", "topic": t}])
    url = f"{g.http}/api/gateways/produce/tenant1/application1/produce"
    r = requests.post(url, data='{"value": "my-value"}', headers={"Content-Type": "application/json"}, timeout=30)
    assert r.status_code == 200 and r.json() == {"status": "OK", "reason": None}
    r = requests.post(url, data='{"key": "my-key", "value": "my-value", "headers": {"header1": "value1"}}',
                      headers={"Content-Type": "application/json"}, timeout=30)
    assert r.status_code == 200 and r.json()["status"] == "OK"
    r = requests.post(url, data="my-value", headers={"Content-Type": "text/plain"}, timeout=30)
    assert r.status_code == 200 and r.json()["status"] == "OK"


def test_send_events(gw):
    """ProduceConsumeHandlerTest.testSendEvents: ClientConnected / ClientDisconnected
    events on the gateways' events topic, the consumer's own connection first."""
    import aiohttp
    t, ev = _topic(), _topic()
    g = gw([t, ev], [{"id": "produce", "type": "produce", "topic": t, "parameters": ["p"], "events-topic": ev},
                     {"id": "consume", "type": "consume", "topic": ev, "parameters": ["p"], "events-topic": ev}])

    async def go():
        async with aiohttp.ClientSession() as s:
            c = await _Collector().start(s, f"{g.ws}/v1/consume/tenant1/application1/consume?param:p=consumer")
            await _produce(s, f"{g.ws}/v1/produce/tenant1/application1/produce?param:p=producer",
                           {"value": "this is a message"})
            other = await s.ws_connect(f"{g.ws}/v1/consume/tenant1/application1/consume?param:p=consumer1")
            await asyncio.sleep(0.3)
            await other.close()
            await c.wait(5)
            await c.close()
            return [json.loads(m["record"]["value"]) for m in c.msgs]
    events = _run(go())
    want = [("ClientConnected", "consume", "consumer"), ("ClientConnected", "produce", "producer"),
            ("ClientDisconnected", "produce", "producer"), ("ClientConnected", "consume", "consumer1"),
            ("ClientDisconnected", "consume", "consumer1")]
    assert [(e["type"], e["source"]["gateway"]["id"], e["data"]["userParameters"]["p"]) for e in events[:5]] == want
    for e in events[:5]:
        assert e["category"] == "Gateway" and e["timestamp"] > 0
        assert (e["source"]["tenant"], e["source"]["applicationId"]) == ("tenant1", "application1")
        assert e["data"]["options"] == {} and e["data"]["httpRequestHeaders"].get("host")


def test_filter_out_messages_by_param_value(gw):
    """ProduceConsumeHandlerTest.testFilterOutMessagesByParamValue: the producer stamps its
    session id as header1, each consumer sees only its own session's records (one from
    the earliest position, one from the latest)."""
    import aiohttp
    t = _topic()
    g = gw([t], [
        {"id": "produce", "type": "produce", "topic": t, "parameters": ["session-id"],
         "produce-options": {"headers": [{"key": "header1", "value-from-parameters": "session-id"}]}},
        {"id": "consume", "type": "consume", "topic": t, "parameters": ["session-id"],
         "consume-options": {"filters": {"headers": [{"key": "header1", "value-from-parameters": "session-id"}]}}}])

    async def go():
        async with aiohttp.ClientSession() as s:
            cons = f"{g.ws}/v1/consume/tenant1/application1/consume?param:session-id="
            prod = f"{g.ws}/v1/produce/tenant1/application1/produce?param:session-id="
            u1 = await _Collector().start(s, cons + "user1&option:position=earliest")
            u2 = await _Collector().start(s, cons + "user2")
            await _produce(s, prod + "user1", {"value": "this is a message for user1"})
            await u1.wait(1)
            assert u1.records() == [(None, "this is a message for user1", {"header1": "user1"})] and u2.msgs == []
            await _produce(s, prod + "user1", {"value": "this is a message for user1, again"})
            await u1.wait(2)
            assert [v for _, v, _ in u1.records()] == ["this is a message for user1",
                                                       "this is a message for user1, again"]
            assert u2.msgs == []
            await _produce(s, prod + "user2", {"value": "this is a message for user2"})
            await u2.wait(1)
            await asyncio.sleep(0.3)
            assert u2.records() == [(None, "this is a message for user2", {"header1": "user2"})]
            assert len(u1.msgs) == 2
            for c in (u1, u2):
                await c.close()
    _run(go())


class _TestAuth:
    """The Java suite's TestGatewayAuthenticationProvider (``test-auth``): credentials
    starting with ``test-user-password`` log in as themselves."""

    def __init__(self, configuration):
        pass

    def authenticate(self, ctx):
        from langstream_amd.gateway.auth import AuthResult
        c = ctx.credentials
        if c is not None and c.startswith("test-user-password"):
            return AuthResult(True, None, {"login": c})
        return AuthResult(False, "Invalid credentials")


def _auth_gateways(t, extra=()):
    auth = {"provider": "test-auth", "allow-test-mode": True}
    return [{"id": "produce", "type": "produce", "topic": t, "authentication": auth,
             "produce-options": {"headers": [{"key": "header1", "value-from-authentication": "login"}]}},
            {"id": "consume", "type": "consume", "topic": t, "authentication": auth,
             "consume-options": {"filters": {"headers": [{"key": "header1", "value-from-authentication": "login"}]}}},
            *extra]


def test_authentication(gw, monkeypatch):
    """ProduceConsumeHandlerTest.testAuthentication: 401 without / with bad credentials;
    the login becomes the produced header and the consumer's filter."""
    import aiohttp
    from langstream_amd.gateway import auth
    monkeypatch.setitem(auth.PROVIDERS, "test-auth", _TestAuth)
    t = _topic()
    g = gw([t], _auth_gateways(t))

    async def go():
        async with aiohttp.ClientSession() as s:
            prod = f"{g.ws}/v1/produce/tenant1/application1/produce"
            for q in ("", "?credentials=", "?credentials=error"):
                with pytest.raises(aiohttp.WSServerHandshakeError) as e:
                    await s.ws_connect(prod + q)
                assert e.value.status == 401
            ws = await s.ws_connect(prod + "?credentials=test-user-password")
            await ws.close()
            cons = f"{g.ws}/v1/consume/tenant1/application1/consume?option:position=earliest&credentials="
            u1 = await _Collector().start(s, cons + "test-user-password")
            u2 = await _Collector().start(s, cons + "test-user-password-2")
            r = await _produce(s, prod + "?credentials=test-user-password", {"value": "hello user"})
            assert r["status"] == "OK"
            await u1.wait(1)
            await asyncio.sleep(0.3)
            assert u1.records() == [(None, "hello user", {"header1": "test-user-password"})] and u2.msgs == []
            for c in (u1, u2):
                await c.close()
    _run(go())


def test_test_credentials(gw, monkeypatch):
    """ProduceConsumeHandlerTest.testTestCredentials: ``test-credentials`` go to the
    gateway's test-mode provider (an HTTP check here, as in the Java suite); the principal
    is the SHA-256 of the credentials; gateways without test mode and credentials the
    provider rejects get 401."""
    import aiohttp
    from ref_runtime_harness import FakeHTTP
    from langstream_amd.gateway import auth
    monkeypatch.setitem(auth.PROVIDERS, "test-auth", _TestAuth)
    fake = FakeHTTP()
    fake.stub("GET", "/auth/tenant1", text="", headers={"Authorization": "Bearer test-user-password", "h1": "v1"})
    t = _topic()
    no_test = {"id": "consume-no-test", "type": "consume", "topic": t,
               "authentication": {"provider": "test-auth", "allow-test-mode": False}}
    g = gw([t], _auth_gateways(t, [no_test]),
           test_auth=("http", {"base-url": fake.url, "path-template": "/auth/{tenant}", "headers": {"h1": "v1"}}))

    async def go():
        async with aiohttp.ClientSession() as s:
            u1 = await _Collector().start(
                s, f"{g.ws}/v1/consume/tenant1/application1/consume?test-credentials=test-user-password")
            r = await _produce(s, f"{g.ws}/v1/produce/tenant1/application1/produce?test-credentials=test-user-password",
                               {"value": "hello user"})
            assert r["status"] == "OK"
            await u1.wait(1)
            assert u1.records() == [(None, "hello user", {
                "header1": "9d75ff199d33e051209b59702de27d1e470eafb58ac6d8865788bf23b48e6818"})]
            await u1.close()
            for url in (f"{g.ws}/v1/consume/tenant1/application1/consume-no-test?test-credentials=test-user-password",
                        f"{g.ws}/v1/produce/tenant1/application1/produce?test-credentials=test-user-password-but-wrong"):
                with pytest.raises(aiohttp.WSServerHandshakeError) as e:
                    await s.ws_connect(url)
                assert e.value.status == 401
    try:
        _run(go())
    finally:
        fake.close()


def test_chat_gateway(gw):
    """ProduceConsumeHandlerTest.testChatGateway: questions and answers on one topic; a
    header comparison without a key is named after its parameter."""
    import aiohttp
    t = _topic()
    g = gw([t], [{"id": "chat", "type": "chat", "chat-options": {
        "questions-topic": t, "answers-topic": t, "headers": [{"value-from-parameters": "session"}]}}])

    async def go():
        async with aiohttp.ClientSession() as s:
            ws = await s.ws_connect(f"{g.ws}/v1/chat/tenant1/application1/chat?param:session=s1")
            await asyncio.sleep(0.3)
            await ws.send_str(json.dumps({"value": "this is a message"}))
            records = []
            for _ in range(4):
                m = json.loads((await ws.receive(timeout=10)).data)
                if "record" in m:
                    records.append((m["record"]["key"], m["record"]["value"], m["record"]["headers"]))
                    break
                assert m["status"] == "OK"      # the produce acknowledgement
            await ws.close()
            assert records == [(None, "this is a message", {"session": "s1"})]
    _run(go())


def test_http_service(gw):
    """GatewayResourceTest.testService: a service gateway writes the request to the input
    topic and answers with the record that comes back on the output topic (an echo
    exchange between the two topics here, as in the Java test), key / value / headers as
    sent plus the gateway's correlation header; 100 requests from 10 threads."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    from langstream_amd.api.topics import TopicConnectionsRuntimeRegistry
    tin, tout = _topic(), _topic()
    g = gw([tin, tout], [{"id": "svc", "type": "service",
                          "service-options": {"input-topic": tin, "output-topic": tout}}])
    sc = g.app.instance.streaming_cluster
    rt = TopicConnectionsRuntimeRegistry.get(sc)
    stop = threading.Event()

    def exchange():
        cons = rt.create_consumer("exchange", sc, {"topic": tin, "subscriptionName": "s"})
        prod = rt.create_producer("exchange", sc, {"topic": tout})
        cons.start()
        prod.start()
        try:
            while not stop.is_set():
                recs = cons.read()
                for r in recs:
                    prod.write(r).result(10)
                if recs:
                    cons.commit(recs)
        finally:
            cons.close()
            prod.close()
    th = threading.Thread(target=exchange, daemon=True)
    th.start()
    url = f"{g.http}/api/gateways/service/tenant1/application1/svc"

    def call(body, ctype="application/json"):
        r = requests.post(url, data=body, headers={"Content-Type": ctype}, timeout=60)
        assert r.status_code == 200, r.text
        rec = r.json()["record"]
        hs = dict(rec["headers"])
        assert hs.pop("langstream-service-request-id")      # the correlation header comes back
        return rec["key"], rec["value"], hs
    try:
        assert call('{"key": "my-key", "value": "my-value"}') == ("my-key", "my-value", {})
        assert call('{"key": "my-key2", "value": "my-value"}') == ("my-key2", "my-value", {})
        assert call("my-text", "text/plain") == (None, "my-text", {})
        assert call('{"key": "my-key2", "value": "my-value", "headers": {"header1": "value1"}}') == \
            ("my-key2", "my-value", {"header1": "value1"})
        with ThreadPoolExecutor(10) as ex:
            outs = list(ex.map(lambda _: call('{"key": "my-key", "value": "my-value"}'), range(100)))
        assert outs == [("my-key", "my-value", {})] * 100
    finally:
        stop.set()
        th.join(10)


def test_producer_cache_eviction_keeps_sessions_working():
    """LRUTopicProducerCacheTest (testGetOrCreate / testConcurrency): producers are shared
    per key, at most ``size`` stay cached, and an evicted producer still serves the
    sessions holding it -- it closes when idle and reopens for a later write."""
    import threading
    from concurrent.futures import Future, ThreadPoolExecutor
    from langstream_amd.gateway.server import _ProducerCache
    opened, closed = [], []

    class P:
        def __init__(self):
            self.closed = False
            opened.append(self)

        def write(self, rec):
            assert not self.closed, "write on a closed producer"
            f = Future()
            f.set_result(None)
            return f

        def close(self):
            self.closed = True
            closed.append(self)
    cache = _ProducerCache(2)
    first = cache.get_or_create(("t", "a", "g"), P)
    assert cache.get_or_create(("t", "a", "g"), P) is first and len(opened) == 1
    second = cache.get_or_create(("t", "a", "g2"), P)
    assert len(opened) == 2 and not closed
    cache.get_or_create(("t", "a", "g3"), P)             # evicts "g" (idle): closed now
    assert len(opened) == 3 and len(closed) == 1 and first.closed
    first.write("x").result(1)                           # a session still holding it: reopened
    assert len(opened) == 4 and len(closed) == 2 and first.closed   # ... and closed once idle
    assert cache.get_or_create(("t", "a", "g"), P) is not first and len(cache._d) == 2
    assert second.closed and len(closed) == 3          # "g2" was evicted in turn

    cache = _ProducerCache(2)
    errors = []

    def worker(i):
        try:
            for j in range(50):
                cache.get_or_create(("t", "a", f"g{(i + j) % 5}"), P).write(j).result(1)
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    with ThreadPoolExecutor(50) as ex:
        list(ex.map(worker, range(50)))
    assert not errors and len(cache._d) == 2
    _ = threading


def test_service_agent(tmp_path):
    """ServiceAgentGatewayResourceTest.testServiceAgent: a service gateway naming an agent
    proxies method, path, query, headers and body to the agent's service endpoint."""
    from ref_runtime_harness import FakeHTTP
    fake = FakeHTTP()
    fake.stub("POST", "/agent-endpoint/custom-path", text="agent response")
    fake.stub("POST", "/agent-endpoint/custom-path-json?q=v", text="agent response",
              headers={"X-Custom-Header": "XXX", "Content-Type": "application/json"})
    fake.stub("POST", "/", body="hello", text="agent response ROOT")
    for m in ("GET", "PUT", "DELETE"):
        fake.stub(m, "/", text="agent response ROOT")
    g = GW([], [{"id": "svc", "type": "service", "service-options": {"agent-id": "my-agent"}}],
           resolver=lambda tenant, app, agent: fake.url)
    try:
        url = f"{g.http}/api/gateways/service/tenant1/application1/svc"
        r = requests.post(url, data="hello", headers={"Content-Type": "text/plain"}, timeout=30)
        assert (r.status_code, r.text) == (200, "agent response ROOT")
        for m in ("GET", "PUT", "DELETE"):
            r = requests.request(m, url, data="hello", headers={"Content-Type": "text/plain"}, timeout=30)
            assert (r.status_code, r.text) == (200, "agent response ROOT")
        r = requests.post(url + "/not-found", data="hello", headers={"Content-Type": "text/plain"}, timeout=30)
        assert r.status_code == 404
        r = requests.post(url + "/agent-endpoint/custom-path", data="hello",
                          headers={"Content-Type": "text/plain"}, timeout=30)
        assert (r.status_code, r.text) == (200, "agent response")
        r = requests.post(url + "/agent-endpoint/custom-path-json?q=v", data="hello",
                          headers={"Content-Type": "application/json", "X-Custom-Header": "XXX"}, timeout=30)
        assert (r.status_code, r.text) == (200, "agent response")
    finally:
        g.close()
        fake.close()


def test_concurrent_consume(gw):
    """ProduceConsumeHandlerTest.testConcurrentConsume: 50 consumers from the earliest
    position each get every record, in order."""
    import aiohttp
    t = _topic()
    g = gw([t], [{"id": "produce", "type": "produce", "topic": t}, {"id": "consume", "type": "consume", "topic": t}])

    async def go():
        async with aiohttp.ClientSession() as s:
            cons = f"{g.ws}/v1/consume/tenant1/application1/consume?option:position=earliest"
            clients = [await _Collector().start(s, cons, settle=False) for _ in range(50)]
            await asyncio.sleep(0.5)
            prod = f"{g.ws}/v1/produce/tenant1/application1/produce"
            await _produce(s, prod, {"value": "msg1"})
            for c in clients:
                await c.wait(1)
                assert c.records() == [(None, "msg1", {})]
            await _produce(s, prod, {"value": "msg2"})
            for c in clients:
                await c.wait(2)
                assert c.records() == [(None, "msg1", {}), (None, "msg2", {})]
            for c in clients:
                await c.close()
    _run(go())
