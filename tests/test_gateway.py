"""API gateway over a running local application (memory topics), aiohttp clients.

Mirrors the reference's gateway tests (ProduceConsumeHandlerTest, ChatHandlerTest,
GatewayResourceTest): produce/consume round trip with header filters from parameters,
chat through a pipeline, HTTP produce, service request/response over topics,
parameter validation, JWT authentication and test mode, events topic."""
import asyncio
import json
import uuid

import pytest

from langstream_amd.core.store import InMemoryApplicationStore, StoredApplication
from langstream_amd.gateway.auth import encode_jwt_hs256
from langstream_amd.gateway.server import GatewayServer, GatewayService
from langstream_amd.runtime.local import LocalApplicationRunner
from langstream_amd.topics.memory import reset_memlogs

PIPE = """
topics:
  - name: "questions"
    creation-mode: create-if-not-exists
  - name: "answers"
    creation-mode: create-if-not-exists
  - name: "events"
    creation-mode: create-if-not-exists
pipeline:
  - name: "answer"
    type: "compute"
    input: "questions"
    output: "answers"
    configuration:
      fields:
        - name: "value"
          expression: "fn:concat('echo: ', value)"
"""

GATEWAYS = """
gateways:
  - id: produce-q
    type: produce
    topic: questions
    parameters: [sessionId]
    events-topic: events
    produce-options:
      headers:
        - key: session
          value-from-parameters: sessionId
  - id: consume-a
    type: consume
    topic: answers
    parameters: [sessionId]
    consume-options:
      filters:
        headers:
          - key: session
            value-from-parameters: sessionId
  - id: chat
    type: chat
    chat-options:
      questions-topic: questions
      answers-topic: answers
      headers:
        - key: session
          value-from-parameters: sessionId
  - id: secure
    type: produce
    topic: questions
    authentication:
      provider: jwt
      allow-test-mode: true
      configuration:
        secret-key: "s3cr3t"
    produce-options:
      headers:
        - key: user
          value-from-authentication: subject
  - id: svc
    type: service
    service-options:
      input-topic: questions
      output-topic: answers
"""


@pytest.fixture(scope="module")
def env():
    reset_memlogs()
    files = {"pipeline.yaml": PIPE, "gateways.yaml": GATEWAYS}
    runner = LocalApplicationRunner.from_yaml(files, application_id="app1").start()
    store = InMemoryApplicationStore()
    store.put(StoredApplication("app1", "default", runner.application, files))
    gw = GatewayServer(GatewayService(store, test_auth=("jwt", {"secret-key": "testkey"})), port=0).start()
    yield runner, gw
    gw.stop()
    runner.stop(5)
    reset_memlogs()


def _run(coro):
    return asyncio.new_event_loop().run_until_complete(coro)


def test_produce_consume_with_session_filter(env):
    import aiohttp
    _, gw = env
    base = gw.url.replace("http", "ws")

    async def go():
        async with aiohttp.ClientSession() as s:
            c1 = await s.ws_connect(f"{base}/v1/consume/default/app1/consume-a?param:sessionId=s1")
            c2 = await s.ws_connect(f"{base}/v1/consume/default/app1/consume-a?param:sessionId=s2")
            p = await s.ws_connect(f"{base}/v1/produce/default/app1/produce-q?param:sessionId=s1")
            await asyncio.sleep(0.3)
            await p.send_str(json.dumps({"value": "hi"}))
            ack = json.loads((await p.receive()).data)
            assert ack["status"] == "OK"
            msg = json.loads((await c1.receive(timeout=10)).data)
            assert msg["record"]["value"] == "echo: hi"
            assert msg["record"]["headers"]["session"] == "s1"
            assert msg["offset"]
            with pytest.raises(asyncio.TimeoutError):
                await c2.receive(timeout=1.0)  # filtered out: other session
            # client may not override a configured header
            await p.send_str(json.dumps({"value": "x", "headers": {"session": "evil"}}))
            assert json.loads((await p.receive()).data)["status"] == "BAD_REQUEST"
            await p.send_str("not json")
            assert json.loads((await p.receive()).data)["status"] == "BAD_REQUEST"
            for w in (c1, c2, p):
                await w.close()
    _run(go())


def test_chat(env):
    import aiohttp
    _, gw = env
    base = gw.url.replace("http", "ws")

    async def go():
        async with aiohttp.ClientSession() as s:
            ws = await s.ws_connect(f"{base}/v1/chat/default/app1/chat?param:sessionId=abc")
            await asyncio.sleep(0.3)
            await ws.send_str(json.dumps({"value": "question?"}))
            ack = json.loads((await ws.receive(timeout=10)).data)
            assert ack["status"] == "OK"
            ans = json.loads((await ws.receive(timeout=10)).data)
            assert ans["record"]["value"] == "echo: question?"
            await ws.close()
    _run(go())


def test_chat_sessions_share_one_routed_reader(env):
    """Concurrent chat sessions of one gateway share one answers-topic reader (the hub),
    each still sees only its own answers, and the hub goes away with the last session."""
    import aiohttp
    _, gw = env
    base = gw.url.replace("http", "ws")
    sids = [f"hub{i}" for i in range(6)]

    async def one(s, sid):
        ws = await s.ws_connect(f"{base}/v1/chat/default/app1/chat?param:sessionId={sid}")
        await asyncio.sleep(0.3)
        got = []
        for q in range(3):
            await ws.send_str(json.dumps({"value": f"{sid}-q{q}"}))
            while True:
                m = json.loads((await ws.receive(timeout=10)).data)
                if "record" in m:
                    got.append(m["record"]["value"])
                    break
        return ws, got

    async def go():
        async with aiohttp.ClientSession() as s:
            res = await asyncio.gather(*[one(s, sid) for sid in sids])
            assert len(gw._hubs) == 1
            hub = next(iter(gw._hubs.values()))
            assert len(hub.subs) == len(sids)
            for sid, (ws, got) in zip(sids, res):
                assert got == [f"echo: {sid}-q{q}" for q in range(3)]
            for ws, _ in res:
                await ws.close()
            for _ in range(50):
                if not gw._hubs:
                    break
                await asyncio.sleep(0.05)
            assert not gw._hubs
    _run(go())


def test_validation_errors(env):
    import aiohttp
    _, gw = env

    async def go():
        async with aiohttp.ClientSession() as s:
            for q, code in (("", 400), ("?param:sessionId=1&param:x=2", 400), ("?bad=1", 400)):
                with pytest.raises(aiohttp.WSServerHandshakeError) as ei:
                    await s.ws_connect(f"{gw.url.replace('http', 'ws')}/v1/produce/default/app1/produce-q{q}")
                assert ei.value.status == code
            with pytest.raises(aiohttp.WSServerHandshakeError) as ei:
                await s.ws_connect(f"{gw.url.replace('http', 'ws')}/v1/produce/default/nope/produce-q")
            assert ei.value.status == 404
    _run(go())


def test_http_produce_auth_and_events(env):
    import aiohttp
    runner, gw = env

    async def go():
        async with aiohttp.ClientSession() as s:
            url = f"{gw.url}/api/gateways/produce/default/app1/secure"
            r = await s.post(url, data="no auth")
            assert r.status == 401
            tok = encode_jwt_hs256({"sub": "alice", "exp": 9999999999}, b"s3cr3t")
            r = await s.post(url + f"?credentials={tok}", data="with auth")
            assert r.status == 200 and (await r.json())["status"] == "OK"
            bad = encode_jwt_hs256({"sub": "alice"}, b"wrong")
            r = await s.post(url + f"?credentials={bad}", data="x")
            assert r.status == 401
            # test mode: credentials validated by the gateway's test provider
            ttok = encode_jwt_hs256({"sub": "t"}, b"testkey")
            r = await s.post(url + f"?test-credentials={ttok}", data="test mode")
            assert r.status == 200
            # connect/disconnect events come from WebSocket sessions on a gateway with an
            # events-topic (independent of which other tests ran first)
            ws = await s.ws_connect(gw.url.replace("http", "ws")
                                    + "/v1/produce/default/app1/produce-q?param:sessionId=ev")
            await ws.close()
    _run(go())
    recs = runner.consume("questions", 10, timeout=5)
    users = {r.value(): r.header_value("user") for r in recs}
    assert users.get("with auth") == "alice"
    assert users.get("test mode") and users["test mode"] != "t"  # sha256-derived principal
    ev = [json.loads(r.value()) for r in runner.consume("events", 2, timeout=5)]
    assert {e["type"] for e in ev} >= {"ClientConnected"}


def test_service_over_topics(env):
    import aiohttp
    _, gw = env

    async def go():
        async with aiohttp.ClientSession() as s:
            r = await s.post(f"{gw.url}/api/gateways/service/default/app1/svc", json={"value": "ping"})
            assert r.status == 200
            body = await r.json()
            assert body["record"]["value"] == "echo: ping"
            assert body["record"]["headers"]["langstream-service-request-id"]
    _run(go())
