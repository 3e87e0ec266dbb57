"""``langstream apps ui <app>`` -- a local web UI for one application
(``langstream-cli/.../applications/UIAppCmd.java``).

A small aiohttp server (default port 8092) that serves:
* ``/`` -- the single-page UI (``app_ui_static/index.html``): the application's gateways
  (produce / consume / chat / service forms talking WebSocket), its pipeline diagram
  (Mermaid text) and a live log panel;
* ``/api/application`` -- the app model the page renders: ``baseUrl`` (this server, as
  ``ws://``), ``remoteBaseUrl`` (the profile's API gateway), ``tenant``,
  ``applicationId``, ``gateways``, ``applicationDefinition`` (the control plane's
  description, JSON text) and ``mermaidDefinition``;
* ``/api/logs`` -- the application's logs from the control plane as a text stream;
* ``/v1/**`` -- a proxy to the API gateway (WebSocket upgrades pumped both ways, plain
  HTTP forwarded), so the page talks to one origin like the reference's Undertow proxy.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import threading
from typing import Any, Dict, Optional

log = logging.getLogger(__name__)

_STATIC = os.path.join(os.path.dirname(__file__), "app_ui_static")


def mermaid_from_plan(plan: Dict[str, Any]) -> str:
    """Mermaid flowchart of an execution-plan dict (the description's ``application``)."""
    lines = ["flowchart LR"]
    ids: Dict[str, str] = {}

    def nid(s: str) -> str:
        return ids.setdefault(s, f"n{len(ids)}")

    for t in plan.get("topics") or []:
        lines.append(f'  {nid("topic:" + t["name"])}(["{t["name"]}"])')
    for node in (plan.get("agents") or {}).values():
        cfg = node.get("configuration") or {}
        steps = [p.get("agentId") for p in cfg.get("processors", [])] if node.get("agent-type") == "composite-agent" \
            else [node.get("id")]
        lines.append(f'  {nid("agent:" + node["id"])}["{"<br/>".join(map(str, steps))}<br/>'
                     f'<i>{node.get("agent-type")}</i>"]')
        if node.get("input"):
            lines.append(f'  {nid("topic:" + node["input"])} --> {nid("agent:" + node["id"])}')
        if node.get("output"):
            lines.append(f'  {nid("agent:" + node["id"])} --> {nid("topic:" + node["output"])}')
    for g in plan.get("gateways") or []:
        gid = nid("gateway:" + str(g.get("id")))
        lines.append(f'  {gid}{{{{"{g.get("id")}<br/><i>{g.get("type")} gateway</i>"}}}}')
        chat = g.get("chat-options") or {}
        if g.get("type") == "chat":
            if chat.get("questions-topic"):
                lines.append(f'  {gid} --> {nid("topic:" + chat["questions-topic"])}')
            if chat.get("answers-topic"):
                lines.append(f'  {nid("topic:" + chat["answers-topic"])} --> {gid}')
        elif g.get("topic"):
            if g.get("type") == "consume":
                lines.append(f'  {nid("topic:" + g["topic"])} --> {gid}')
            else:
                lines.append(f'  {gid} --> {nid("topic:" + g["topic"])}')
    return "\n".join(lines)


_AI_CONFIGS = ("vertex-configuration", "open-ai-configuration", "hugging-face-configuration",
               "bedrock-configuration", "ollama-configuration")


def mermaid_from_description(desc: Dict[str, Any]) -> str:
    """Mermaid flowchart of an application DESCRIPTION (the control plane's ``apps get``
    JSON: ``application.{resources, modules[].topics / pipelines[].agents, gateways}``),
    laid out as ``MermaidAppDiagramGenerator.java:37-504`` lays it out: external systems,
    then Resources / Topics / Gateways / one subgraph per pipeline, then the links --
    agent inputs (dotted, green), gateway topics, client -> gateways, agent outputs (to a
    topic / external sink / lone resource: yellow; agent to agent: blue; to a resource
    beside another output: dotted blue)."""
    app = desc.get("application") or {}

    def rid(kind: str, name: str) -> str:
        return f"{kind}-" + str(name).replace(" ", "___").lower()

    gateways = []
    for g in (app.get("gateways") or {}).get("gateways") or []:
        prod, cons = [], []
        chat = g.get("chat-options")
        if chat is not None:
            if chat.get("questions-topic") is not None:
                prod.append(rid("topic", chat["questions-topic"]))
            if chat.get("answers-topic") is not None:
                cons.append(rid("topic", chat["answers-topic"]))
        elif g.get("topic") is not None:
            (prod if g.get("type") == "produce" else cons).append(rid("topic", g["topic"]))
        gateways.append((rid("gateway", g.get("id")), g.get("id"), prod, cons))
    resources = [(k, r.get("name"), r.get("type")) for k, r in (app.get("resources") or {}).items()]
    topics, pipelines, ext_src, ext_sink = [], [], [], []
    for mod in app.get("modules") or []:
        topics += [(rid("topic", t.get("name")), t.get("name")) for t in mod.get("topics") or []]
        for p in mod.get("pipelines") or []:
            agents = []
            for a in p.get("agents") or []:
                aid = rid("agent", a.get("id"))
                inp = a.get("input")
                if inp is None:
                    src = "external-source-" + aid
                    ext_src.append(src)
                    inp_id = src
                else:
                    inp_id = rid("topic", inp.get("definition")) if inp.get("connectionType") == "TOPIC" else None
                outs = []
                out = a.get("output")
                if out is None:
                    ext_sink.append("external-sink-" + aid)
                    outs.append("external-sink-" + aid)
                else:
                    outs.append(rid("topic" if out.get("connectionType") == "TOPIC" else "agent", out.get("definition")))
                cfg = a.get("configuration") or {}
                if isinstance(cfg.get("datasource"), str):
                    outs.append(rid("resource", cfg["datasource"]))
                if isinstance(cfg.get("stream-to-topic"), str):
                    outs.append(rid("topic", cfg["stream-to-topic"]))
                if a.get("type") in ("ai-text-completions", "ai-chat-completions", "compute-ai-embeddings"):
                    if "ai-service" in cfg:
                        outs.append(rid("resource", cfg["ai-service"]))
                    else:
                        svc = next((r for r in resources if r[2] in _AI_CONFIGS), None)
                        if svc is not None:
                            outs.append(rid("resource", svc[0]))
                agents.append((aid, a.get("name"), inp_id, outs))
            pipelines.append((p.get("id"), agents))

    m = ["flowchart LR", ""]
    if gateways:
        m += ["external-client((Client))", ""]
    for e in list(dict.fromkeys(ext_sink)) + list(dict.fromkeys(ext_src)):
        m += [f'{e}(["External system"])', ""]
    m.append('subgraph resources["Resources"]')
    for k, name, typ in resources:
        m.append(rid("resource", k) + (f'[("{name}")]' if typ == "datasource" else f'("{name}")'))
    m += ["end", "", 'subgraph streaming-cluster["Topics"]']
    m += [f'{t}(["{label}"])' for t, label in topics]
    m += ["end", "", 'subgraph gateways["Gateways"]']
    m += [f'{g}[/"{label}"\\]' for g, label, _, _ in gateways]
    m += ["end", ""]
    for pid, agents in pipelines:
        m.append(f'subgraph pipeline-{pid}["Pipeline: <b>{pid}</b>"]')
        m += [f'{aid}("{label}")' for aid, label, _, _ in agents]
        m += ["end", ""]
    n = 0

    def link(a: str, b: str, dotted: bool, style: Optional[str]) -> None:
        nonlocal n
        m.append(a + ("-.->" if dotted else "-->") + b)
        if style:
            m.append(f"linkStyle {n} {style}")
        n += 1

    for _, agents in pipelines:
        for aid, _, inp, _ in agents:
            if inp is not None:
                link(aid, inp, True, "stroke:#82E0AA")
    for g, _, prod, cons in gateways:
        for t in cons:
            link(g, t, True, None)
        for t in prod:
            link(g, t, False, None)
    link("external-client", "gateways", False, None)
    for _, agents in pipelines:
        for aid, _, _, outs in agents:
            ends = [o for o in outs if o.startswith(("topic-", "external-sink-"))]
            for o in outs:
                if o in ends or (not ends and o.startswith("resource-")):
                    link(aid, o, False, "stroke:#F4D03F")
                else:
                    link(aid, o, o.startswith("resource-"), "stroke:#5DADE2")
    return "\n".join(m) + "\n"


def app_model(client, app_id: str, api_gateway_url: str, tenant: str) -> Dict[str, Any]:
    desc = client.get(app_id)
    plan = desc.get("application") or {}
    gws = plan.get("gateways") or []
    if isinstance(gws, dict):   # the reference description: {"gateways": [...]}
        gws = gws.get("gateways") or []
    return {"remoteBaseUrl": api_gateway_url, "tenant": tenant, "applicationId": app_id,
            "gateways": gws,
            "applicationDefinition": json.dumps(desc, default=str),
            "mermaidDefinition": mermaid_from_description(desc) if "modules" in plan else mermaid_from_plan(plan)}


def make_app(client, app_id: str, api_gateway_url: str, tenant: str):
    import aiohttp
    from aiohttp import web

    gw_ws = api_gateway_url.rstrip("/")
    gw_http = gw_ws.replace("wss://", "https://", 1).replace("ws://", "http://", 1)

    async def index(request):
        return web.FileResponse(os.path.join(_STATIC, "index.html"))

    async def application(request):
        model = await asyncio.get_running_loop().run_in_executor(
            None, app_model, client, app_id, api_gateway_url, tenant)
        model["baseUrl"] = f"ws://{request.host}"
        return web.json_response(model)

    async def logs(request):
        resp = web.StreamResponse(headers={"Content-Type": "text/plain; charset=utf-8"})
        await resp.prepare(request)
        loop = asyncio.get_running_loop()
        q: "asyncio.Queue[Optional[str]]" = asyncio.Queue()
        follow = request.query.get("follow", "true") != "false"

        def pump():
            try:
                for rec in client.logs(app_id, follow=follow):
                    line = f"[{rec.get('replica')}] {rec.get('level')} {rec.get('message')}"
                    loop.call_soon_threadsafe(q.put_nowait, line)
            except Exception as e:  # noqa: BLE001 - the stream ended or failed
                loop.call_soon_threadsafe(q.put_nowait, f"-- logs unavailable: {e}")
            loop.call_soon_threadsafe(q.put_nowait, None)

        threading.Thread(target=pump, daemon=True, name="app-ui-logs").start()
        try:
            while True:
                line = await q.get()
                if line is None:
                    break
                await resp.write((line + "\n").encode())
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        return resp

    async def proxy(request):
        tail = request.match_info["tail"]
        qs = ("?" + request.query_string) if request.query_string else ""
        if request.headers.get("Upgrade", "").lower() == "websocket":
            down = web.WebSocketResponse()
            await down.prepare(request)
            async with aiohttp.ClientSession() as s:
                try:
                    up = await s.ws_connect(f"{gw_ws}/v1/{tail}{qs}")
                except aiohttp.ClientError as e:
                    await down.close(code=1011, message=str(e).encode()[:120])
                    return down

                async def up_to_down():
                    async for m in up:
                        if m.type == aiohttp.WSMsgType.TEXT:
                            await down.send_str(m.data)
                        elif m.type == aiohttp.WSMsgType.BINARY:
                            await down.send_bytes(m.data)
                        else:
                            break
                    await down.close()

                t = asyncio.ensure_future(up_to_down())
                async for m in down:
                    if m.type == aiohttp.WSMsgType.TEXT:
                        await up.send_str(m.data)
                    elif m.type == aiohttp.WSMsgType.BINARY:
                        await up.send_bytes(m.data)
                    else:
                        break
                await up.close()
                t.cancel()
            return down
        async with aiohttp.ClientSession() as s:
            body = await request.read()
            async with s.request(request.method, f"{gw_http}/v1/{tail}{qs}", data=body or None,
                                 headers={k: v for k, v in request.headers.items()
                                          if k.lower() in ("content-type", "authorization")}) as r:
                return web.Response(status=r.status, body=await r.read(),
                                    content_type=r.content_type or "application/octet-stream")

    app = web.Application()
    app.router.add_get("/", index)
    app.router.add_get("/index.html", index)
    app.router.add_get("/api/application", application)
    app.router.add_get("/api/logs", logs)
    app.router.add_route("*", "/v1/{tail:.*}", proxy)
    return app


class AppUIServer:
    def __init__(self, client, app_id: str, api_gateway_url: str, tenant: str, host: str = "127.0.0.1",
                 port: int = 8092):
        self.args = (client, app_id, api_gateway_url, tenant)
        self.host, self.port = host, port
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._ready = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def start(self) -> "AppUIServer":
        from aiohttp import web

        def run():
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._runner = web.AppRunner(make_app(*self.args))
            self._loop.run_until_complete(self._runner.setup())
            site = web.TCPSite(self._runner, self.host, self.port)
            self._loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            self._ready.set()
            self._loop.run_forever()

        self._thread = threading.Thread(target=run, daemon=True, name="app-ui")
        self._thread.start()
        if not self._ready.wait(15):
            raise RuntimeError("app UI server did not start")
        return self

    @property
    def url(self) -> str:
        return f"http://{'localhost' if self.host in ('0.0.0.0', '127.0.0.1') else self.host}:{self.port}"

    def stop(self) -> None:
        if self._loop is None:
            return
        fut = asyncio.run_coroutine_threadsafe(self._runner.cleanup(), self._loop)
        try:
            fut.result(10)
        except Exception:  # noqa: BLE001
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(10)


def check_and_launch(open_command: str, port: int) -> bool:
    """``UIAppCmd.checkAndLaunch``: run ``<open_command> http://localhost:<port>`` when the
    command exists on disk; False when it does not or cannot start."""
    import subprocess
    if not os.path.exists(open_command):
        return False
    try:
        subprocess.Popen([open_command, f"http://localhost:{port}"], stdout=subprocess.DEVNULL,
                         stderr=subprocess.DEVNULL, start_new_session=True)
        return True
    except OSError:
        return False


def open_browser_at_port(port: int) -> bool:
    """``UIAppCmd.openBrowserAtPort``: xdg-open on Linux, the platform browser elsewhere."""
    import sys
    if sys.platform.startswith("linux"):
        return check_and_launch("/usr/bin/xdg-open", port)
    try:
        import webbrowser
        return bool(webbrowser.open(f"http://localhost:{port}"))
    except Exception:  # noqa: BLE001
        return False


def serve_forever(client, app_id: str, api_gateway_url: str, tenant: str, port: int = 8092,
                  open_browser: bool = True) -> int:
    client.get(app_id)                      # fail fast: the application must exist
    srv = AppUIServer(client, app_id, api_gateway_url, tenant, host="0.0.0.0", port=port).start()
    if open_browser and open_browser_at_port(srv.port):
        print(f"Started UI at http://localhost:{srv.port}", flush=True)
    else:
        print("Could not Start browser.  Either add the proper command to your OS (open for mac or xdg-open for "
              f"linux) or start a browser manually at http://localhost:{srv.port}", flush=True)
    stop = threading.Event()
    try:
        import signal
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
    except ValueError:
        pass
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    srv.stop()
    return 0
