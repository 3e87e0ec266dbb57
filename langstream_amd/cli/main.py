"""``langstream`` command line (``langstream-cli/.../commands/**``).

    python -m langstream_amd.cli <group> <command> ...

Groups:
* ``profiles``  list | get | get-current | create | update | import | delete | set-current
  (~/.langstream/config.yaml: webServiceUrl, apiGatewayUrl, tenant, token)
* ``configure`` <webServiceUrl|apiGatewayUrl|tenant|token> <value>  (the default profile)
* ``tenants``   list | get | create | update | put | delete
* ``apps``      deploy | update | get | list | delete | logs | download | diagram | ui
* ``gateway``   produce | consume | chat  (WebSocket client; chat re-assembles streamed
  answers from ``stream-id`` / ``stream-index`` / ``stream-last-message`` headers,
  ``ChatGatewayCmd.java:45-120``)
* ``run`` / ``docker run``  the ``docker run`` equivalent (``LocalRunApplicationCmd.java``):
  the bundled broker / S3 / database services (``--start-broker/-s3/-database``), control
  plane (8090), gateway (8091), agent control API (8790) and the UI (``-up`` 8092)
  in-process, ``--only-agent``, ``--watch-files`` hot reload, and the local GPU services
* app / instance / secrets paths may be ``file://``, ``https://`` or GitHub URLs (sources.py)
* ``archetypes`` list | get | deploy
* ``python``    load-pip-requirements | run-tests
* ``code-download`` (k8s init container: fetch + unzip the app code archive)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time
from typing import Any, Dict, List, Optional

CONFIG = os.path.expanduser(os.environ.get("LANGSTREAM_CLI_CONFIG", "~/.langstream/config.yaml"))
DEFAULT_PROFILE = {"webServiceUrl": "http://localhost:8090", "apiGatewayUrl": "ws://localhost:8091",
                   "tenant": "default", "token": None}
DEFAULT_PROFILE_NAME = "default"
_PROFILE_KEYS = ("webServiceUrl", "apiGatewayUrl", "tenant", "token")


class CliError(Exception):
    """A command failure reported as its message alone, exit code 1 (LangStreamCLI.execute)."""


# ---------------------------------------------------------------- profiles
def load_config() -> Dict[str, Any]:
    """The CLI config file in the reference's layout (LangStreamCLIConfig): the default
    profile's keys at the top level, named profiles under ``profiles``, ``currentProfile``.
    A ``profiles.default`` entry written by earlier versions moves to the top level."""
    import yaml
    if os.path.exists(CONFIG):
        with open(CONFIG) as f:
            c = yaml.safe_load(f) or {}
    else:
        c = {}
    c["profiles"] = dict(c.get("profiles") or {})
    old = c["profiles"].pop(DEFAULT_PROFILE_NAME, None)
    if isinstance(old, dict):
        for k in _PROFILE_KEYS:
            if c.get(k) is None and old.get(k) is not None:
                c[k] = old[k]
    for name, prof in c["profiles"].items():
        prof["name"] = name
    c.setdefault("currentProfile", DEFAULT_PROFILE_NAME)
    return c


def save_config(c: Dict[str, Any]) -> None:
    import yaml
    os.makedirs(os.path.dirname(CONFIG) or ".", exist_ok=True)
    out = {k: c.get(k) for k in _PROFILE_KEYS if c.get(k) is not None}
    out["profiles"] = {n: {k: v for k, v in p.items() if v is not None} for n, p in sorted(c["profiles"].items())}
    out["currentProfile"] = c.get("currentProfile", DEFAULT_PROFILE_NAME)
    with open(CONFIG, "w") as f:
        yaml.safe_dump(out, f, sort_keys=False)


def default_profile(c: Dict[str, Any]) -> Dict[str, Any]:
    """BaseCmd.getDefaultProfile: the top-level keys with the local defaults filled in."""
    return {"webServiceUrl": c.get("webServiceUrl") or DEFAULT_PROFILE["webServiceUrl"],
            "apiGatewayUrl": c.get("apiGatewayUrl") or DEFAULT_PROFILE["apiGatewayUrl"],
            "tenant": c.get("tenant") or DEFAULT_PROFILE["tenant"], "token": c.get("token"),
            "name": DEFAULT_PROFILE_NAME}


def named_profile(c: Dict[str, Any], name: str) -> Optional[Dict[str, Any]]:
    if name == DEFAULT_PROFILE_NAME:
        return default_profile(c)
    p = c["profiles"].get(name)
    if p is None:
        return None
    return {"webServiceUrl": p.get("webServiceUrl"), "apiGatewayUrl": p.get("apiGatewayUrl"),
            "tenant": p.get("tenant"), "token": p.get("token"), "name": name}


def current_profile(args) -> Dict[str, Any]:
    """BaseCmd.getCurrentProfile: ``-p`` / ``--profile``, else the current one; the
    LANGSTREAM_<key> environment variables override it (overrideFromEnv)."""
    c = load_config()
    name = getattr(args, "profile", None) or c.get("currentProfile", DEFAULT_PROFILE_NAME)
    p = named_profile(c, name)
    if p is None:
        raise CliError(f"No profile '{name}' defined in configuration")
    for k in _PROFILE_KEYS:
        v = os.environ.get(f"LANGSTREAM_{k}")
        if v is not None:
            p[k] = v
    if getattr(args, "tenant", None):
        p["tenant"] = args.tenant
    return p


def _client(args):
    from .client import AdminClient
    p = current_profile(args)
    if not p.get("webServiceUrl"):
        raise CliError(f"No webServiceUrl defined for profile '{p.get('name')}'")
    return AdminClient(p["webServiceUrl"], p.get("tenant"), p.get("token"))


def _tenant_client(args):
    cl = _client(args)
    if not cl.tenant:
        raise CliError("Tenant not set. Please set the tenant in the configuration.")
    return cl


def _print(obj, fmt: str = "json") -> None:
    from .printer import jackson_json, jackson_yaml
    print(jackson_yaml(obj) if fmt == "yaml" else jackson_json(obj))


def _validate_profile(p: Dict[str, Any]) -> None:
    """BaseProfileCmd.validateProfile."""
    if not str(p.get("webServiceUrl") or "").strip():
        raise CliError("webServiceUrl is required")


PROFILE_COLUMNS = ("profile", "webServiceUrl", "tenant", "token", "current")


def _profile_cell(c: Dict[str, Any]):
    """ListProfileCmd.rawMapping: the token masked, ``*`` on the current profile."""
    def value(p, col):
        if col == "profile":
            return p.get("name")
        if col == "token":
            return None if p.get("token") is None else "********"
        if col == "current":
            return "*" if p.get("name") == c.get("currentProfile") else ""
        return p.get(col)
    return value


def _profile_not_found(c: Dict[str, Any], name: str) -> CliError:
    names = [DEFAULT_PROFILE_NAME] + list(c["profiles"])
    return CliError(f"Profile {name} not found, maybe you meant one of these: {', '.join(names)}")


def _check_formats(fmt: str, allowed) -> None:
    if fmt not in allowed:
        raise CliError(f"Format {fmt} is not allowed. Allowed formats are: {', '.join(allowed)}")


def cmd_profiles(args) -> int:
    """``profiles`` (commands/profiles/*.java): messages, errors and output formats as the
    reference CLI prints them; the default profile lives in the config's top-level keys."""
    from .printer import render
    if getattr(args, "profile", None):
        raise CliError("Global profile flag is not allowed for profiles commands")
    c = load_config()
    if args.cmd in ("list", "get"):
        fmt = args.output or "raw"
        _check_formats(fmt, ("raw", "json", "yaml"))
        if args.cmd == "get":
            prof = named_profile(c, args.name)
            if prof is None:
                raise _profile_not_found(c, args.name)
            body: Any = [prof] if fmt == "raw" else prof
        else:
            profs = [default_profile(c)] + [named_profile(c, n) for n in c["profiles"]]
            body = profs if fmt == "raw" else {
                **{k: c.get(k) for k in _PROFILE_KEYS}, "profiles": {n: named_profile(c, n) for n in c["profiles"]},
                "currentProfile": c.get("currentProfile")}
        print(render(fmt, body, PROFILE_COLUMNS, _profile_cell(c)))
    elif args.cmd == "get-current":
        print(c.get("currentProfile", DEFAULT_PROFILE_NAME))
    elif args.cmd in ("create", "update", "import"):
        if args.cmd == "import":
            # ImportProfileCmd.java: exactly one of --file (YAML / JSON) or --inline (JSON, or
            # base64:<JSON>); an existing profile only with --update (overwritten, not merged)
            import base64
            import yaml
            if args.file is None and args.inline is None:
                raise CliError("Either --file or --inline must be specified")
            if args.file is not None and args.inline is not None:
                raise CliError("Only one of --file or --inline must be specified")
            if args.file is not None:
                if not os.path.isfile(args.file):
                    raise CliError(f"File {args.file} does not exist")
                with open(args.file) as f:
                    src = yaml.safe_load(f) or {}
            else:
                text = args.inline
                if text.startswith("base64:"):
                    text = base64.b64decode(text[len("base64:"):]).decode()
                src = json.loads(text)
            prof = {k: src.get(k) for k in _PROFILE_KEYS}
            _validate_profile(prof)
            existed = named_profile(c, args.name) is not None
            if existed and not args.update:
                raise CliError(f"Profile {args.name} already exists")
            created = not existed
        else:
            existing = named_profile(c, args.name)
            if args.cmd == "create" and existing is not None:
                raise CliError(f"Profile {args.name} already exists")
            if args.cmd == "update" and existing is None:
                raise _profile_not_found(c, args.name)
            prof = dict(existing or {})
            if args.name == DEFAULT_PROFILE_NAME:
                # the stored keys, not the filled-in defaults
                prof = {k: c.get(k) for k in _PROFILE_KEYS}
            for k, a in (("webServiceUrl", args.web_service_url), ("apiGatewayUrl", args.api_gateway_url),
                         ("tenant", args.tenant_name), ("token", args.token)):
                if a is not None:
                    prof[k] = a
            _validate_profile(prof)
            created = args.cmd == "create"
        if args.name == DEFAULT_PROFILE_NAME:
            for k in _PROFILE_KEYS:
                c[k] = prof.get(k)
        else:
            c["profiles"][args.name] = {**{k: prof.get(k) for k in _PROFILE_KEYS}, "name": args.name}
        print(f"profile {args.name} {'created' if created else 'updated'}")
        if args.set_current:
            c["currentProfile"] = args.name
            print(f"profile {args.name} set as current")
        save_config(c)
    elif args.cmd == "delete":
        if args.name == DEFAULT_PROFILE_NAME:
            raise CliError(f"Profile name {args.name} can't be deleted")
        if named_profile(c, args.name) is None:
            raise _profile_not_found(c, args.name)
        if c.get("currentProfile") == args.name:
            raise CliError("Cannot delete the current profile")
        c["profiles"].pop(args.name, None)
        save_config(c)
        print(f"profile {args.name} deleted")
    elif args.cmd == "set-current":
        if named_profile(c, args.name) is None:
            raise _profile_not_found(c, args.name)
        c["currentProfile"] = args.name
        save_config(c)
        print(f"profile {args.name} set as current")
    return 0


def cmd_configure(args) -> int:
    """ConfigureCmd.java: set one key of the default profile."""
    if getattr(args, "profile", None):
        raise ValueError("Global profile flag is not allowed here")
    c = load_config()
    c[args.key] = args.value
    save_config(c)
    print(f"profile default updated: {args.key}={args.value}")
    return 0


def cmd_tenants(args) -> int:
    """``tenants`` (commands/tenants/*.java): get / list print the server's body as sent."""
    cl = _client(args)
    if args.cmd == "list":
        print(cl.raw("GET", "/api/tenants"))
    elif args.cmd == "get":
        print(cl.raw("GET", f"/api/tenants/{args.name}"))
    elif args.cmd == "create":
        cl.tenant_create(args.name, args.max_units)
        print(f"tenant {args.name} created")
    elif args.cmd == "update":
        cl.tenant_update(args.name, args.max_units)
        print(f"tenant {args.name} updated")
    elif args.cmd == "put":
        cl.raw("PUT", f"/api/tenants/{args.name}", data="{}", headers={"Content-Type": "application/json"})
        print(f"tenant {args.name} created/updated")
    elif args.cmd == "delete":
        cl.tenant_delete(args.name)
        print(f"Tenant {args.name} deleted")
    return 0


def mermaid(app_dir: str, instance: Optional[str] = None, secrets: Optional[str] = None) -> str:
    """Mermaid flowchart of the execution plan (topics as stadiums, agents as boxes)."""
    from ..core.deployer import ApplicationDeployer
    from ..core.parser import build_from_directory
    info = build_from_directory(app_dir, instance, secrets)
    plan = ApplicationDeployer().create_implementation("app", info.application)
    lines = ["flowchart LR"]
    ids = {}

    def nid(s):
        return ids.setdefault(s, f"n{len(ids)}")

    for t in plan.topics:
        lines.append(f'  {nid("topic:" + t)}(["{t}"])')
    for node in plan.agents.values():
        steps = [p["agentId"] for p in node.configuration.get("processors", [])] if \
            node.agent_type == "composite-agent" else [node.id]
        label = "<br/>".join(steps)
        lines.append(f'  {nid("agent:" + node.id)}["{label}<br/><i>{node.agent_type}</i>"]')
        if node.input is not None:
            lines.append(f'  {nid("topic:" + node.input.name)} --> {nid("agent:" + node.id)}')
        if node.output is not None:
            lines.append(f'  {nid("agent:" + node.id)} --> {nid("topic:" + node.output.name)}')
    return "\n".join(lines)


APP_COLUMNS = ("id", "streaming", "compute", "status", "executors", "replicas")


def _path(d, path: str):
    for part in path.split("."):
        if not isinstance(d, dict):
            return None
        d = d.get(part)
    return d


def _app_cell(app, col):
    """ListApplicationCmd.getRawFormatValuesSupplier: executors DEPLOYED / all, replicas
    RUNNING / all (empty when no executor reports replicas)."""
    if col == "id":
        return _path(app, "application-id")
    if col == "streaming":
        return _path(app, "application.instance.streamingCluster.type")
    if col == "compute":
        return _path(app, "application.instance.computeCluster.type")
    if col == "status":
        return _path(app, "status.status.status")
    executors = _path(app, "status.executors") or []
    if col == "executors":
        ok = sum(1 for e in executors if str(_path(e, "status.status")) == "DEPLOYED")
        return f"{ok}/{len(executors)}"
    if col == "replicas":
        reps = [r for e in executors for r in (e.get("replicas") or [])]
        if not reps:
            return ""
        return f"{sum(1 for r in reps if str(r.get('status')) == 'RUNNING')}/{len(reps)}"
    return app.get(col) if isinstance(app, dict) else None


def cmd_apps(args) -> int:
    """``apps`` (commands/applications/*.java): the reference CLI's messages and formats."""
    from .printer import render
    if args.cmd == "diagram":
        print(mermaid(args.app, args.instance, args.secrets))
        return 0
    if args.cmd == "ui":
        from .app_ui import serve_forever
        p = current_profile(args)
        return serve_forever(_client(args), args.name, p["apiGatewayUrl"], p["tenant"], args.port,
                             open_browser=not args.no_browser)
    cl = _tenant_client(args)
    if args.cmd in ("deploy", "update"):
        # https:// / GitHub / file:// sources (BaseCmd.checkFileExistsOrDownload)
        args.app, args.instance, args.secrets = _resolve_sources(args)
        if args.cmd == "update" and not (args.app or args.instance or args.secrets):
            raise CliError("no application, instance or secrets file provided")
        if args.cmd == "deploy" and not (args.app and args.instance):
            raise CliError("application and instance files are required")
        if args.app:
            from .sources import download_dependencies
            download_dependencies(args.app, print)
        size = len(_zip_size_probe(args.app)) // 1024 if args.app else 0
    if args.cmd == "deploy":
        if args.dry_run:
            print(f"resolving application: {args.name}. Dry run mode is enabled, the application will NOT be "
                  f"deployed")
        else:
            print(f"deploying application: {args.name} ({size} KB)")
        r = cl.deploy_raw(args.name, args.app, args.instance, args.secrets, args.dry_run, args.auto_upgrade)
        if args.dry_run:
            fmt = args.output or "yaml"
            _check_formats(fmt, ("json", "yaml"))
            print(render(fmt, r.text))
        else:
            print(f"application {args.name} deployed")
    elif args.cmd == "update":
        print(f"updating application: {args.name} ({size} KB)")
        cl.update(args.name, args.app, args.instance, args.secrets, args.auto_upgrade, args.force_restart)
        print(f"application {args.name} updated")
    elif args.cmd == "get":
        fmt = args.output or "raw"
        _check_formats(fmt, ("raw", "json", "yaml", "mermaid"))
        body = cl.raw("GET", f"/api/applications/{cl.tenant}/{args.name}", params={"stats": str(args.stats).lower()})
        if fmt == "mermaid":   # GetApplicationCmd: -o mermaid
            from .app_ui import mermaid_from_description
            print(mermaid_from_description(json.loads(body)), end="")
        else:
            print(render(fmt, body, APP_COLUMNS, _app_cell))
    elif args.cmd == "list":
        fmt = args.output or "raw"
        _check_formats(fmt, ("raw", "json", "yaml"))
        print(render(fmt, cl.raw("GET", f"/api/applications/{cl.tenant}"), APP_COLUMNS, _app_cell))
    elif args.cmd == "delete":
        cl.delete(args.name, args.force)
        print(f"Application '{args.name}' marked for deletion" + (" (forced)" if args.force else ""))
    elif args.cmd == "logs":
        for line in cl.log_lines(args.name, args.output or "text", args.filter, follow=not args.no_follow):
            if line != "Heartbeat":
                print(line, flush=True)
    elif args.cmd == "download":
        import re
        r = cl.download_response(args.name)
        out = args.output_file
        if out is None:
            m = re.search(r"""filename=["']?([^"'\r\n]+)["']?""", r.headers.get("Content-Disposition") or "")
            out = m.group(1) if m else f"{cl.tenant}-{args.name}.zip"
        with open(out, "wb") as f:
            f.write(r.content)
        print(f"Downloaded application code to {os.path.abspath(out)}")
    return 0


def _zip_size_probe(app: str) -> bytes:
    from .client import zip_directory
    return zip_directory(app) if os.path.isdir(app) else open(app, "rb").read()


# ---------------------------------------------------------------- gateway
def _gw_url(args, kind: str, gateway: str) -> str:
    import urllib.parse
    p = current_profile(args)
    q = [(f"param:{k}", v) for k, v in (kv.split("=", 1) for kv in args.param or [])]
    if getattr(args, "position", None):
        q.append(("option:position", args.position))
    if args.credentials:
        q.append(("credentials", args.credentials))
    if args.test_credentials:
        q.append(("test-credentials", args.test_credentials))
    base = p["apiGatewayUrl"].rstrip("/")
    return f"{base}/v1/{kind}/{p['tenant']}/{args.application}/{gateway}" + (
        "?" + urllib.parse.urlencode(q) if q else "")


def cmd_gateway(args) -> int:
    import asyncio
    import aiohttp

    async def produce():
        async with aiohttp.ClientSession() as s, s.ws_connect(_gw_url(args, "produce", args.gateway)) as ws:
            msg = {"key": args.key, "value": args.value,
                   "headers": dict(kv.split("=", 1) for kv in args.header or [])}
            await ws.send_str(json.dumps(msg))
            print((await ws.receive()).data)

    async def consume():
        n = 0
        async with aiohttp.ClientSession() as s, s.ws_connect(_gw_url(args, "consume", args.gateway)) as ws:
            async for m in ws:
                print(m.data, flush=True)
                n += 1
                if args.num_messages and n >= args.num_messages:
                    return

    async def chat():
        loop = asyncio.get_running_loop()
        async with aiohttp.ClientSession() as s, s.ws_connect(_gw_url(args, "chat", args.gateway)) as ws:
            done = asyncio.Event()
            parts: Dict[str, Dict[int, str]] = {}

            async def reader():
                async for m in ws:
                    d = json.loads(m.data)
                    if "record" not in d:
                        continue
                    rec = d["record"]
                    h = rec.get("headers") or {}
                    sid = h.get("stream-id")
                    if sid is None:
                        print(f"\n< {rec.get('value')}", flush=True)
                        done.set()
                        continue
                    parts.setdefault(sid, {})[int(h.get("stream-index", 0))] = rec.get("value") or ""
                    print(rec.get("value") or "", end="", flush=True)
                    if h.get("stream-last-message") == "true":
                        print(flush=True)
                        done.set()
            task = asyncio.ensure_future(reader())
            while True:
                line = await loop.run_in_executor(None, sys.stdin.readline)
                if not line:
                    break
                line = line.strip()
                if not line:
                    continue
                done.clear()
                await ws.send_str(json.dumps({"value": line}))
                await asyncio.wait_for(done.wait(), timeout=600)
            task.cancel()

    fn = {"produce": produce, "consume": consume, "chat": chat}[args.cmd]
    asyncio.new_event_loop().run_until_complete(fn())
    return 0


# ---------------------------------------------------------------- local run (docker run)
LOCAL_RUN_PROFILE = "local-docker-run"


def _java_dependencies(app_dir: str):
    import yaml
    path = os.path.join(app_dir, "configuration.yaml")
    if not os.path.exists(path):
        return []
    with open(path, encoding="utf-8") as f:
        data = yaml.safe_load(f) or {}
    return (data.get("configuration") or {}).get("dependencies") or []


def _resolve_sources(args):
    """app / instance / secrets through ``BaseCmd.checkFileExistsOrDownload`` (sources.py)."""
    from .sources import as_app_directory, check_file_exists_or_download
    cache = not getattr(args, "disable_local_repositories_cache", False)
    app = check_file_exists_or_download(getattr(args, "app", None), cache)
    inst = check_file_exists_or_download(getattr(args, "instance", None), cache)
    sec = check_file_exists_or_download(getattr(args, "secrets", None), cache)
    return (as_app_directory(app) if app else None), inst, sec


def cmd_run(args) -> int:
    """``langstream docker run`` (``LocalRunApplicationCmd.java:165-440``) without the
    container: the bundled services (broker / S3 / database, runtime/local_services.py),
    the control plane (8090), the gateway (8091), the agent-control API (8790) and the
    application's agents all run in this process; ``--watch-files`` hot-reloads python/,
    ``--start-ui`` serves the application UI on ``-up`` (8092)."""
    import logging
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(threadName)s %(message)s")
    from ..core.store import InMemoryApplicationStore
    from ..gateway.server import GatewayServer, GatewayService
    from ..runtime.local_services import ApplicationWatcher, LocalServices, restart_agents
    from ..runtime.pod import AgentAPIServer
    from ..webservice.server import ControlPlane, WebServiceServer
    from ..core.file_refs import read_yaml_with_references
    from .client import zip_directory
    dry = args.dry_run
    app_dir, inst_path, sec_path = _resolve_sources(args)
    # LocalRunApplicationCmd.java:210 fetches configuration.dependencies into java/lib for the
    # container's JVM; the agents run in this process and no JVM loads them, so the
    # application directory is left as it is
    for dep in _java_dependencies(app_dir):
        print(f"Dependency {dep.get('name')} ({dep.get('url')}): not needed, the agents run without a JVM",
              flush=True)
    tenant = args.tenant or "default"
    print(f"Tenant: {tenant}\nApplication: {args.name}\nApplication directory: {os.path.abspath(app_dir)}", flush=True)
    print(f"Filter agent: {args.only_agent}" if args.only_agent else "Running all the agents in the application",
          flush=True)
    for flag in ("memory", "cpus", "docker_command", "langstream_runtime_version", "langstream_runtime_docker_image"):
        if getattr(args, flag, None):
            print(f"--{flag.replace('_', '-')} ignored: the application runs in this process, not in a container",
                  flush=True)
    services = LocalServices(broker=args.start_broker and not dry, s3=args.start_s3 and not dry,
                             database=args.start_database and not dry, host=args.host,
                             # LANGSTREAM_LOCAL_SERVICES_PORTS=random: free ports + aliases (tests)
                             well_known_ports=os.environ.get("LANGSTREAM_LOCAL_SERVICES_PORTS") != "random").start()
    print(f"Start broker: {services.broker is not None}" +
          (f" (kafka bootstrap {services.broker.bootstrap})" if services.broker else ""), flush=True)
    print(f"Start S3: {services.s3 is not None}" + (f" ({services.s3.endpoint})" if services.s3 else ""), flush=True)
    print(f"Start Database: {services.database is not None}" +
          (f" ({services.database.url})" if services.database else ""), flush=True)
    stop = threading.Event()
    started: list = []
    try:
        if inst_path:
            instance = read_yaml_with_references(inst_path)
        else:
            instance = services.default_instance()
            print("Using default instance file that connects to the Kafka broker started here" if services.broker
                  else "The broker is disabled: using the in-process memory streaming cluster", flush=True)
        secrets = read_yaml_with_references(sec_path) if sec_path else None
        store = InMemoryApplicationStore()
        cp = ControlPlane(store)
        cp.only_agents = [args.only_agent] if args.only_agent else None
        cp.local_runs = True
        store.put_tenant(tenant)
        res = cp.deploy(tenant, args.name, zip_directory(app_dir), instance, secrets, dry_run=dry)
        if dry:
            _print(res, "yaml")
            return 0
        sa = store.get(tenant, args.name)
        if sa.status != "DEPLOYED":
            print(f"application {args.name} failed to start: {sa.error}", file=sys.stderr, flush=True)
            return 1
        ws = gw = None
        if args.start_webservices:
            ws = WebServiceServer(cp, host=args.host, port=args.web_port).start()
            gw = GatewayServer(GatewayService(store), host=args.host, port=args.gateway_port).start()
            started += [gw, ws]
            _update_local_run_profile(tenant, ws.url, gw.url.replace("http", "ws"))
        api = AgentAPIServer(sa.runner.runners if sa.runner else [], host=args.host, port=args.agents_port).start()
        started.insert(0, api)
        agents_url = f"http://{args.host}:{api.port}"
        print(f"application {args.name} running: webservice {ws.url if ws else '-'}  "
              f"gateway {gw.url.replace('http', 'ws') if gw else '-'}  agents {agents_url}", flush=True)
        if args.watch_files:
            if os.path.isdir(os.path.join(app_dir, "python")):
                code = cp.local_code(sa) if sa.code_archive_id else None
                started.insert(0, ApplicationWatcher(app_dir, code, lambda _c: restart_agents(agents_url)).start())
            else:
                print(f"Python directory {os.path.join(app_dir, 'python')} not found, not watching files", flush=True)
        if args.start_ui and ws is not None:
            from .app_ui import AppUIServer
            from .client import AdminClient
            ui = AppUIServer(AdminClient(ws.url, tenant), args.name, gw.url.replace("http", "ws"), tenant,
                             host=args.host, port=args.ui_port).start()
            started.insert(0, ui)
            print(f"Started UI at {ui.url}", flush=True)
        try:
            import signal
            signal.signal(signal.SIGTERM, lambda *_: stop.set())
        except ValueError:
            pass
        try:
            while not stop.is_set():
                stop.wait(1.0)
                if sa.runner is not None and sa.runner.errors:
                    print(f"agent failure: {sa.runner.errors[0]!r}", file=sys.stderr)
                    return 1
        except KeyboardInterrupt:
            pass
        finally:
            for srv in started:
                try:
                    srv.stop()
                except Exception:  # noqa: BLE001
                    pass
            cp.delete(tenant, args.name, force=True)
        return 0
    finally:
        services.stop()


def _update_local_run_profile(tenant: str, web: str, gateway: str) -> None:
    """``LocalRunApplicationCmd.updateLocalDockerRunProfile``: a ``local-docker-run``
    profile pointing at this run."""
    try:
        c = load_config()
        c["profiles"][LOCAL_RUN_PROFILE] = {"webServiceUrl": web, "apiGatewayUrl": gateway, "tenant": tenant,
                                            "token": None}
        save_config(c)
        print(f"profile {LOCAL_RUN_PROFILE} updated", flush=True)
    except OSError as e:
        print(f"could not update the {LOCAL_RUN_PROFILE} profile: {e}", flush=True)


def cmd_archetypes(args) -> int:
    cl = _client(args)
    if args.cmd == "list":
        _print(cl.archetypes())
    elif args.cmd == "get":
        _print(next((a for a in cl.archetypes() if a["id"] == args.id), {}))
    elif args.cmd == "deploy":
        params = json.loads(args.parameters) if args.parameters else {}
        _print(cl.archetype_deploy(args.id, args.name, params))
    return 0


def cmd_python(args) -> int:
    pydir = os.path.join(args.app, "python")
    if args.cmd == "load-pip-requirements":
        req = os.path.join(pydir, "requirements.txt")
        if not os.path.exists(req):
            print("no python/requirements.txt")
            return 0
        import importlib.util
        missing = []
        for line in open(req):
            name = line.split("#")[0].strip().split("==")[0].split(">=")[0].strip()
            if name and importlib.util.find_spec(name.replace("-", "_")) is None:
                missing.append(name)
        os.makedirs(os.path.join(pydir, "lib"), exist_ok=True)
        if missing:
            print("not installed (no package index available in this environment): " + ", ".join(missing))
            return 1
        print("all requirements importable")
        return 0
    if args.cmd == "run-tests":
        import subprocess
        env = dict(os.environ, PYTHONPATH=os.pathsep.join([pydir, os.path.join(pydir, "lib"),
                                                           os.environ.get("PYTHONPATH", "")]))
        return subprocess.call([sys.executable, "-m", "pytest", pydir, "-q"], env=env)
    return 2


def cmd_broker(args) -> int:
    from ..topics.kafka.broker import KafkaBroker
    b = KafkaBroker(args.host, args.port, default_partitions=args.partitions).start()
    print(f"kafka-protocol broker listening on {b.bootstrap}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        b.stop()
    return 0


def cmd_pulsar_standalone(args) -> int:
    from ..topics.pulsar.standalone import main as pulsar_main
    return pulsar_main(["--host", args.host, "--port", str(args.port)])


def cmd_pravega_standalone(args) -> int:
    from ..topics.pravega.standalone import main as pravega_main
    return pravega_main(["--host", args.host, "--port", str(args.port)])


def cmd_pg_standalone(args) -> int:
    """The PostgreSQL v3 protocol stand-in over SQLite (agents/vector/pg_standalone.py)."""
    import signal
    from ..agents.vector.pg_standalone import PgStandalone
    users = {}
    for u in args.user or ["postgres:password"]:
        name, _, pw = u.partition(":")
        users[name] = pw
    srv = PgStandalone(args.host, args.port, users=users, auth=args.auth, db_path=args.db).start()
    print(f"pg-standalone listening on {srv.host}:{srv.port} ({srv.url})", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    srv.stop()
    return 0


def cmd_operator(args) -> int:
    from ..operator import main as operator_main
    argv = ["--resync", str(args.resync)] + (["--in-process"] if args.in_process else [])
    for k in ("api_server", "token", "namespace", "image"):
        v = getattr(args, k)
        if v:
            argv += ["--" + k.replace("_", "-"), v]
    return operator_main(argv)


def _json_arg(v: Optional[str]) -> Optional[dict]:
    """A JSON object given inline or as ``@file``."""
    if not v:
        return None
    if v.startswith("@"):
        with open(v[1:]) as f:
            v = f.read()
    return json.loads(v)


def cmd_code_download(args) -> int:
    """Agent init step: fetch the application archive (from the code storage directly when
    ``--code-storage`` is given, else through the control plane) and unpack it."""
    import io
    import zipfile
    cs = _json_arg(args.code_storage or os.environ.get("LANGSTREAM_CODE_STORAGE"))
    if cs is not None and args.code_archive_id:
        from ..core.codestorage import code_storage_for
        data = code_storage_for(cs).download_application_code(args.tenant, args.code_archive_id)
    else:
        from .client import AdminClient
        url = args.web_service_url or os.environ.get("LANGSTREAM_WEBSERVICE_URL",
                                                     "http://langstream-control-plane:8090")
        data = AdminClient(url, args.tenant).download(args.application)
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        z.extractall(args.target)
    return 0


# ---------------------------------------------------------------- parser
def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="langstream", description="LangStream (MI355X-native) command line")
    ap.add_argument("-p", "--profile")
    ap.add_argument("--tenant")
    ap.add_argument("--conf", help="CLI configuration file (default ~/.langstream/config.yaml, or "
                                   "$LANGSTREAM_CLI_CONFIG)")
    ap.add_argument("--disable-local-repositories-cache", action="store_true",
                    help="clone GitHub application sources afresh instead of updating the local cache")
    sub = ap.add_subparsers(dest="group", required=True)

    p = sub.add_parser("profiles")
    ps = p.add_subparsers(dest="cmd", required=True)
    ps.add_parser("list").add_argument("-o", dest="output", help="raw (default), json or yaml")
    ps.add_parser("get-current")
    for c in ("get", "delete", "set-current"):
        x = ps.add_parser(c)
        x.add_argument("name")
        if c == "get":
            x.add_argument("-o", dest="output", help="raw (default), json or yaml")
    x = ps.add_parser("import", help="import a profile from a file or inline JSON")
    x.add_argument("name")
    x.add_argument("-f", "--file")
    x.add_argument("-i", "--inline", help="JSON, or base64:<JSON>")
    x.add_argument("-u", "--update", action="store_true", help="overwrite an existing profile")
    x.add_argument("--set-current", action="store_true")
    for c in ("create", "update"):
        x = ps.add_parser(c)
        x.add_argument("name")
        x.add_argument("--web-service-url")
        x.add_argument("--api-gateway-url")
        x.add_argument("--tenant", dest="tenant_name")
        x.add_argument("--token")
        x.add_argument("--set-current", action="store_true")
    p.set_defaults(fn=cmd_profiles)

    t = sub.add_parser("tenants")
    ts = t.add_subparsers(dest="cmd", required=True)
    ts.add_parser("list")
    for c in ("get", "delete"):
        ts.add_parser(c).add_argument("name")
    for c in ("create", "update", "put"):
        x = ts.add_parser(c)
        x.add_argument("name")
        x.add_argument("--max-total-resource-units", "--max-units", dest="max_units", type=int)
    t.set_defaults(fn=cmd_tenants)

    cf = sub.add_parser("configure", help="set a key of the default profile")
    cf.add_argument("key", choices=("webServiceUrl", "apiGatewayUrl", "tenant", "token"))
    cf.add_argument("value")
    cf.set_defaults(fn=cmd_configure)

    a = sub.add_parser("apps")
    asub = a.add_subparsers(dest="cmd", required=True)
    for c in ("deploy", "update"):
        x = asub.add_parser(c)
        x.add_argument("name")
        x.add_argument("-app", "--app", required=(c == "deploy"))
        x.add_argument("-i", "--instance")
        x.add_argument("-s", "--secrets")
        x.add_argument("--auto-upgrade", action="store_true")
        if c == "deploy":
            x.add_argument("--dry-run", action="store_true")
            x.add_argument("-o", "--output", help="dry-run output: yaml (default) or json")
        else:
            x.add_argument("--force-restart", action="store_true")
    x = asub.add_parser("get")
    x.add_argument("name")
    x.add_argument("-o", "--output", help="raw (default), json, yaml or mermaid")
    x.add_argument("-s", "--stats", action="store_true", help="include agent metrics")
    x = asub.add_parser("list")
    x.add_argument("-o", "--output", help="raw (default), json or yaml")
    x = asub.add_parser("delete")
    x.add_argument("name")
    x.add_argument("-f", "--force", action="store_true")
    x = asub.add_parser("logs")
    x.add_argument("name")
    x.add_argument("-f", "--filter", action="append", help="only these replicas (repeatable)")
    x.add_argument("-o", "--output", help="text (default) or json")
    x.add_argument("--no-follow", action="store_true", help="print the logs so far and exit")
    x = asub.add_parser("download")
    x.add_argument("name")
    x.add_argument("-o", "--output-file")
    x = asub.add_parser("diagram")
    x.add_argument("-app", "--app", required=True)
    x.add_argument("-i", "--instance")
    x.add_argument("-s", "--secrets")
    x = asub.add_parser("ui", help="local web UI for the application's gateways, diagram and logs")
    x.add_argument("name")
    x.add_argument("-p", "--port", type=int, default=8092, help="0 = a random port")
    x.add_argument("--no-browser", action="store_true")
    a.set_defaults(fn=cmd_apps)

    g = sub.add_parser("gateway")
    gs = g.add_subparsers(dest="cmd", required=True)
    for c in ("produce", "consume", "chat"):
        x = gs.add_parser(c)
        x.add_argument("application")
        x.add_argument("gateway")
        x.add_argument("-p", "--param", action="append")
        x.add_argument("-c", "--credentials")
        x.add_argument("--test-credentials")
        if c == "produce":
            x.add_argument("-v", "--value")
            x.add_argument("-k", "--key")
            x.add_argument("--header", action="append")
        if c == "consume":
            x.add_argument("--position")
            x.add_argument("-n", "--num-messages", type=int, default=0)
        if c == "chat":
            x.add_argument("--position")
    g.set_defaults(fn=cmd_gateway)

    def run_args(r):
        b = argparse.BooleanOptionalAction
        r.add_argument("name")
        r.add_argument("-app", "--app", "--application", dest="app", required=True,
                       help="application directory, zip, file:// path, https:// URL or GitHub URL")
        r.add_argument("-i", "--instance")
        r.add_argument("-s", "--secrets")
        r.add_argument("--dry-run", action="store_true")
        r.add_argument("--start-broker", action=b, default=True, help="start the Kafka-protocol broker (9092)")
        r.add_argument("--start-s3", action=b, default=True, help="start the S3 service (9000)")
        r.add_argument("--start-database", action=b, default=True, help="start the database service (7000)")
        r.add_argument("--start-webservices", action=b, default=True, help="start the control plane and gateway")
        r.add_argument("--start-ui", action=b, default=True, help="start the application UI")
        r.add_argument("--watch-files", action=b, default=True, help="hot-reload python/ changes")
        r.add_argument("-up", "--ui-port", type=int, default=8092, help="UI port (0: a random port)")
        r.add_argument("--only-agent", help="run only this agent")
        r.add_argument("--host", default="127.0.0.1")
        r.add_argument("--web-port", type=int, default=8090)
        r.add_argument("--gateway-port", type=int, default=8091)
        r.add_argument("--agents-port", type=int, default=8790)
        for opt in ("--memory", "--cpus", "--docker-command", "--langstream-runtime-version",
                    "--langstream-runtime-docker-image"):
            r.add_argument(opt, help="accepted for compatibility (no container)")
        r.add_argument("--docker-args", action="append", help="accepted for compatibility (no container)")
        r.set_defaults(fn=cmd_run)

    run_args(sub.add_parser("run", help="run an application locally (the `docker run` equivalent)"))
    dk = sub.add_parser("docker", help="local runs (`langstream docker run`)")
    dks = dk.add_subparsers(dest="cmd", required=True)
    run_args(dks.add_parser("run", help="run an application locally with the bundled services"))

    ar = sub.add_parser("archetypes")
    ars = ar.add_subparsers(dest="cmd", required=True)
    ars.add_parser("list")
    ars.add_parser("get").add_argument("id")
    x = ars.add_parser("deploy")
    x.add_argument("id")
    x.add_argument("name")
    x.add_argument("-p", "--parameters", help="JSON object of archetype parameters")
    ar.set_defaults(fn=cmd_archetypes)

    py = sub.add_parser("python")
    pys = py.add_subparsers(dest="cmd", required=True)
    for c in ("load-pip-requirements", "run-tests"):
        pys.add_parser(c).add_argument("-app", "--app", required=True)
    py.set_defaults(fn=cmd_python)

    bk = sub.add_parser("broker", help="run the in-tree single-node Kafka-protocol broker")
    bk.add_argument("--host", default="127.0.0.1")
    bk.add_argument("--port", type=int, default=9092)
    bk.add_argument("--partitions", type=int, default=1, help="default partitions of auto-created topics")
    bk.set_defaults(fn=cmd_broker)

    ps = sub.add_parser("pulsar-standalone",
                        help="run the in-tree Pulsar-compatible broker (WebSocket API + admin REST)")
    ps.add_argument("--host", default="127.0.0.1")
    ps.add_argument("--port", type=int, default=8080)
    ps.set_defaults(fn=cmd_pulsar_standalone)

    pv = sub.add_parser("pravega-standalone",
                        help="run the in-tree single-node Pravega-style server (controller + segment store)")
    pv.add_argument("--host", default="127.0.0.1")
    pv.add_argument("--port", type=int, default=9090)
    pv.set_defaults(fn=cmd_pravega_standalone)

    s3 = sub.add_parser("s3-standalone", help="run the S3-protocol object store (the docker image's MinIO)")
    s3.add_argument("--host", default="127.0.0.1")
    s3.add_argument("--port", type=int, default=9000)
    s3.add_argument("--data-dir", default=None)
    s3.set_defaults(fn=lambda a: __import__("langstream_amd.agents.s3_standalone", fromlist=["main"]).main(
        ["--host", a.host, "--port", str(a.port)] + (["--data-dir", a.data_dir] if a.data_dir else [])))

    pg = sub.add_parser("pg-standalone",
                        help="run the in-tree PostgreSQL wire-protocol stand-in (SQL on SQLite) for jdbc:postgresql://")
    pg.add_argument("--host", default="127.0.0.1")
    pg.add_argument("--port", type=int, default=5432)
    pg.add_argument("--user", action="append", help="user:password (repeatable; default postgres:password)")
    pg.add_argument("--auth", choices=("scram-sha-256", "md5", "password", "trust"), default="scram-sha-256")
    pg.add_argument("--db", default=None, help="SQLite file (default: in memory)")
    pg.set_defaults(fn=cmd_pg_standalone)

    opr = sub.add_parser("operator", help="run the Kubernetes operator (Application / Agent CRs)")
    opr.add_argument("--api-server", default=None)
    opr.add_argument("--token", default=None)
    opr.add_argument("--namespace", default=None)
    opr.add_argument("--image", default=None)
    opr.add_argument("--resync", type=float, default=5.0)
    opr.add_argument("--in-process", action="store_true",
                     help="run application setup / deployer in the operator instead of as Kubernetes Jobs")
    opr.set_defaults(fn=cmd_operator)

    gws = sub.add_parser("gateway-server", help="run the API gateway (WebSocket + HTTP) over an application store")
    gws.add_argument("--host", default="0.0.0.0")
    gws.add_argument("--port", type=int, default=8091)
    gws.add_argument("--store", choices=("kubernetes",), default="kubernetes")
    gws.add_argument("--api-server", default=None, help="Kubernetes API server (default: in-cluster)")
    gws.set_defaults(fn=cmd_gateway_server)

    dc = sub.add_parser("docs", help="generate the agents / resources / assets configuration reference")
    dc.add_argument("--format", choices=("json", "markdown"), default="json")
    dc.add_argument("--output", "-o", default=None, help="file to write (default: stdout)")
    dc.set_defaults(fn=cmd_docs)

    cd = sub.add_parser("code-download")
    cd.add_argument("--tenant", default="default")
    cd.add_argument("--application", required=True)
    cd.add_argument("--code-archive-id")
    cd.add_argument("--target", required=True)
    cd.add_argument("--web-service-url")
    cd.add_argument("--code-storage", help="code storage config JSON (or @file), e.g. "
                                           "'{\"type\": \"s3\", \"configuration\": {...}}'")
    cd.set_defaults(fn=cmd_code_download)

    cp = sub.add_parser("control-plane", help="run the control-plane web service (applications, tenants, code)")
    cp.add_argument("--host", default="0.0.0.0")
    cp.add_argument("--port", type=int, default=8090)
    cp.add_argument("--store", choices=("memory", "kubernetes"), default="memory")
    cp.add_argument("--api-server", default=None, help="Kubernetes API server (store=kubernetes)")
    cp.add_argument("--code-storage", default=None, help="code storage config JSON (or @file)")
    cp.add_argument("--code-dir", default=None, help="local cache of unpacked archives")
    cp.add_argument("--auth-secret", default=None, help="raw HMAC secret for bearer tokens on /api/* "
                                                         "(shorthand for --security secret-key)")
    cp.add_argument("--security", default=None,
                    help="application.security.token properties as JSON (or @file): secret-key, public-key, "
                         "public-alg, auth-claim, audience-claim, audience, admin-roles, jwks-hosts-allowlist, "
                         "allow-kubernetes-service-accounts, kubernetes-namespace-prefix")
    cp.add_argument("--admin-roles", default=None, help="comma-separated principals granted ROLE_ADMIN")
    cp.add_argument("--max-units-per-tenant", type=int, default=0)
    cp.add_argument("--max-units-limit", type=int, default=0,
                    help="cap on a tenant's maxTotalResourceUnits (0: none)")
    cp.add_argument("--default-tenant", default="default", help="tenant created at start when missing")
    cp.add_argument("--no-default-tenant", action="store_true")
    cp.set_defaults(fn=cmd_control_plane)
    return ap


def cmd_control_plane(args) -> int:
    import logging
    import signal
    logging.basicConfig(level=logging.INFO)
    from ..core.codestorage import code_storage_for
    from ..webservice.server import ControlPlane, WebServiceServer
    store = None
    if args.store == "kubernetes":
        from ..operator.kube import KubeClient
        from ..operator.store import KubernetesApplicationStore
        store = KubernetesApplicationStore(KubeClient(args.api_server))
    cs = _json_arg(args.code_storage or os.environ.get("LANGSTREAM_CODE_STORAGE"))
    cp = ControlPlane(store, code_dir=args.code_dir, max_units_per_tenant=args.max_units_per_tenant,
                      code_storage=code_storage_for(cs) if cs else None,
                      default_tenant=None if args.no_default_tenant else args.default_tenant,
                      max_units_limit=args.max_units_limit)
    sec = dict(_json_arg(args.security or os.environ.get("LANGSTREAM_SECURITY_TOKEN")) or {})
    if args.admin_roles:
        sec["admin-roles"] = [r.strip() for r in args.admin_roles.split(",") if r.strip()]
    srv = WebServiceServer(cp, host=args.host, port=args.port, auth_secret=args.auth_secret, security=sec).start()
    print(f"control plane listening on {srv.url}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    srv.stop()
    return 0


def cmd_gateway_server(args) -> int:
    """The reference's langstream-api-gateway deployment: gateways of the applications in
    the Kubernetes application store, topics reached through each app's instance."""
    import logging
    import signal
    logging.basicConfig(level=logging.INFO)
    from ..gateway.server import GatewayServer, GatewayService
    from ..operator.kube import KubeClient
    from ..operator.store import KubernetesApplicationStore
    gw = GatewayServer(GatewayService(KubernetesApplicationStore(KubeClient(args.api_server))),
                       host=args.host, port=args.port).start()
    print(f"api gateway listening on {args.host}:{args.port}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    gw.stop()
    return 0


def cmd_docs(args) -> int:
    """``DocumentationGeneratorStarter`` equivalent: the configuration models as JSON or Markdown."""
    from ..core.config_model import docs_markdown, generate_docs
    docs = generate_docs()
    text = json.dumps(docs, indent=2) if args.format == "json" else docs_markdown(docs)
    if args.output:
        with open(args.output, "w") as f:
            f.write(text + "\n")
    else:
        print(text)
    return 0


def _picocli_booleans(argv: List[str]) -> List[str]:
    """picocli's ``--start-broker=false`` form of the boolean options -> ``--no-start-broker``."""
    import re
    out = []
    for a in argv:
        m = re.match(r"^--((?:start-[\w-]+)|watch-files)=(true|false)$", a, re.I)
        out.append(a if not m else (f"--{m.group(1)}" if m.group(2).lower() == "true" else f"--no-{m.group(1)}"))
    return out


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(_picocli_booleans(list(sys.argv[1:] if argv is None else argv)))
    global CONFIG
    if getattr(args, "conf", None):
        CONFIG = os.path.abspath(os.path.expanduser(args.conf))
    try:
        return args.fn(args) or 0
    except Exception as e:  # noqa: BLE001
        # the message alone, exit code 1 (LangStreamCLI.execute)
        print(str(e) or type(e).__name__, file=sys.stderr)
        return 1


if __name__ == "__main__":
    sys.exit(main())
