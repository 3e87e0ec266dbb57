"""Control plane REST API (``WS/application/ApplicationResource.java:79-546``,
``ApplicationService.java:65-385``, ``WS/common/TenantResource.java``, ``WS/archetype/*``).

Endpoints:
* ``/api/tenants`` GET (all) | ``/api/tenants/{tenant}`` GET / PUT / POST / DELETE;
* ``/api/applications/{tenant}`` GET (list);
* ``/api/applications/{tenant}/{id}`` POST (deploy, multipart ``app`` zip + ``instance``
  + ``secrets`` text parts, ``?dry-run=true`` returns the execution plan only), PATCH
  (update: same parts; unchanged python code keeps its code archive id -- digest
  check, ``ModelBuilder.java:275-349``), DELETE (``?force=``), GET (``?stats=true`` adds
  live agent status);
* ``/api/applications/{tenant}/{id}/logs`` NDJSON stream of the app's agent logs;
* ``/api/applications/{tenant}/{id}/code`` (zip download) and ``/code/info``;
* ``/api/archetypes/{tenant}`` list, ``/api/archetypes/{tenant}/{id}`` get,
  ``/api/archetypes/{tenant}/{id}/applications/{app}`` POST (deploy from archetype with
  JSON parameters).

Deploy = parse (``core.parser``) -> resolve placeholders + plan (validation, the tenant
resource-unit limit Σ size×parallelism, ``ApplicationService.java:95-125``) -> store ->
start on the compute cluster: ``local``/``none``/``docker`` run in-process
(``LocalApplicationRunner``, the docker-run path); ``kubernetes`` renders the Agent
custom resources + StatefulSets (``core.k8s``) into the store (and applies them with
kubectl when ``apply`` is configured).

Security (``security.py``, ``SecurityConfiguration.java``): with a token configuration every
``/api/**`` call needs a bearer JWT (HMAC secret, RSA / EC public key, allowlisted
``jwks_uri`` claims or the local Kubernetes issuer); ``/api/tenants/**`` needs a principal
in ``admin-roles``; application / archetype / log / code calls on tenant T need ROLE_ADMIN
or principal == T.  No token configuration: the API is open (the reference's
``application.security.enabled=false`` default).
"""
from __future__ import annotations

import asyncio
import collections
import hashlib
import io
import json
import logging
import os
import shutil
import tempfile
import threading
import time
import zipfile
from typing import Any, Dict, List, Optional

from ..core.parser import build_application_instance, archetype_application_files, directory_digest, read_app_directory
from ..core.store import ApplicationStore, InMemoryApplicationStore, StoredApplication

log = logging.getLogger(__name__)


class _AppLogBuffer(logging.Handler):
    """Collects log records emitted by one application's agent threads."""

    def __init__(self, maxlen: int = 5000):
        super().__init__()
        self.records: "collections.deque" = collections.deque(maxlen=maxlen)
        self.threads: set = set()
        self.seq = 0
        self.cv = threading.Condition()

    def emit(self, record: logging.LogRecord) -> None:
        # agent threads and their worker pools are named "agent-<agent id>..."
        if not any(record.threadName.startswith(p) for p in self.threads):
            return
        with self.cv:
            self.seq += 1
            self.records.append((self.seq, {"timestamp": int(record.created * 1000), "level": record.levelname,
                                             "replica": record.threadName, "message": self.format(record)}))
            self.cv.notify_all()

    def wait_new(self, last: int, timeout: float) -> None:
        with self.cv:
            if self.seq <= last:
                self.cv.wait(timeout)


def gateway_summary(g) -> Dict[str, Any]:
    """A gateway as the application description lists it (the ``apps ui`` page reads
    these: id, type, topic, parameters, auth provider, chat / service options)."""
    out: Dict[str, Any] = {"id": g.id, "type": g.type, "topic": g.topic, "parameters": list(g.parameters or [])}
    if g.authentication is not None:
        out["authentication"] = {"provider": g.authentication.provider,
                                 "allow-test-mode": g.authentication.allow_test_mode}
    if g.chat_options is not None:
        out["chat-options"] = {"questions-topic": g.chat_options.questions_topic,
                               "answers-topic": g.chat_options.answers_topic}
    if g.service_options is not None:
        out["service-options"] = {"agent-id": g.service_options.agent_id,
                                  "input-topic": g.service_options.input_topic,
                                  "output-topic": g.service_options.output_topic}
    if g.events_topic:
        out["events-topic"] = g.events_topic
    return out


def _kv_list(items):
    if items is None:
        return None
    return [{"key": h.key, "value": h.value, "valueFromParameters": h.value_from_parameters,
             "valueFromAuthentication": h.value_from_authentication} for h in items]


def application_definition(app) -> Dict[str, Any]:
    """The application as the reference's description carries it
    (``ApplicationDescription.ApplicationDefinition``, ApplicationDescription.java:65-110):
    resources by id, modules with their topics and pipelines (agents with their
    connections, configuration as declared), gateways and the instance.  Placeholders stay
    as written; a dry run passes the resolved application."""
    def res(r):
        return None if r is None else {"parallelism": r.parallelism, "size": r.size}

    def err(e):
        return None if e is None else {"retries": e.retries, "on-failure": e.on_failure}

    def conn(c):
        return None if c is None else {"connectionType": c.connection_type, "definition": c.definition,
                                       "enableDeadletterQueue": bool(c.enable_dead_letter_queue)}

    def sch(x):
        return None if x is None else {"type": x.type, "schema": x.schema, "name": x.name}

    modules = []
    for m in app.modules.values():
        md: Dict[str, Any] = {"id": m.id}
        if m.pipelines:
            md["pipelines"] = [{
                "id": p.id, "module": p.module, "name": p.name, "resources": res(p.resources),
                "errors": err(p.errors),
                "agents": [{"id": a.id, "name": a.name, "type": a.type, "input": conn(a.input),
                            "output": conn(a.output), "configuration": a.configuration,
                            "resources": res(a.resources), "errors": err(a.errors)} for a in p.agents]}
                for p in m.pipelines.values()]
        if m.topics:
            md["topics"] = [{"name": t.name, "config": t.config or None, "options": t.options or None,
                             "keySchema": sch(t.key_schema), "valueSchema": sch(t.value_schema),
                             "partitions": t.partitions, "implicit": t.implicit, "creation-mode": t.creation_mode}
                            for t in m.topics.values()]
        modules.append(md)
    gws = []
    for g in app.gateways or []:
        d = gateway_summary(g)
        d["produceOptions"] = None if g.produce_options is None else {"headers": _kv_list(g.produce_options)}
        d["consumeOptions"] = None if g.consume_options is None else {
            "filters": {"headers": _kv_list(g.consume_options)}}
        gws.append(d)
    inst = app.instance
    return {
        "resources": {k: {"id": r.id, "name": r.name, "type": r.type, "configuration": r.configuration}
                      for k, r in app.resources.items()},
        "modules": modules,
        "gateways": {"gateways": gws} if app.gateways else None,
        "instance": None if inst is None else {
            "streamingCluster": None if inst.streaming_cluster is None else {
                "type": inst.streaming_cluster.type, "configuration": inst.streaming_cluster.configuration},
            "computeCluster": None if inst.compute_cluster is None else {
                "type": inst.compute_cluster.type, "configuration": inst.compute_cluster.configuration},
            "globals": inst.globals or None},
    }


def _topic_key(td) -> Dict[str, Any]:
    """What makes two topic definitions the same topic (``TopicDefinition`` equality)."""
    def sch(x):
        return None if x is None else (x.type, x.schema, x.name)
    return {"name": td.name, "creation-mode": td.creation_mode, "deletion-mode": td.deletion_mode,
            "implicit": td.implicit, "partitions": td.partitions, "key-schema": sch(td.key_schema),
            "value-schema": sch(td.value_schema), "options": td.options, "config": td.config}


def validate_topics_update(existing_plan, new_plan) -> None:
    """An update may not add, remove, rename or redefine a topic
    (``ApplicationService.validateTopicsUpdate``, ApplicationService.java:303-336)."""
    old = {t.name: t.definition for t in existing_plan.topics.values()}
    new = {t.name: t.definition for t in new_plan.topics.values()}
    if len(old) != len(new):
        raise ValueError(f"Detected a change in the topics which is not supported. New topics: {len(new)}. "
                         f"Existing topics: {len(old)}")
    for name, td in new.items():
        if name not in old:
            raise ValueError(f"Detected a change in the topics which is not supported. Topic {name} is not "
                             f"present in the existing application. Rename or adding new topics is not supported.")
        if _topic_key(td) != _topic_key(old[name]):
            raise ValueError(f"Detected a change in the topics which is not supported. Topic {name} has changed "
                             f"from: {_topic_key(old[name])} to: {_topic_key(td)}")


def validate_agents_update(existing_plan, new_plan) -> None:
    """An update keeps the same agents with the same type and connections; configuration,
    names and resources may change (``ApplicationService.validateAgentsUpdate``,
    ApplicationService.java:232-301)."""
    old, new = existing_plan.agents, new_plan.agents
    if len(old) != len(new):
        raise ValueError(f"Detected a change in the agents which is not supported. New agents: {len(new)}. "
                         f"Existing agents: {len(old)}")
    for key, n in new.items():
        o = old.get(key)
        if o is None:
            raise ValueError(f"Detected a change in the agents which is not supported. Agent {key} is not present "
                             f"in the existing application. Rename or adding new agents is not supported.")
        for field, a, b in (("type", o.agent_type, n.agent_type), ("type", o.component_type, n.component_type),
                            ("type", (o.metadata or {}).get("declared-type"), (n.metadata or {}).get("declared-type")),
                            ("input", o.input.name if o.input else None, n.input.name if n.input else None),
                            ("output", o.output.name if o.output else None, n.output.name if n.output else None)):
            if a != b:
                raise ValueError(f"Detected a change in the agents which is not supported. For agent {n.id} field "
                                 f"{field} changed from {getattr(a, 'value', a)} to {getattr(b, 'value', b)}")


class ControlPlane:
    """Application lifecycle independent of HTTP (also used by the CLI's local mode)."""

    def __init__(self, store: Optional[ApplicationStore] = None, code_dir: Optional[str] = None,
                 services=None, max_units_per_tenant: int = 0, code_storage=None,
                 default_tenant: Optional[str] = "default", max_units_limit: int = 0):
        """``default_tenant``: created at start when missing (``application.tenants.
        default-tenant.{create,name}``, LangStreamEventListener.java:35-45); ``max_units_limit``:
        the largest ``maxTotalResourceUnits`` a tenant may ask for (0 = no cap,
        ``maxTotalResourceUnitsLimit``); ``max_units_per_tenant``: the limit of a tenant that
        sets none (``defaultMaxTotalResourceUnits``)."""
        from ..core.codestorage import LocalDiskCodeStorage
        self.store = store or InMemoryApplicationStore(default_tenant)
        self.code_dir = code_dir or tempfile.mkdtemp(prefix="langstream-code-")
        os.makedirs(self.code_dir, exist_ok=True)
        # archives live in the code storage; code_dir only caches unpacked copies for local runners
        self.code_storage = code_storage or LocalDiskCodeStorage({"path": os.path.join(self.code_dir, "archives")})
        self.services = services
        self.max_units = max_units_per_tenant
        self.max_units_limit = max_units_limit
        if default_tenant and self.store.get_tenant(default_tenant) is None:
            self.store.put_tenant(default_tenant, {})
        self._logs: Dict[tuple, _AppLogBuffer] = {}
        self.archetypes_dir: Optional[str] = None
        self.only_agents: Optional[List[str]] = None   # `run --only-agent`: local runners start only these
        # `run`: agents always run here, whatever the instance's compute cluster (the
        # runtime-tester deploys through the k8s path into a mock API server, then runs
        # every agent pod as a thread: TESTER/LocalApplicationRunner.java:214-272)
        self.local_runs = False

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def unzip(data: bytes, dest: str) -> Dict[str, str]:
        with zipfile.ZipFile(io.BytesIO(data)) as z:
            for n in z.namelist():
                p = os.path.normpath(os.path.join(dest, n))
                if not p.startswith(os.path.abspath(dest)):
                    raise ValueError(f"bad path in archive: {n}")
            z.extractall(dest)
        # the app may be at the root or inside a single top-level directory
        root = dest
        entries = [e for e in os.listdir(dest) if not e.startswith(".")]
        if not any(e.endswith(".yaml") for e in entries) and len(entries) == 1 and \
                os.path.isdir(os.path.join(dest, entries[0])):
            root = os.path.join(dest, entries[0])
        return {"__root__": root, **read_app_directory(root)}

    def tenant_limit(self, tenant: str) -> int:
        """The tenant's ``maxTotalResourceUnits`` when set (> 0), else the default
        (``ApplicationService.java:95-125``)."""
        cfg = self.store.get_tenant(tenant) or {}
        own = int(cfg.get("maxTotalResourceUnits") or cfg.get("max-total-resource-units") or 0)
        return own if own > 0 else self.max_units

    def _units(self, plan) -> int:
        return sum(int(n.resources.size or 1) * int(n.resources.parallelism or 1) for n in plan.agents.values())

    def check_resource_usage(self, tenant: str, app_id: str, plan,
                             usage: Optional[Dict[str, int]] = None) -> None:
        """``ApplicationService.checkResourceUsage`` (ApplicationService.java:98-119): the
        plan's units (size x parallelism per agent) plus the tenant's other applications'
        must fit the tenant limit; ``usage`` (application id -> units) defaults to what
        the stored applications request."""
        limit = self.tenant_limit(tenant)
        if limit <= 0:
            return
        current = (sum(u for a, u in usage.items() if a != app_id) if usage is not None
                   else self._tenant_units(tenant, exclude=app_id))
        if limit < current + self._units(plan):
            raise PermissionError(f"Not enough resources to deploy application {app_id}")

    def _tenant_units(self, tenant: str, exclude: Optional[str] = None) -> int:
        from ..core.deployer import ApplicationDeployer
        tot = 0
        for a in self.store.list(tenant):
            if a.application_id == exclude:
                continue
            try:
                tot += self._units(ApplicationDeployer().create_implementation(a.application_id, a.application))
            except Exception:  # noqa: BLE001
                pass
        return tot

    # ---------------------------------------------------------------- lifecycle
    def deploy(self, tenant: str, app_id: str, app_zip: Optional[bytes], instance: Optional[str],
               secrets: Optional[str], dry_run: bool = False, update: bool = False,
               files: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
        from ..core.deployer import ApplicationDeployer
        if self.store.get_tenant(tenant) is None:
            raise KeyError(f"tenant {tenant} not found")
        existing = self.store.get(tenant, app_id)
        if update and existing is None:
            raise KeyError(f"application {app_id} not found")
        if not update and existing is not None and not dry_run:
            raise FileExistsError(f"application {app_id} already exists")
        code_root, digest, archive = None, None, None
        if app_zip is not None:
            tmp = tempfile.mkdtemp(prefix="app-", dir=self.code_dir)
            unzipped = self.unzip(app_zip, tmp)
            code_root = unzipped.pop("__root__")
            if files is None:       # an archetype passes its own files beside its code archive
                files = unzipped
            digest = directory_digest(os.path.join(code_root, "python"))
        elif files is None:
            if existing is None:
                raise ValueError("missing application archive")
            files = existing.files
        instance = instance if instance is not None else (existing.instance if existing else None)
        secrets = secrets if secrets is not None else (existing.secrets if existing else None)
        info = build_application_instance(files, instance, secrets)
        plan = ApplicationDeployer().create_implementation(app_id, info.application)
        if update and existing is not None:
            old_plan = ApplicationDeployer().create_implementation(app_id, existing.application)
            validate_topics_update(old_plan, plan)
            validate_agents_update(old_plan, plan)
        self.check_resource_usage(tenant, app_id, plan)
        if dry_run:
            if code_root is not None:
                shutil.rmtree(tmp, ignore_errors=True)
            from ..core.placeholders import resolve_placeholders
            return application_definition(resolve_placeholders(info.application))
        if update and existing is not None and existing.code_archive_id and digest is not None:
            md = self.code_storage.describe_application_code(tenant, existing.code_archive_id)
            if md is not None and md.py_binaries_digest == digest:
                archive = existing.code_archive_id  # python code unchanged: keep the archive
        if code_root is not None:
            if archive is None:
                version = hashlib.sha256(app_zip).hexdigest()[:12]
                archive = self.code_storage.store_application_code(tenant, app_id, version, app_zip,
                                                                   digest).code_store_id
            dst = os.path.join(self.code_dir, archive)
            if not os.path.exists(dst):
                shutil.move(code_root, dst)
            shutil.rmtree(tmp, ignore_errors=True)
        if existing is not None and existing.runner is not None:
            existing.runner.stop(10)
        sa = StoredApplication(app_id, tenant, info.application, dict(files), instance, secrets,
                               archive or (existing.code_archive_id if existing else None), "DEPLOYING")
        if existing is not None:
            sa.created_at = existing.created_at
        self.store.put(sa)
        self._start(sa, plan)
        return self.describe(tenant, app_id)

    def _start(self, sa: StoredApplication, plan) -> None:
        cc = sa.application.instance.compute_cluster.type if sa.application.instance and \
            sa.application.instance.compute_cluster else "local"
        if cc == "kubernetes" and not self.local_runs:
            from ..core.k8s import render_manifests
            sa.manifests = render_manifests(plan, sa.tenant, sa.code_archive_id)
            sa.status = "DEPLOYED"
            self.store.put(sa)
            return
        from ..runtime.local import LocalApplicationRunner
        code = self.local_code(sa) if sa.code_archive_id else ""
        runner = LocalApplicationRunner(sa.application, application_id=sa.application_id, tenant=sa.tenant,
                                        code_directory=code, services=self.services, agents=self.only_agents)
        buf = _AppLogBuffer()
        buf.setFormatter(logging.Formatter("%(name)s %(message)s"))
        logging.getLogger().addHandler(buf)
        self._logs[(sa.tenant, sa.application_id)] = buf
        try:
            runner.start(wait=30)
            buf.threads = {f"agent-{n.id}" for n in plan.agents.values()}
            sa.runner = runner
            sa.status = "DEPLOYED"
        except Exception as e:  # noqa: BLE001
            log.exception("deploy failed")
            sa.status = "ERROR_DEPLOYING"
            sa.error = str(e)
        self.store.put(sa)

    def local_code(self, sa: StoredApplication) -> str:
        """Unpacked code directory of ``sa``'s archive (fetched from the code storage on a miss,
        e.g. after a control-plane restart)."""
        dst = os.path.join(self.code_dir, sa.code_archive_id)
        if not os.path.exists(dst):
            tmp = tempfile.mkdtemp(prefix="app-", dir=self.code_dir)
            root = self.unzip(self.code_storage.download_application_code(sa.tenant, sa.code_archive_id), tmp)
            shutil.move(root["__root__"], dst)
            shutil.rmtree(tmp, ignore_errors=True)
        return dst

    def delete(self, tenant: str, app_id: str, force: bool = False) -> None:
        sa = self.store.get(tenant, app_id)
        if sa is None:
            raise KeyError(f"application {app_id} not found")
        if sa.runner is not None:
            sa.runner.stop(10)
            try:
                from ..core.deployer import ApplicationDeployer
                ApplicationDeployer().cleanup(tenant, sa.runner.plan)
            except Exception:  # noqa: BLE001
                if not force:
                    log.warning("cleanup of %s failed", app_id)
        buf = self._logs.pop((tenant, app_id), None)
        if buf is not None:
            logging.getLogger().removeHandler(buf)
        self.store.delete(tenant, app_id)
        try:
            self.code_storage.delete_application(tenant, app_id)
        except Exception:  # noqa: BLE001
            log.warning("deleting the code archives of %s failed", app_id)

    def describe(self, tenant: str, app_id: str, stats: bool = False) -> Dict[str, Any]:
        sa = self.store.get(tenant, app_id)
        if sa is None:
            raise KeyError(f"application {app_id} not found")
        from ..core.deployer import ApplicationDeployer
        plan = ApplicationDeployer().create_implementation(app_id, sa.application)
        out = sa.summary()
        out["application"] = application_definition(sa.application)
        out["status"]["status"]["reason"] = getattr(sa, "error", None)
        agents = {}
        if sa.runner is not None and stats:
            agents = sa.runner.agent_info()
        out["status"]["agents"] = agents
        # ApplicationStatus.executors (the CLI's EXECUTORS / REPLICAS columns): one executor
        # per planned agent, its replicas RUNNING while this control plane runs them
        running = sa.runner is not None and sa.status == "DEPLOYED"
        execs = []
        for node in plan.agents.values():
            n = max(1, int(getattr(node.resources, "parallelism", 1) or 1))
            execs.append({"id": node.id, "status": {"status": sa.status, "reason": None},
                          "replicas": [{"id": f"{app_id}-{node.id}-{r}", "status": "RUNNING" if running else "UNKNOWN",
                                        "reason": None} for r in range(n)]})
        out["status"]["executors"] = execs
        if getattr(sa, "manifests", None):
            out["manifests"] = sa.manifests
        return out

    def logs(self, tenant: str, app_id: str):
        return self._logs.get((tenant, app_id))

    # ---------------------------------------------------------------- archetypes
    def get_archetype(self, archetype: str) -> Optional[Dict[str, Any]]:
        """``ArchetypeDefinition`` (ArchetypeDefinition.java): the archetype.yaml with every
        field of the reference's records present (null when unset)."""
        import yaml
        if not self.archetypes_dir:
            return None
        p = os.path.join(self.archetypes_dir, archetype, "archetype.yaml")
        if not os.path.exists(p):
            return None
        with open(p) as f:
            spec = (yaml.safe_load(f) or {}).get("archetype") or {}
        sections = [{"title": sec.get("title"), "description": sec.get("description"),
                     "parameters": [{"default": par.get("default"), "name": par.get("name"),
                                     "label": par.get("label"), "description": par.get("description"),
                                     "type": par.get("type"), "subtype": par.get("subtype"),
                                     "binding": par.get("binding"), "required": bool(par.get("required", False))}
                                    for par in sec.get("parameters") or []]}
                    for sec in spec.get("sections") or []]
        return {"archetype": {"id": spec.get("id", archetype), "title": spec.get("title"),
                              "labels": spec.get("labels"), "description": spec.get("description"),
                              "icon": spec.get("icon"), "sections": sections}}

    def list_archetypes(self) -> List[Dict[str, Any]]:
        """``ArchetypeBasicInfo`` of every archetype: id, title, labels, description, icon."""
        out = []
        if not self.archetypes_dir or not os.path.isdir(self.archetypes_dir):
            return out
        for d in sorted(os.listdir(self.archetypes_dir)):
            a = self.get_archetype(d)
            if a is not None:
                a = a["archetype"]
                out.append({"id": a["id"], "title": a["title"], "labels": a["labels"],
                            "description": a["description"], "icon": a["icon"]})
        return out

    def deploy_archetype(self, tenant: str, archetype: str, app_id: str, params: Dict[str, Any],
                         dry_run: bool = False) -> Dict[str, Any]:
        """ArchetypeResource.deployApplication: the deployed application's definition
        (placeholders resolved on a dry run, which deploys nothing)."""
        d = os.path.join(self.archetypes_dir or "", archetype)
        if not os.path.isdir(d):
            raise KeyError(f"archetype {archetype} not found")
        files, inst, sec = archetype_application_files(d, params)
        from ..cli.client import zip_directory   # ArchetypeService.buildArchetypeZip
        res = self.deploy(tenant, app_id, None if dry_run else zip_directory(d), inst, sec, files=files,
                          dry_run=dry_run)
        if dry_run:
            return res
        return application_definition(self.store.get(tenant, app_id).application)


# ---------------------------------------------------------------- HTTP layer
class WebServiceServer:
    def __init__(self, cp: ControlPlane, host: str = "127.0.0.1", port: int = 8090,
                 auth_secret: Optional[str] = None, security: Optional[Dict[str, Any]] = None,
                 authenticator=None):
        """``security``: ``application.security.token`` properties (``secret-key``,
        ``public-key``, ``public-alg``, ``auth-claim``, ``audience-claim``, ``audience``,
        ``admin-roles``, ``jwks-hosts-allowlist``, ``allow-kubernetes-service-accounts``,
        ``kubernetes-namespace-prefix``).  ``auth_secret``: shorthand for a raw HMAC secret
        with ``admin-roles`` from ``security`` (default ``["admin"]``)."""
        from urllib.parse import quote
        from .security import TokenAuthenticator, TokenProperties
        self.cp = cp
        self.host, self.port = host, port
        sec = dict(security or {})
        if auth_secret:
            sec.setdefault("secret-key", "data:," + quote(auth_secret, safe=""))
            sec.setdefault("admin-roles", ["admin"])
        self.auth = authenticator
        if self.auth is None and any(sec.get(k) for k in ("secret-key", "public-key", "jwks-hosts-allowlist",
                                                          "allow-kubernetes-service-accounts")):
            self.auth = TokenAuthenticator(TokenProperties.from_dict(sec))
        self._loop = None
        self._thread = None
        self._started = threading.Event()

    def make_app(self):
        from aiohttp import web

        from .security import AuthenticationError, Principal, route_policy

        @web.middleware
        async def auth_mw(request, handler):
            request["principal"] = None
            policy = route_policy(request.path, request.method)
            if self.auth is not None and policy != "public":
                # a missing or bad token leaves the request unauthenticated, which the
                # reference's security chain answers with 403 (TokenAuthFilter.java:66-108,
                # SecurityConfigurationTest.shouldBeForbiddenIfTokenIsInvalid)
                h = request.headers.get("Authorization", "")
                if not h.startswith("Bearer ") or len(h) <= len("Bearer "):
                    raise web.HTTPForbidden(text="Missing token")
                try:
                    # JWKS / issuer fetches may block: off the event loop
                    name = await self._off(self.auth.authenticate, h[len("Bearer "):])
                except AuthenticationError as e:
                    raise web.HTTPForbidden(text=str(e))
                principal = Principal(name, self.auth.is_admin(name))
                if policy == "admin" and not principal.admin:
                    raise web.HTTPForbidden(text="ROLE_ADMIN required")
                request["principal"] = principal
            try:
                return await handler(request)
            except KeyError as e:
                raise web.HTTPNotFound(text=str(e).strip("'"))
            except FileExistsError as e:
                raise web.HTTPConflict(text=str(e))
            except PermissionError as e:
                raise web.HTTPForbidden(text=str(e))
            except ValueError as e:
                raise web.HTTPBadRequest(text=str(e))

        app = web.Application(middlewares=[auth_mw], client_max_size=256 * 1024 * 1024)
        r = app.router
        r.add_get("/api/tenants", self.tenants)
        r.add_route("*", "/api/tenants/{tenant}", self.tenant)
        r.add_get("/api/applications/{tenant}", self.list_apps)
        r.add_route("*", "/api/applications/{tenant}/{id}", self.app)
        r.add_get("/api/applications/{tenant}/{id}/logs", self.app_logs)
        r.add_get("/api/applications/{tenant}/{id}/code", self.app_code)
        r.add_get("/api/applications/{tenant}/{id}/code/info", self.app_code_info)
        r.add_get("/api/applications/{tenant}/{id}/code/{ref}", self.app_code)
        r.add_get("/api/applications/{tenant}/{id}/code/{ref}/info", self.app_code_info)
        r.add_get("/api/archetypes/{tenant}", self.archetypes)
        r.add_get("/api/archetypes/{tenant}/{id}", self.archetype)
        r.add_post("/api/archetypes/{tenant}/{id}/applications/{app}", self.archetype_deploy)
        r.add_get("/management/health", lambda req: web.json_response({"status": "UP"}))
        r.add_get("/api/docs", self.docs)
        return app

    async def docs(self, request):
        from aiohttp import web
        from ..core.config_model import generate_docs
        return web.json_response(generate_docs())

    @staticmethod
    def _authorize(request) -> None:
        """``performAuthorization`` of ApplicationResource / ArchetypeResource."""
        from .security import authorize_tenant
        authorize_tenant(request.get("principal"), request.match_info["tenant"])

    async def _off(self, fn, *a, **kw):
        return await asyncio.get_running_loop().run_in_executor(None, lambda: fn(*a, **kw))

    async def tenants(self, request):
        from aiohttp import web
        return web.json_response(self.cp.store.list_tenants())

    async def tenant(self, request):
        """``TenantResource.java``: GET; POST creates (409 when it exists); PATCH updates
        (404 when missing); PUT creates or replaces; DELETE.  The body carries
        ``maxTotalResourceUnits`` (>= 0; 0 = the control plane's default limit)."""
        from aiohttp import web
        t = request.match_info["tenant"]
        if request.method == "GET":
            v = self.cp.store.get_tenant(t)
            if v is None:
                raise KeyError(f"tenant {t} not found")
            return web.json_response(v)
        if request.method in ("PUT", "POST", "PATCH"):
            body = (await request.json() if request.can_read_body else {}) or {}
            units = body.get("maxTotalResourceUnits", body.get("max-total-resource-units"))
            if units is not None and int(units) < 0:
                raise ValueError("maxTotalResourceUnits must be positive")
            lim = self.cp.max_units_limit   # GlobalMetadataService.validateMaxTotalResourceUnits
            if lim > 0 and units is not None and int(units) > lim:
                raise ValueError(f"Max total resource units limit is {lim}")
            existing = self.cp.store.get_tenant(t)
            if request.method == "POST" and existing is not None:
                raise FileExistsError("tenant already exists")
            if request.method == "PATCH" and existing is None:
                raise KeyError("tenant not found")
            cfg = dict(existing or {}) if request.method == "PATCH" else {}
            cfg.pop("name", None)
            cfg.pop("max-total-resource-units", None)
            if units is not None or request.method != "PATCH":
                cfg["maxTotalResourceUnits"] = int(units or 0)
            self.cp.store.put_tenant(t, cfg)
            return web.json_response(self.cp.store.get_tenant(t))
        if request.method == "DELETE":
            if not self.cp.store.delete_tenant(t):
                raise KeyError(f"tenant {t} not found")
            return web.json_response({})
        raise web.HTTPMethodNotAllowed(request.method, ["GET", "PUT", "POST", "PATCH", "DELETE"])

    async def list_apps(self, request):
        from aiohttp import web
        self._authorize(request)
        return web.json_response([a.summary() for a in self.cp.store.list(request.match_info["tenant"])])

    async def _parts(self, request) -> Dict[str, Any]:
        out: Dict[str, Any] = {}
        if not request.content_type.startswith("multipart/"):
            return out
        reader = await request.multipart()
        async for part in reader:
            data = await part.read()
            out[part.name] = data if part.name == "app" else data.decode()
        return out

    async def app(self, request):
        from aiohttp import web
        t, i = request.match_info["tenant"], request.match_info["id"]
        self._authorize(request)
        q = request.query
        if request.method == "GET":
            return web.json_response(await self._off(self.cp.describe, t, i, q.get("stats") == "true"),
                                     dumps=lambda o: json.dumps(o, default=str))
        if request.method in ("POST", "PATCH"):
            parts = await self._parts(request)
            res = await self._off(self.cp.deploy, t, i, parts.get("app"), parts.get("instance"),
                                  parts.get("secrets"), q.get("dry-run") == "true", request.method == "PATCH")
            return web.json_response(res, dumps=lambda o: json.dumps(o, default=str))
        if request.method == "DELETE":
            await self._off(self.cp.delete, t, i, q.get("force") == "true")
            return web.json_response({})
        raise web.HTTPMethodNotAllowed(request.method, ["GET", "POST", "PATCH", "DELETE"])

    async def app_logs(self, request):
        from aiohttp import web
        t, i = request.match_info["tenant"], request.match_info["id"]
        self._authorize(request)
        if self.cp.store.get(t, i) is None:
            raise KeyError(f"application {i} not found")
        buf = self.cp.logs(t, i)
        # ApplicationResource.getApplicationLogs: format=text (default: "[replica] message"
        # lines, coloured per replica) or json (NDJSON {timestamp, replica, message}); filter=
        # replica names (repeatable); follow=false (this server's extension) ends the stream
        fmt = request.query.get("format", "text")
        wanted = set(request.query.getall("filter", []))
        resp = web.StreamResponse(headers={"Content-Type": "application/x-ndjson" if fmt == "json"
                                           else "text/plain"})
        await resp.prepare(request)
        if buf is None:
            await resp.write_eof()
            return resp
        follow = request.query.get("follow", "true") != "false"
        colors = ("32", "33", "34", "35", "36", "37", "38")

        def line(r) -> str:
            if fmt == "json":
                return json.dumps({"timestamp": r["timestamp"], "replica": r["replica"], "message": r["message"]},
                                  separators=(",", ":"), ensure_ascii=False) + "\n"
            digits = "".join(ch for ch in str(r["replica"]).rsplit("-", 1)[-1] if ch.isdigit())
            color = colors[(int(digits) if digits else 0) % len(colors)]
            return f"\x1b[{color}m[{r['replica']}] {r['message']}\x1b[0m\n"
        last = 0
        loop = asyncio.get_running_loop()
        while True:
            with buf.cv:
                batch = [r for s, r in buf.records if s > last]
                last = buf.seq
            for r in batch:
                if wanted and r["replica"] not in wanted:
                    continue
                await resp.write(line(r).encode())
            if not follow:
                break
            await loop.run_in_executor(None, buf.wait_new, last, 1.0)
        await resp.write_eof()
        return resp

    async def app_code(self, request):
        from aiohttp import web
        self._authorize(request)
        sa = self.cp.store.get(request.match_info["tenant"], request.match_info["id"])
        if sa is None:
            raise KeyError("application not found")
        ref = request.match_info.get("ref") or sa.code_archive_id   # /code/{codeArchiveReference}
        if not ref or ref.startswith(".") or "/" in ref or "\\" in ref:
            raise KeyError("code not found")
        data = await self._off(self.cp.code_storage.download_application_code, sa.tenant, ref)
        return web.Response(body=data, content_type="application/zip", headers={
            "Content-Disposition": f'attachment; filename="{sa.tenant}-{sa.application_id}.zip"'})

    async def app_code_info(self, request):
        from aiohttp import web
        self._authorize(request)
        sa = self.cp.store.get(request.match_info["tenant"], request.match_info["id"])
        if sa is None:
            raise KeyError("application not found")
        ref = request.match_info.get("ref") or sa.code_archive_id
        md = self.cp.code_storage.describe_application_code(sa.tenant, ref) if ref else None
        return web.json_response({"code-archive-id": ref,
                                  "python-digest": md.py_binaries_digest if md else None})

    async def archetypes(self, request):
        from aiohttp import web
        self._authorize(request)
        return web.json_response(self.cp.list_archetypes())

    async def archetype(self, request):
        from aiohttp import web
        self._authorize(request)
        a = self.cp.get_archetype(request.match_info["id"])
        if a is None:
            raise KeyError("archetype not found")
        return web.json_response(a)

    async def archetype_deploy(self, request):
        from aiohttp import web
        self._authorize(request)
        params = await request.json() if request.can_read_body else {}
        res = await self._off(self.cp.deploy_archetype, request.match_info["tenant"], request.match_info["id"],
                              request.match_info["app"], params or {},
                              request.query.get("dry-run", "false").lower() == "true")
        return web.json_response(res, dumps=lambda o: json.dumps(o, default=str))

    def start(self) -> "WebServiceServer":
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

        self._thread = threading.Thread(target=run, daemon=True, name="webservice")
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
        fut = asyncio.run_coroutine_threadsafe(self._runner.cleanup(), self._loop)
        try:
            fut.result(10)
        except Exception:  # noqa: BLE001
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)
        self._thread.join(10)

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"
