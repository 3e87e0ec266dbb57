"""LangStream Kubernetes operator: reconciles ``Application``
and ``Agent`` custom resources.

Parity with the reference operator (``OPER/controllers/apps/AppController.java:97-190``,
``OPER/controllers/agents/AgentController.java``, ``OPER/TenantLimitsChecker.java``):
* AppController: a new or changed Application (spec generation != status.observedGeneration)
  is "set up" (topics + assets: ``ApplicationDeployer.setup``, the reference's setup Job)
  and "deployed" (Agent CRs + config Secrets: the deployer Job); both run in-process
  here.  A finalizer holds deletion until the cleanup ran: Agent CRs deleted, then the
  topics/assets with ``deletion-mode: delete`` removed (deployer-cleanup, then
  setup-cleanup).  ``options.markedForDeletion`` triggers the same cleanup and then deletes
  the CR.  Agents that vanished from the plan are deleted.  Status phases
  DEPLOYING -> DEPLOYED | ERROR_DEPLOYING, DELETING.
* Tenant limits: the sum of ``size x parallelism`` over a tenant's agents must fit the
  tenant's ``maxTotalResourceUnits`` (ConfigMap ``langstream-tenant-limits`` key = tenant),
  else the app goes to ERROR_DEPLOYING with the reason.
* AgentController: Agent CR -> StatefulSet + headless Service (``core/k8s.py``
  ``render_agent_workload``) with owner references, so Kubernetes garbage-collects them
  with the Agent; status reflects the StatefulSet's ready replicas.
The loop is level-triggered (list + reconcile every ``resync`` seconds), which needs no
watch bookkeeping and converges after restarts.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from typing import Any, Dict, List, Optional

from ..core.deployer import ApplicationDeployer
from ..core.k8s import render_agent_resources, render_agent_workload
from ..core.parser import build_application_instance
from .kube import CR_API, KubeClient, KubeError, owner_ref

log = logging.getLogger(__name__)

FINALIZER = "langstream.ai/cleanup"
LIMITS_CONFIGMAP = "langstream-tenant-limits"


def _spec_files(app_cr: Dict[str, Any]) -> Dict[str, Any]:
    raw = app_cr["spec"].get("application") or "{}"
    return json.loads(raw) if isinstance(raw, str) else raw


def _options(app_cr: Dict[str, Any]) -> Dict[str, Any]:
    raw = app_cr["spec"].get("options") or "{}"
    return json.loads(raw) if isinstance(raw, str) else raw


class AppController:
    def __init__(self, kube: KubeClient, image: str = "langstream-amd/runtime:latest",
                 system_namespace: str = "langstream"):
        self.kube = kube
        self.image = image
        self.system_namespace = system_namespace
        self.deployer = ApplicationDeployer()

    # ------------------------------------------------------------------ helpers
    def _plan(self, app_cr):
        from .store import read_app_secrets
        spec, md = app_cr["spec"], app_cr["metadata"]
        files = _spec_files(app_cr)
        secrets = read_app_secrets(self.kube, md["namespace"], md["name"])
        built = build_application_instance(files.get("files") or {}, files.get("instance"), secrets)
        app = getattr(built, "application", built)
        return self.deployer.create_implementation(md["name"], app), spec.get("tenant") or "default"

    def _status(self, app_cr, phase: str, reason: str = "", observed: Optional[int] = None) -> None:
        md = app_cr["metadata"]
        st: Dict[str, Any] = {"status": {"status": phase, "reason": reason}}
        if observed is not None:
            st["observedGeneration"] = observed
        self.kube.merge_patch(CR_API, "Application", md["namespace"], md["name"], {"status": st}, "status")

    def _tenant_limit(self, tenant: str) -> Optional[int]:
        cm = self.kube.get("v1", "ConfigMap", self.system_namespace, LIMITS_CONFIGMAP)
        v = ((cm or {}).get("data") or {}).get(tenant)
        return int(v) if v not in (None, "") else None

    def _units_used(self, namespace: str, exclude_app: str) -> int:
        used = 0
        for a in self.kube.list(CR_API, "Agent", namespace):
            if a["spec"].get("applicationId") == exclude_app:
                continue
            r = a["spec"].get("resources") or {}
            used += int(r.get("size") or 1) * int(r.get("parallelism") or 1)
        return used

    # ------------------------------------------------------------------ reconcile
    def reconcile(self, app_cr: Dict[str, Any]) -> str:
        md = app_cr["metadata"]
        ns, name = md["namespace"], md["name"]
        if md.get("deletionTimestamp") or _options(app_cr).get("markedForDeletion"):
            return self._cleanup(app_cr)
        if FINALIZER not in (md.get("finalizers") or []):
            self.kube.merge_patch(CR_API, "Application", ns, name,
                                  {"metadata": {"finalizers": (md.get("finalizers") or []) + [FINALIZER]}})
        gen = md.get("generation", 1)
        status = (app_cr.get("status") or {})
        if status.get("observedGeneration") == gen and (status.get("status") or {}).get("status") == "DEPLOYED":
            return "DEPLOYED"
        try:
            plan, tenant = self._plan(app_cr)
            limit = self._tenant_limit(tenant)
            if limit is not None:
                need = sum(int(n.resources.size or 1) * int(n.resources.parallelism or 1) for n in plan.agents.values())
                used = self._units_used(ns, name)
                if used + need > limit:
                    raise ValueError(f"Not enough resources to deploy application {name}: tenant {tenant} uses "
                                     f"{used} of {limit} units and the application needs {need}")
            self._status(app_cr, "DEPLOYING")
            self.deployer.setup(tenant, plan)                       # setup job: topics + assets
            resources = render_agent_resources(plan, tenant, app_cr["spec"].get("codeArchiveId"), self.image,
                                               namespace_prefix="")
            wanted = set()
            for obj in resources:                                   # deployer job: secrets + Agent CRs
                obj["metadata"]["namespace"] = ns
                obj["metadata"]["ownerReferences"] = [owner_ref(app_cr)]
                self.kube.apply(obj)
                if obj["kind"] == "Agent":
                    wanted.add(obj["metadata"]["name"])
            for a in self.kube.list(CR_API, "Agent", ns):           # agents removed from the plan
                if a["spec"].get("applicationId") == name and a["metadata"]["name"] not in wanted:
                    self.kube.delete(CR_API, "Agent", ns, a["metadata"]["name"])
            self._status(app_cr, "DEPLOYED", observed=gen)
            return "DEPLOYED"
        except Exception as e:  # noqa: BLE001
            log.exception("deploying %s/%s failed", ns, name)
            self._status(app_cr, "ERROR_DEPLOYING", str(e), observed=gen)
            return "ERROR_DEPLOYING"

    def _cleanup(self, app_cr: Dict[str, Any]) -> str:
        md = app_cr["metadata"]
        ns, name = md["namespace"], md["name"]
        try:
            self._status(app_cr, "DELETING")
        except KubeError:
            pass
        for a in self.kube.list(CR_API, "Agent", ns):               # deployer cleanup
            if a["spec"].get("applicationId") == name:
                self.kube.delete(CR_API, "Agent", ns, a["metadata"]["name"])
                self.kube.delete("v1", "Secret", ns, a["spec"].get("agentConfigSecretRef", ""))
        try:                                                        # setup cleanup
            plan, tenant = self._plan(app_cr)
            self.deployer.cleanup(tenant, plan)
        except Exception:  # noqa: BLE001
            log.exception("cleanup of topics/assets for %s/%s failed", ns, name)
        fins = [f for f in (md.get("finalizers") or []) if f != FINALIZER]
        self.kube.merge_patch(CR_API, "Application", ns, name, {"metadata": {"finalizers": fins}})
        if not md.get("deletionTimestamp"):
            self.kube.delete(CR_API, "Application", ns, name)
        return "DELETED"


class AgentController:
    def __init__(self, kube: KubeClient):
        self.kube = kube

    def reconcile(self, agent_cr: Dict[str, Any]) -> str:
        md = agent_cr["metadata"]
        if md.get("deletionTimestamp"):
            return "DELETING"  # owner references garbage-collect the workload
        for obj in render_agent_workload(agent_cr):
            obj["metadata"]["ownerReferences"] = [owner_ref(agent_cr)]
            self.kube.apply(obj)
        sts = self.kube.get("apps/v1", "StatefulSet", md["namespace"], md["name"]) or {}
        want = int(((agent_cr["spec"].get("resources") or {}).get("parallelism")) or 1)
        ready = int((sts.get("status") or {}).get("readyReplicas") or 0)
        phase = "DEPLOYED" if ready >= want else "DEPLOYING"
        self.kube.merge_patch(CR_API, "Agent", md["namespace"], md["name"],
                              {"status": {"status": phase, "readyReplicas": ready, "replicas": want}}, "status")
        return phase


class Operator:
    def __init__(self, kube: KubeClient, namespace: Optional[str] = None, resync: float = 5.0, **kw):
        self.kube = kube
        self.namespace = namespace
        self.resync = resync
        self.apps = AppController(kube, **kw)
        self.agents = AgentController(kube)
        self._stop = threading.Event()

    def reconcile_all(self) -> Dict[str, str]:
        out = {}
        for a in self.kube.list(CR_API, "Application", self.namespace):
            out[f"app/{a['metadata']['namespace']}/{a['metadata']['name']}"] = self.apps.reconcile(a)
        for a in self.kube.list(CR_API, "Agent", self.namespace):
            out[f"agent/{a['metadata']['namespace']}/{a['metadata']['name']}"] = self.agents.reconcile(a)
        return out

    def run(self) -> None:
        while not self._stop.is_set():
            try:
                self.reconcile_all()
            except Exception:  # noqa: BLE001
                log.exception("reconcile loop")
            self._stop.wait(self.resync)

    def stop(self) -> None:
        self._stop.set()


def main(argv: Optional[List[str]] = None) -> int:
    import argparse
    ap = argparse.ArgumentParser(description="LangStream (MI355X) Kubernetes operator")
    ap.add_argument("--api-server", default=None, help="API server URL (default: in-cluster)")
    ap.add_argument("--token", default=None)
    ap.add_argument("--namespace", default=None, help="watch one namespace (default: all)")
    ap.add_argument("--image", default="langstream-amd/runtime:latest")
    ap.add_argument("--resync", type=float, default=5.0)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    op = Operator(KubeClient(a.api_server, a.token), a.namespace, a.resync, image=a.image)
    try:
        op.run()
    except KeyboardInterrupt:
        op.stop()
    return 0
