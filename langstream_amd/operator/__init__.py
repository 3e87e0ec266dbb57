"""LangStream Kubernetes operator: reconciles ``Application``
and ``Agent`` custom resources.

Parity with the reference operator (``OPER/controllers/apps/AppController.java:97-190``,
``OPER/controllers/agents/AgentController.java``, ``OPER/TenantLimitsChecker.java``):
* AppController: a new or changed Application (spec generation != status.observedGeneration)
  is "set up" (topics + assets: ``ApplicationDeployer.setup``) and "deployed" (Agent CRs +
  config Secrets).  With ``use_jobs`` (the default of ``main``) both run as Kubernetes
  Jobs like the reference's (RT/application/ApplicationSetupRunner.java:30-139,
  RT/deployer/RuntimeDeployer.java): ``langstream-runtime-setup-<app>-<gen>`` then
  ``langstream-runtime-deployer-<app>-<gen>`` (``runtime/jobs.py``), the controller
  advancing on each Job's completion (ERROR_SETUP / ERROR_DEPLOYING on failure); without
  it they run in-process (tests, single-binary mode).  A finalizer holds deletion until the cleanup ran: Agent CRs deleted, then the
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


def deploy_agents(kube: KubeClient, app_cr: Dict[str, Any], plan, tenant: str, image: str) -> None:
    """The deployer step: config Secrets + Agent CRs of the plan (owned by the Application)
    and removal of the app's Agents that left the plan."""
    md = app_cr["metadata"]
    ns, name = md["namespace"], md["name"]
    resources = render_agent_resources(plan, tenant, app_cr["spec"].get("codeArchiveId"), image, namespace_prefix="")
    wanted = set()
    for obj in resources:
        obj["metadata"]["namespace"] = ns
        obj["metadata"]["ownerReferences"] = [owner_ref(app_cr)]
        kube.apply(obj)
        if obj["kind"] == "Agent":
            wanted.add(obj["metadata"]["name"])
    for a in kube.list(CR_API, "Agent", ns):
        if a["spec"].get("applicationId") == name and a["metadata"]["name"] not in wanted:
            kube.delete(CR_API, "Agent", ns, a["metadata"]["name"])


def delete_agents(kube: KubeClient, namespace: str, app_name: str) -> None:
    for a in kube.list(CR_API, "Agent", namespace):
        if a["spec"].get("applicationId") == app_name:
            kube.delete(CR_API, "Agent", namespace, a["metadata"]["name"])
            kube.delete("v1", "Secret", namespace, a["spec"].get("agentConfigSecretRef", ""))


def _job_state(job: Optional[Dict[str, Any]]) -> Optional[str]:
    if job is None:
        return None
    st = job.get("status") or {}
    if int(st.get("succeeded") or 0) >= 1:
        return "succeeded"
    for c in st.get("conditions") or []:
        if c.get("type") == "Failed" and c.get("status") == "True":
            return "failed"
    if int(st.get("failed") or 0) > int((job.get("spec") or {}).get("backoffLimit", 0)):
        return "failed"
    return "running"


class AppController:
    def __init__(self, kube: KubeClient, image: str = "langstream-amd/runtime:latest",
                 system_namespace: str = "langstream", use_jobs: bool = False,
                 service_account: str = "langstream-deployer"):
        self.kube = kube
        self.image = image
        self.system_namespace = system_namespace
        self.deployer = ApplicationDeployer()
        self.use_jobs = use_jobs
        self.service_account = service_account

    # ------------------------------------------------------------------ jobs
    @staticmethod
    def _job_name(kind: str, app: str, gen: int) -> str:
        return f"langstream-runtime-{kind}-{app}-{gen}"[:63].rstrip("-")

    def _job_config(self, app_cr: Dict[str, Any]) -> str:
        """The Secret every Job of this app mounts at /app-config/config."""
        from .store import read_app_secrets
        md = app_cr["metadata"]
        name = f"langstream-runtime-config-{md['name']}"[:63]
        import base64
        cfg = {"applicationId": md["name"], "namespace": md["namespace"], "tenant": app_cr["spec"].get("tenant"),
               "application": _spec_files(app_cr),
               "secrets": read_app_secrets(self.kube, md["namespace"], md["name"]),
               "codeArchiveId": app_cr["spec"].get("codeArchiveId"), "image": self.image}
        self.kube.apply({"apiVersion": "v1", "kind": "Secret",
                         "metadata": {"name": name, "namespace": md["namespace"],
                                      "ownerReferences": [owner_ref(app_cr)]},
                         "data": {"config": base64.b64encode(json.dumps(cfg).encode()).decode()}})
        return name

    def _start_job(self, app_cr: Dict[str, Any], job: str, entry: str, phase: str, cfg_secret: str) -> None:
        md = app_cr["metadata"]
        self.kube.apply({
            "apiVersion": "batch/v1", "kind": "Job",
            "metadata": {"name": job, "namespace": md["namespace"], "ownerReferences": [owner_ref(app_cr)],
                         "labels": {"app.kubernetes.io/name": md["name"], "langstream.ai/job": entry}},
            "spec": {"backoffLimit": 1, "ttlSecondsAfterFinished": 3600, "template": {"spec": {
                "restartPolicy": "Never", "serviceAccountName": self.service_account,
                "containers": [{"name": entry, "image": self.image,
                                "command": ["python", "-m", "langstream_amd.runtime.jobs", entry,
                                            "/app-config/config"],
                                "env": [{"name": "LANGSTREAM_JOB_PHASE", "value": phase}],
                                "volumeMounts": [{"name": "app-config", "mountPath": "/app-config"}]}],
                "volumes": [{"name": "app-config", "secret": {"secretName": cfg_secret}}]}}}})

    def _run_jobs(self, app_cr: Dict[str, Any], steps, done_phase: str, gen: int) -> Optional[str]:
        """Advance a chain of (kind, entry, phase, error-phase) Jobs by one reconcile pass;
        returns the app phase to report, or None when the chain completed."""
        md = app_cr["metadata"]
        cfg = self._job_config(app_cr)
        for kind, entry, phase, err_phase in steps:
            job = self._job_name(kind, md["name"], gen)
            st = _job_state(self.kube.get("batch/v1", "Job", md["namespace"], job))
            if st is None:
                self._start_job(app_cr, job, entry, phase, cfg)
                return done_phase
            if st == "running":
                return done_phase
            if st == "failed":
                return err_phase
        return None

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
            if self.use_jobs:
                phase = self._run_jobs(app_cr, [("setup", "application-setup", "setup", "ERROR_SETUP"),
                                                ("deployer", "deployer-runtime", "deploy", "ERROR_DEPLOYING")],
                                       "DEPLOYING", gen)
                if phase is not None:
                    if phase.startswith("ERROR"):
                        self._status(app_cr, phase, f"{phase.lower()} job failed", observed=gen)
                    elif (status.get("status") or {}).get("status") != "DEPLOYING":
                        self._status(app_cr, "DEPLOYING")
                    return phase
                self._status(app_cr, "DEPLOYED", observed=gen)
                return "DEPLOYED"
            self._status(app_cr, "DEPLOYING")
            self.deployer.setup(tenant, plan)                       # setup step: topics + assets
            deploy_agents(self.kube, app_cr, plan, tenant, self.image)   # deployer step
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
        if self.use_jobs:   # deployer-cleanup then setup-cleanup Jobs (the reference's order)
            phase = self._run_jobs(app_cr, [("deployer-cleanup", "deployer-runtime", "delete", "ERROR_DELETING"),
                                            ("setup-cleanup", "application-setup", "cleanup", "ERROR_DELETING")],
                                   "DELETING", int(md.get("generation", 1)))
            if phase is not None:
                return phase
        else:
            delete_agents(self.kube, ns, name)                      # deployer cleanup
            try:                                                    # setup cleanup
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
    ap.add_argument("--in-process", action="store_true", help="run setup / deployer in the operator, not as Jobs")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    op = Operator(KubeClient(a.api_server, a.token), a.namespace, a.resync, image=a.image,
                  use_jobs=not a.in_process)
    try:
        op.run()
    except KeyboardInterrupt:
        op.stop()
    return 0
