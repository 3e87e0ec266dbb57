"""Kubernetes compute-cluster runtime: plan -> manifests.

Parity: ``K8SRT/KubernetesClusterRuntime.java:93-380`` (one Secret with the
RuntimePodConfiguration + one ``Agent`` custom resource per plan agent),
``DEPL/agents/AgentResourcesFactory.java:98-586`` (StatefulSet with replicas =
parallelism (max 8), parallel pod management, code-download init containers, the
``agent-runtime`` container on ports 8080 (http) / 8000 (service), probes on
``/metrics``, CPU = size x 0.5, memory = size x 512M, PVCs for agent disks, headless
Service) and the CRD shapes of ``helm/crds``.

MI355X deployment additions: each replica is one process per GPU -- the container
requests ``amd.com/gpu: 1`` when the agent uses a GPU service (embeddings / completions /
vector store) and the pod sets ``HIP_VISIBLE_DEVICES`` through the device plugin; a
tensor-parallel chat agent (``tp`` > 1 in its resource) requests ``tp`` GPUs on one node
and runs ``torchrun --nproc-per-node tp``.

Manifests are returned as plain dicts (``kubectl apply -f -`` ready once dumped to
YAML); ``apply_manifests`` shells out to kubectl when it exists.
"""
from __future__ import annotations

import base64
import hashlib
import json
import re
import shutil
import subprocess
from typing import Any, Dict, List, Optional

from .planner import AgentNode, ExecutionPlan

MAX_REPLICAS = 8
GPU_AGENT_TYPES = ("ai-tools", "compute-ai-embeddings", "ai-chat-completions", "ai-text-completions",
                   "query-vector-db", "vector-db-sink", "re-rank", "composite-agent")
DEFAULT_IMAGE = "langstream-amd/runtime:latest"


def _uses_gpu(node: AgentNode) -> bool:
    if node.agent_type in ("ai-tools", "composite-agent"):
        txt = json.dumps(node.configuration)
        return any(t in txt for t in ("compute-ai-embeddings", "ai-chat-completions", "ai-text-completions",
                                      "query", "vector"))
    return node.agent_type in GPU_AGENT_TYPES


MAX_APPLICATION_ID_LENGTH = 20
MAX_AGENT_ID_LENGTH = 37
_RESOURCE_NAME = re.compile(r"^([a-z])[-a-z0-9]+$")


def validate_application_id(app_id: str) -> None:
    """``AppResourcesFactory.validateApplicationId`` (AppResourcesFactory.java:588-606):
    the id names the Application resource and every agent's."""
    if len(app_id) <= 1:
        raise ValueError(f"Application id '{app_id}' is too short. Must be at least 2 characters long.")
    if not _RESOURCE_NAME.match(app_id):
        raise ValueError(f"Application id '{app_id}' contains illegal characters. Allowed characters are "
                         f"alphanumeric and dash.")
    if len(app_id) > MAX_APPLICATION_ID_LENGTH:
        raise ValueError(f"Application id '{app_id}' is too long, max length is {MAX_APPLICATION_ID_LENGTH}")


def validate_agent_id(agent_id: str, app_id: str) -> None:
    """``AgentResourcesFactory.validateAgentId`` (AgentResourcesFactory.java:859-873): the
    custom resource ``<app>-<agent>`` must be a valid resource name."""
    full = f"{app_id}-{agent_id}"
    if not _RESOURCE_NAME.match(full):
        raise ValueError(f"Agent id '{agent_id}' (computed as '{full}') contains illegal characters. Allowed "
                         f"characters are alphanumeric and dash. To fully control the agent id, you can set the "
                         f"'id' field.")
    if len(agent_id) > MAX_AGENT_ID_LENGTH:
        raise ValueError(f"Agent id '{agent_id}' is too long, max length is {MAX_AGENT_ID_LENGTH}. To fully control "
                         f"the agent id, you can set the 'id' field.")


def validate_execution_plan(plan: ExecutionPlan) -> None:
    """``KubernetesClusterRuntime.validateExecutionPlan`` (KubernetesClusterRuntime.java:381-391)."""
    validate_application_id(plan.application_id)
    for node in plan.agents.values():
        validate_agent_id(node.id, plan.application_id)


def _name(s: str) -> str:
    return "".join(c if c.isalnum() or c == "-" else "-" for c in s.lower()).strip("-")[:63]


def agent_pod_configuration(plan: ExecutionPlan, node: AgentNode, tenant: str) -> Dict[str, Any]:
    inst = plan.application.instance
    sc = inst.streaming_cluster if inst is not None else None
    inp: Dict[str, Any] = {}
    if node.input is not None:
        inp = node.input.consumer_configuration()
        if node.input.deadletter is not None:
            inp["deadLetterTopicProducer"] = node.input.deadletter.producer_configuration()
    return {
        "input": inp,
        "output": node.output.producer_configuration() if node.output is not None else {},
        "agent": {"componentType": node.component_type.value, "tenant": tenant, "agentId": node.id,
                  "applicationId": plan.application_id, "agentType": node.agent_type,
                  "configuration": node.configuration,
                  "errorHandlerConfiguration": {"retries": node.errors.retries or 0,
                                                "onFailure": node.errors.on_failure or "fail"},
                  "agentsWithDisk": sorted(node.disks)},
        "streamingCluster": {"type": sc.type, "configuration": sc.configuration} if sc else None,
    }


def render_agent_resources(plan: ExecutionPlan, tenant: str, code_archive_id: Optional[str] = None,
                           image: str = DEFAULT_IMAGE, namespace_prefix: str = "langstream-") -> List[Dict[str, Any]]:
    """What the deployer job of the reference produces (``KubernetesClusterRuntime.java:93-140``):
    per plan agent a Secret holding the RuntimePodConfiguration and an ``Agent`` custom
    resource carrying everything the agent controller needs to build the workload."""
    ns = f"{namespace_prefix}{tenant}"
    out: List[Dict[str, Any]] = []
    app = _name(plan.application_id)
    for node in plan.agents.values():
        agent = _name(f"{plan.application_id}-{node.id}")
        size = int(node.resources.size or 1)
        replicas = max(1, min(MAX_REPLICAS, int(node.resources.parallelism or 1)))
        tp = int(getattr(node.resources, "tp", 1) or 1)
        secret_name = f"{agent}-config"
        pod_cfg = agent_pod_configuration(plan, node, tenant)
        cfg_b64 = base64.b64encode(json.dumps(pod_cfg).encode()).decode()
        out.append({"apiVersion": "v1", "kind": "Secret", "metadata": {"name": secret_name, "namespace": ns},
                    "data": {"app-config": cfg_b64}})
        out.append({"apiVersion": "langstream.ai/v1alpha1", "kind": "Agent",
                    "metadata": {"name": agent, "namespace": ns, "labels": {"app.kubernetes.io/name": app}},
                    "spec": {"agentId": node.id, "applicationId": plan.application_id, "tenant": tenant,
                             "agentConfigSecretRef": secret_name,
                             "agentConfigSecretRefChecksum": hashlib.sha256(cfg_b64.encode()).hexdigest()[:16],
                             "codeArchiveId": code_archive_id, "image": image,
                             "resources": {"parallelism": replicas, "size": size, "tp": tp,
                                           "gpus": tp if _uses_gpu(node) else 0},
                             "options": {"disks": [{"agentId": k, "size": v.size, "type": v.type}
                                                   for k, v in node.disks.items()]}}})
    return out


def render_agent_workload(agent_cr: Dict[str, Any]) -> List[Dict[str, Any]]:
    """Agent CR -> StatefulSet + headless Service (``DEPL/agents/AgentResourcesFactory.java:98-586``):
    replicas = parallelism, parallel pod management, the code-download init container,
    ``agent-runtime`` on 8080/8000, probes on /metrics, CPU = size x 0.5, memory =
    size x 512M, one PVC template per agent disk; GPUs as ``amd.com/gpu``."""
    md, spec = agent_cr["metadata"], agent_cr["spec"]
    ns, agent = md["namespace"], md["name"]
    app = _name(spec["applicationId"])
    res = spec.get("resources") or {}
    size = int(res.get("size") or 1)
    replicas = max(1, min(MAX_REPLICAS, int(res.get("parallelism") or 1)))
    tp, gpus = int(res.get("tp") or 1), int(res.get("gpus") or 0)
    image = spec.get("image") or DEFAULT_IMAGE
    secret_name = spec["agentConfigSecretRef"]
    disks = (spec.get("options") or {}).get("disks") or []
    limits = {"cpu": f"{size * 0.5:g}", "memory": f"{size * 512}M"}
    if gpus:
        limits["amd.com/gpu"] = str(gpus)
    cmd = ["python", "-m", "langstream_amd.runtime.pod", "/app-config/config"]
    if tp > 1:
        cmd = ["torchrun", "--nnodes=1", f"--nproc-per-node={tp}", "--master-addr=127.0.0.1", "-m",
               "langstream_amd.runtime.pod", "/app-config/config"]
    container = {
        "name": "agent-runtime", "image": image, "command": cmd,
        "ports": [{"name": "http", "containerPort": 8080}, {"name": "service", "containerPort": 8000}],
        "env": [{"name": "LANGSTREAM_AGENT_RUNNER_POD_CONFIGURATION", "value": "/app-config/config"},
                {"name": "LANGSTREAM_AGENT_RUNNER_CODE_PATH", "value": "/app-code-download"},
                {"name": "LANGSTREAM_AGENT_RUNNER_PERSISTENT_STATE_DIRECTORY", "value": "/persistent-state"},
                {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
        "resources": {"requests": dict(limits), "limits": limits},
        "livenessProbe": {"httpGet": {"path": "/metrics", "port": 8080}, "initialDelaySeconds": 10,
                          "periodSeconds": 30, "timeoutSeconds": 5},
        "readinessProbe": {"httpGet": {"path": "/metrics", "port": 8080}, "initialDelaySeconds": 10,
                           "periodSeconds": 30, "timeoutSeconds": 5},
        "volumeMounts": [{"name": "app-config", "mountPath": "/app-config"},
                         {"name": "code-download", "mountPath": "/app-code-download"}]
                        + [{"name": _name(f"{d['agentId']}-disk"), "mountPath": f"/persistent-state/{d['agentId']}"}
                           for d in disks],
    }
    init = [{"name": "code-download", "image": image,
             "command": ["python", "-m", "langstream_amd.cli", "code-download", "--tenant", spec["tenant"],
                         "--application", spec["applicationId"], "--code-archive-id",
                         str(spec.get("codeArchiveId")), "--target", "/app-code-download"],
             # the code storage config (same as the control plane's) comes from an optional
             # secret; without it the archive is fetched through the control plane
             "env": [{"name": "LANGSTREAM_CODE_STORAGE",
                      "valueFrom": {"secretKeyRef": {"name": "langstream-code-storage", "key": "config",
                                                     "optional": True}}}],
             "volumeMounts": [{"name": "code-download", "mountPath": "/app-code-download"}]}]
    sts = {
        "apiVersion": "apps/v1", "kind": "StatefulSet",
        "metadata": {"name": agent, "namespace": ns,
                     "labels": {"app": agent, "langstream-application": app, "langstream-agent": spec["agentId"]}},
        "spec": {"replicas": replicas, "podManagementPolicy": "Parallel", "serviceName": agent,
                 "selector": {"matchLabels": {"app": agent}},
                 "template": {"metadata": {"labels": {"app": agent},
                                           "annotations": {"langstream.ai/config-checksum":
                                                           str(spec.get("agentConfigSecretRefChecksum", ""))}},
                              "spec": {"initContainers": init, "containers": [container],
                                       "terminationGracePeriodSeconds": 60,
                                       "volumes": [{"name": "app-config", "secret": {
                                           "secretName": secret_name,
                                           "items": [{"key": "app-config", "path": "config"}]}},
                                           {"name": "code-download", "emptyDir": {}}]}},
                 "volumeClaimTemplates": [
                     {"metadata": {"name": _name(f"{d['agentId']}-disk")},
                      "spec": {"accessModes": ["ReadWriteOnce"],
                               "resources": {"requests": {"storage": d.get("size") or "256M"}},
                               **({"storageClassName": d["type"]} if d.get("type") and d["type"] != "default"
                                  else {})}}
                     for d in disks]}}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": agent, "namespace": ns},
           "spec": {"clusterIP": "None", "selector": {"app": agent},
                    "ports": [{"name": "http", "port": 8080}, {"name": "service", "port": 8000}]}}
    return [sts, svc]


def render_manifests(plan: ExecutionPlan, tenant: str, code_archive_id: Optional[str] = None,
                     image: str = DEFAULT_IMAGE, namespace_prefix: str = "langstream-") -> List[Dict[str, Any]]:
    """Everything at once (no operator): Secret + Agent CR + StatefulSet + Service per agent."""
    out: List[Dict[str, Any]] = []
    res = render_agent_resources(plan, tenant, code_archive_id, image, namespace_prefix)
    for i in range(0, len(res), 2):
        out += res[i: i + 2]
        out += render_agent_workload(res[i + 1])
    return out


def to_yaml(manifests: List[Dict[str, Any]]) -> str:
    import yaml
    return yaml.safe_dump_all(manifests, sort_keys=False)


def apply_manifests(manifests: List[Dict[str, Any]]) -> bool:
    kubectl = shutil.which("kubectl")
    if kubectl is None:
        return False
    subprocess.run([kubectl, "apply", "-f", "-"], input=to_yaml(manifests).encode(), check=True)
    return True
