"""ApplicationDeployer (CORE/deploy/ApplicationDeployer.java:58-249).

* create_implementation = resolve placeholders, then build the execution plan;
* setup   = create topics (TopicConnectionsRuntime.deploy) + assets (create-if-not-exists);
* deploy  / delete = hand the plan to the compute cluster;
* cleanup = delete topics and assets whose deletion-mode is ``delete``.
Also turns plan nodes into RuntimePodConfiguration (K8SRT/KubernetesClusterRuntime.java:249-380).
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

from ..api.model import Application
from ..api.topics import TopicConnectionsRuntimeRegistry
from .placeholders import resolve_placeholders
from .planner import AgentNode, ExecutionPlan, Planner

log = logging.getLogger(__name__)


def referenced_resources(app: Application) -> set:
    """Ids / names of the resources the application's agents and assets use: any string in
    an agent's or asset's configuration naming a resource (``datasource``, ``ai-service``,
    step fields), plus the default AI service of agents that call a model without naming
    one (the first AI resource, as GenAIToolKitFunctionAgentProvider.java:210-290 picks)."""
    from .genai import AI_SERVICE_KEYS, AI_STEPS
    names = {k for k in app.resources} | {r.name for r in app.resources.values() if r.name} | \
            {r.id for r in app.resources.values() if r.id}
    used: set = set()

    def walk(v):
        if isinstance(v, str):
            if v in names:
                used.add(v)
        elif isinstance(v, dict):
            for x in v.values():
                walk(x)
        elif isinstance(v, (list, tuple)):
            for x in v:
                walk(x)
    needs_ai = False
    for m in app.modules.values():
        for p in m.pipelines.values():
            for a in p.agents:
                cfg = a.configuration or {}
                walk(cfg)
                steps = cfg.get("steps") if isinstance(cfg.get("steps"), list) else []
                kinds = [a.type] + [s.get("type") for s in steps if isinstance(s, dict)]
                if any(k in AI_STEPS for k in kinds) and "ai-service" not in cfg:
                    needs_ai = True
        for asset in m.assets:
            walk(asset.config)
    if needs_ai:
        for k, r in app.resources.items():
            if r.type in AI_SERVICE_KEYS:
                used.add(k)
                break
    return used


class ApplicationDeployer:
    def __init__(self, compute_cluster=None, planner: Optional[Planner] = None):
        self.compute_cluster = compute_cluster
        self.planner = planner or Planner()

    def create_implementation(self, application_id: str, application: Application) -> ExecutionPlan:
        """Resources are validated when an agent or asset uses them (the reference builds a
        resource's configuration only through ``getResourceImplementation``, called by the
        agent / asset providers: BasicClusterRuntime.java:150-157); an unused resource is not
        looked at, whatever its type (ApplicationDeployerTest.testDeploy)."""
        from .resources import validate_resource
        resolved = resolve_placeholders(application)
        used = referenced_resources(resolved)
        for key, r in resolved.resources.items():
            if key in used or r.id in used or r.name in used:
                validate_resource(r)
        return self.planner.build_execution_plan(application_id, resolved)

    def setup(self, tenant: str, plan: ExecutionPlan) -> None:
        inst = plan.application.instance
        sc = inst.streaming_cluster if inst is not None else None
        if sc is not None:
            rt = TopicConnectionsRuntimeRegistry.get(sc)
            rt.deploy(plan)
        from ..agents.assets import AssetManagerRegistry
        for asset in plan.assets:
            mgr = AssetManagerRegistry.create(asset)
            if asset.creation_mode == "create-if-not-exists" and not mgr.asset_exists():
                log.info("creating asset %s (%s)", asset.id, asset.asset_type)
                mgr.deploy_asset()

    def deploy(self, tenant: str, plan: ExecutionPlan, code_archive_id: Optional[str] = None):
        if self.compute_cluster is None:
            raise ValueError("no compute cluster configured")
        return self.compute_cluster.deploy(tenant, plan, code_archive_id)

    def delete(self, tenant: str, plan: ExecutionPlan, code_archive_id: Optional[str] = None) -> None:
        if self.compute_cluster is not None:
            self.compute_cluster.delete(tenant, plan, code_archive_id)

    def cleanup(self, tenant: str, plan: ExecutionPlan) -> None:
        inst = plan.application.instance
        sc = inst.streaming_cluster if inst is not None else None
        if sc is not None:
            TopicConnectionsRuntimeRegistry.get(sc).delete(plan)
        from ..agents.assets import AssetManagerRegistry
        for asset in plan.assets:
            if asset.deletion_mode == "delete":
                AssetManagerRegistry.create(asset).delete_asset_if_exists()


def pod_configuration(plan: ExecutionPlan, node: AgentNode, tenant: str = "default",
                      code_directory: str = "", state_dir: Optional[str] = None, replica: int = 0):
    from ..runtime.runner import RuntimePodConfiguration
    inst = plan.application.instance
    sc = inst.streaming_cluster if inst is not None else None
    inp: Dict[str, Any] = {}
    if node.input is not None:
        inp = node.input.consumer_configuration()
        if node.input.deadletter is not None:
            inp["deadLetterTopicProducer"] = node.input.deadletter.producer_configuration()
    out: Dict[str, Any] = node.output.producer_configuration() if node.output is not None else {}
    errors = {"retries": node.errors.retries or 0, "onFailure": node.errors.on_failure or "fail"}
    return RuntimePodConfiguration(
        agent_id=node.id, agent_type=node.agent_type, component_type=node.component_type.value,
        application_id=plan.application_id, tenant=tenant, configuration=node.configuration, input=inp,
        output=out, streaming_cluster=sc, errors=errors, code_directory=code_directory,
        persistent_state_directory=state_dir, replica=replica)
