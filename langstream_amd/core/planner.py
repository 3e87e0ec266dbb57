"""Execution planner: application -> ExecutionPlan (topics, assets, agent nodes), with
agent fusion.

Parity:
* BasicClusterRuntime.buildExecutionPlan (CORE/common/BasicClusterRuntime.java:50-255):
  detectTopics -> detectAssets -> detectAgents -> validate; agents built in pipeline
  order; output connection computed before input; implicit topics ``agent-<id>-input``
  (create-if-not-exists, 1 partition) and ``<input>-deadletter`` topics (:322-409).
* AbstractAgentProvider.createImplementation (CORE/common/AbstractAgentProvider.java:188-271):
  SERVICE agents may not have input/output/retries.
* ComposableAgentExecutionPlanOptimiser (CORE/agents/ComposableAgentExecutionPlanOptimiser.java:37-181):
  consecutive composable, non-SERVICE agents joined by an implicit topic with equal
  (parallelism, size) and equal errors merge into one ``composite-agent``
  ``{source:{}, processors:[{agentType, agentId, configuration}], sink:{}}``; the
  intermediate implicit topics are discarded -> one process, in-memory hand-off.
"""
from __future__ import annotations

import copy
import logging
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..api.agent import ComponentType
from ..api.model import (CREATE_IF_NOT_EXISTS, AgentConfiguration, Application, AssetDefinition, Connection,
                         DiskSpec, ErrorsSpec, Module, Pipeline, ResourcesSpec, TopicDefinition)
from .catalog import AGENT_CATALOG, COMPOSITE_AGENT, agent_spec
from .genai import build_genai_configuration

log = logging.getLogger(__name__)
DEFAULT_PARTITIONS_FOR_IMPLICIT_TOPICS = 0


@dataclass
class Topic:
    """Streaming-runtime view of a topic (partitions already defaulted)."""
    name: str
    partitions: int
    creation_mode: str
    deletion_mode: str
    implicit: bool
    definition: TopicDefinition
    deadletter: Optional["Topic"] = None
    config: Dict[str, Any] = field(default_factory=dict)
    options: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> dict:
        return {"name": self.name, "partitions": self.partitions, "creation-mode": self.creation_mode,
                "deletion-mode": self.deletion_mode, "implicit": self.implicit,
                "deadletter": self.deadletter.name if self.deadletter else None, "config": self.config}

    def _schemas(self) -> Dict[str, Any]:
        out = {}
        for k, s in (("keySchema", self.definition.key_schema if self.definition else None),
                     ("valueSchema", self.definition.value_schema if self.definition else None)):
            if s is not None:
                out[k] = {"type": s.type, "schema": s.schema, "name": s.name}
        return out

    def consumer_configuration(self) -> Dict[str, Any]:
        """What an agent's input connection carries (KAFKA/KafkaTopic.java:62-88): the topic,
        the key / value deserializer its schemas select, the schemas themselves, and the
        ``consumer.*`` options (prefix stripped)."""
        from ..topics.kafka.serde import deserializer_for_schema
        sch = self._schemas()
        cfg: Dict[str, Any] = {"topic": self.name, **_serde_keys(deserializer_for_schema, sch, "deserializer"), **sch}
        for k, v in (self.options or {}).items():
            if k.startswith("consumer."):
                cfg[k[len("consumer."):]] = v
        return cfg

    def producer_configuration(self) -> Dict[str, Any]:
        """Output connection (KAFKA/KafkaTopic.java:123-138): serializers + schemas +
        ``producer.*`` options."""
        from ..topics.kafka.serde import serializer_for_schema
        sch = self._schemas()
        cfg: Dict[str, Any] = {"topic": self.name, **_serde_keys(serializer_for_schema, sch, "serializer"), **sch}
        for k, v in (self.options or {}).items():
            if k.startswith("producer."):
                cfg[k[len("producer."):]] = v
        return cfg


def _serde_keys(pick, sch: Dict[str, Any], kind: str) -> Dict[str, Any]:
    """Kafka key / value (de)serializer classes for the topic's schemas.  A schema type the
    Kafka mapping has no class for (``int32``, ``json``: Pulsar schema types) leaves the
    key out: the Kafka adapter then raises 'Unsupported schema type' when it builds the
    consumer / producer, other streaming types use the schema themselves."""
    out: Dict[str, Any] = {}
    for which, k in (("key", "keySchema"), ("value", "valueSchema")):
        try:
            out[f"{which}.{kind}"] = pick(sch.get(k))
        except ValueError:
            pass
    return out


@dataclass
class AgentNode:
    id: str
    agent_type: str
    component_type: ComponentType
    configuration: Dict[str, Any]
    composable: bool
    input: Optional[Topic]
    output: Optional[Topic]
    resources: ResourcesSpec
    errors: ErrorsSpec
    disks: Dict[str, DiskSpec] = field(default_factory=dict)
    module: str = "default"
    pipeline: str = ""
    metadata: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> dict:
        return {"id": self.id, "agent-type": self.agent_type, "component-type": self.component_type.value,
                "configuration": self.configuration, "input": self.input.name if self.input else None,
                "output": self.output.name if self.output else None,
                "resources": self.resources.to_dict() if self.resources else None,
                "errors": self.errors.to_dict() if self.errors else None}


@dataclass
class AssetNode:
    id: str
    name: str
    asset_type: str
    creation_mode: str
    deletion_mode: str
    config: Dict[str, Any]


class ExecutionPlan:
    def __init__(self, application_id: str, application: Application):
        self.application_id = application_id
        self.application = application
        self.topics: Dict[str, Topic] = {}
        self.assets: List[AssetNode] = []
        self.agents: Dict[str, AgentNode] = {}  # "module#agentId" -> node

    def register_topic(self, t: Topic) -> Topic:
        existing = self.topics.get(t.name)
        if existing is not None:
            return existing
        self.topics[t.name] = t
        return t

    def discard_topic(self, t: Optional[Topic]) -> None:
        if t is not None and t.implicit:
            self.topics.pop(t.name, None)

    def get_topic(self, name: str) -> Optional[Topic]:
        return self.topics.get(name)

    def register_agent(self, module: Module, node: AgentNode) -> None:
        self.agents[f"{module.id}#{node.id}"] = node

    def get_agent(self, agent_id: str) -> Optional[AgentNode]:
        for k, n in self.agents.items():
            if n.id == agent_id or k.endswith("#" + agent_id):
                return n
        return None

    def topics_to_create(self) -> List[Topic]:
        return [t for t in self.topics.values() if t.creation_mode == CREATE_IF_NOT_EXISTS]

    def to_dict(self) -> dict:
        return {"application-id": self.application_id,
                "topics": [t.to_dict() for t in self.topics.values()],
                "assets": [a.__dict__ for a in self.assets],
                "agents": {k: v.to_dict() for k, v in self.agents.items()}}


def _topic_impl(td: TopicDefinition) -> Topic:
    return Topic(name=td.name, partitions=td.partitions if td.partitions > 0 else 1, creation_mode=td.creation_mode,
                 deletion_mode=td.deletion_mode, implicit=td.implicit, definition=td, config=dict(td.config),
                 options=dict(td.options))


class Planner:
    """ComputeClusterRuntime planning half (kubernetes / none / local share it)."""

    def __init__(self, resource_providers: Optional[Dict[str, Callable]] = None):
        self.resource_providers = resource_providers or {}

    def build_execution_plan(self, application_id: str, application: Application) -> ExecutionPlan:
        if not application_id:
            raise ValueError("Application id cannot be empty")
        plan = ExecutionPlan(application_id, application)
        for module in application.modules.values():
            for td in module.topics.values():
                plan.register_topic(_topic_impl(td))
        for module in application.modules.values():
            for asset in module.assets:
                plan.assets.append(_asset_node(asset, application))
        for module in application.modules.values():
            for pipeline in module.pipelines.values():
                prev: Optional[AgentNode] = None
                for ac in pipeline.agents:
                    prev = self._build_agent(module, pipeline, ac, plan, prev)
        inst = application.instance
        if inst is not None and inst.compute_cluster is not None and inst.compute_cluster.type == "kubernetes":
            from .k8s import validate_execution_plan
            validate_execution_plan(plan)
        return plan

    # ------------------------------------------------------------------ connections
    def _ensure_deadletter(self, conn: Connection, plan: ExecutionPlan, topic: Topic) -> None:
        if not conn.enable_dead_letter_queue:
            return
        td = topic.definition
        dl = TopicDefinition(name=td.name + "-deadletter", creation_mode=CREATE_IF_NOT_EXISTS,
                             deletion_mode=td.deletion_mode, implicit=td.implicit, partitions=td.partitions,
                             key_schema=td.key_schema, value_schema=td.value_schema)
        topic.deadletter = plan.register_topic(_topic_impl(dl))

    def _implicit_topic_for(self, agent: AgentConfiguration, plan: ExecutionPlan) -> Topic:
        td = TopicDefinition(name=f"agent-{agent.id}-input", creation_mode=CREATE_IF_NOT_EXISTS,
                             implicit=True, partitions=DEFAULT_PARTITIONS_FOR_IMPLICIT_TOPICS)
        return plan.register_topic(_topic_impl(td))

    def _connection(self, pipeline: Pipeline, conn: Optional[Connection], direction: str,
                    plan: ExecutionPlan) -> Optional[Topic]:
        if conn is None:
            return None
        if conn.connection_type == "TOPIC":
            t = plan.get_topic(conn.definition)
            if t is None:
                raise ValueError(f"Topic {conn.definition} not found, only {sorted(plan.topics)} are available")
            self._ensure_deadletter(conn, plan, t)
            return t
        target = pipeline.get_agent(conn.definition)
        if target is None:
            raise ValueError(f"Agent {conn.definition} not found in pipeline {pipeline.id}")
        if direction == "OUTPUT":
            t = self._implicit_topic_for(target, plan)
            self._ensure_deadletter(conn, plan, t)
            return t
        if target.output is None:
            raise ValueError(f"Invalid agent configuration for ({target.name}), missing output")
        return self._connection(pipeline, target.output, "OUTPUT", plan)

    # ------------------------------------------------------------------ agents
    def _build_agent(self, module: Module, pipeline: Pipeline, ac: AgentConfiguration, plan: ExecutionPlan,
                     prev: Optional[AgentNode]) -> AgentNode:
        spec = agent_spec(ac.type)
        configuration = spec.compute_configuration(ac, module, pipeline, plan)
        output = self._connection(pipeline, ac.output, "OUTPUT", plan)
        inp = self._connection(pipeline, ac.input, "INPUT", plan)
        ctype = spec.component_type(ac)
        if ctype == ComponentType.SERVICE:
            if inp is not None:
                raise ValueError(f"Service agents ({ac.type}) cannot have an input")
            if output is not None:
                raise ValueError(f"Service agents ({ac.type}) cannot have an output")
            if ac.errors is not None and ac.errors.retries and ac.errors.retries > 0:
                raise ValueError(f"Service agents ({ac.type}) cannot have retries")
        node = AgentNode(id=ac.id, agent_type=spec.runtime_type(ac), component_type=ctype,
                         configuration=configuration, composable=spec.composable, input=inp, output=output,
                         resources=ac.resources or ResourcesSpec.DEFAULT, errors=ac.errors or ErrorsSpec.DEFAULT,
                         disks=spec.disks(ac), module=module.id, pipeline=pipeline.id,
                         metadata={"name": ac.name, "declared-type": ac.type})
        if prev is not None:
            if prev.output is None:
                raise ValueError(f"Invalid agent configuration for ({prev.id}), missing output")
            if prev.output is node.input and prev.output.implicit and can_merge(prev, node):
                merge_agents(prev, node, plan)
                return prev
        plan.register_agent(module, node)
        return node


def _asset_node(asset: AssetDefinition, app: Application) -> AssetNode:
    from .assets import validate_asset
    cfg = validate_asset(asset, app)
    return AssetNode(asset.id, asset.name, asset.asset_type, asset.creation_mode, asset.deletion_mode, cfg)


# ---------------------------------------------------------------- fusion
def _composable_flag(cfg: Dict[str, Any]) -> bool:
    return str(cfg.get("composable", "true")).lower() == "true"


def can_merge(a1: AgentNode, a2: AgentNode) -> bool:
    return (a1.composable and a2.composable
            and a1.component_type != ComponentType.SERVICE and a2.component_type != ComponentType.SERVICE
            and _composable_flag(a1.configuration) and _composable_flag(a2.configuration)
            and (a1.resources.parallelism, a1.resources.size) == (a2.resources.parallelism, a2.resources.size)
            and a1.errors == a2.errors)


def _as_step(n: AgentNode) -> Dict[str, Any]:
    return {"agentType": n.agent_type, "configuration": n.configuration, "agentId": n.id}


def merge_agents(a1: AgentNode, a2: AgentNode, plan: ExecutionPlan) -> AgentNode:
    if a1.agent_type == COMPOSITE_AGENT:
        cfg = copy.copy(a1.configuration)
        cfg["processors"] = list(cfg.get("processors", []))
        cfg["source"] = dict(cfg.get("source", {}))
        cfg["sink"] = dict(cfg.get("sink", {}))
        step = _as_step(a2)
        if a2.component_type == ComponentType.PROCESSOR:
            cfg["processors"].append(step)
        elif a2.component_type == ComponentType.SOURCE:
            if cfg["source"]:
                raise ValueError("Cannot merge two sources")
            cfg["source"].update(step)
        elif a2.component_type == ComponentType.SINK:
            if cfg["sink"]:
                raise ValueError("Cannot merge two sinks")
            cfg["sink"].update(step)
    else:
        source, sink, processors = {}, {}, []
        for n in (a1, a2):
            step = _as_step(n)
            if n.component_type == ComponentType.SOURCE:
                if source:
                    raise ValueError("Cannot merge two sources")
                source.update(step)
            elif n.component_type == ComponentType.SINK:
                if sink:
                    raise ValueError("Cannot merge two sinks")
                sink.update(step)
            elif n.component_type == ComponentType.PROCESSOR:
                processors.append(step)
            else:
                raise ValueError(f"Invalid agent type {n.component_type}")
        cfg = {"processors": processors, "source": source, "sink": sink}
    plan.discard_topic(a1.output)
    plan.discard_topic(a2.input)
    a1.agent_type = COMPOSITE_AGENT
    a1.configuration = cfg
    a1.output = a2.output
    a1.disks = {**a1.disks, **a2.disks}
    # the fused node's component type is what it exposes to the runner
    if cfg["source"] and not cfg["sink"]:
        a1.component_type = ComponentType.SOURCE
    elif cfg["sink"] and not cfg["source"]:
        a1.component_type = ComponentType.SINK if not a1.output else ComponentType.PROCESSOR
    else:
        a1.component_type = ComponentType.PROCESSOR
    return a1
