"""Agent-type catalog: the DSL surface the planner accepts.

For every agent type: component type, composability, runtime type, configuration
validation/enrichment and disks.  Parity: the provider list in
langstream-k8s-runtime-core/.../META-INF/services/ai.langstream.api.runtime.AgentNodeProvider
and the agents index files (``langstream-agents/*/META-INF/ai.langstream.agents.index``).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Optional, Sequence

from ..api.agent import ComponentType
from ..api.model import AgentConfiguration, DiskSpec

COMPOSITE_AGENT = "composite-agent"

GENAI_STEPS = ("drop-fields", "merge-key-value", "unwrap-key-value", "cast", "flatten", "drop", "compute",
               "compute-ai-embeddings", "query", "ai-chat-completions", "ai-text-completions")


@dataclass
class AgentSpec:
    types: Sequence[str]
    component: ComponentType
    composable: bool = True
    required: Sequence[str] = ()
    runtime: Optional[str] = None                       # runtime agent type (default = declared)
    configure: Optional[Callable] = None                # (ac, module, pipeline, plan) -> config
    disk_fn: Optional[Callable[[AgentConfiguration], Dict[str, DiskSpec]]] = None
    description: str = ""

    def component_type(self, ac: AgentConfiguration) -> ComponentType:
        return self.component

    def runtime_type(self, ac: AgentConfiguration) -> str:
        return self.runtime or ac.type

    def compute_configuration(self, ac: AgentConfiguration, module, pipeline, plan) -> Dict[str, Any]:
        from .config_model import validate_agent
        cfg = dict(ac.configuration or {})
        service = None
        if ac.type == "vector-db-sink" and isinstance(cfg.get("datasource"), str):
            r = plan.application.resources.get(cfg["datasource"])
            service = (r.configuration or {}).get("service") if r is not None else None
        cfg = validate_agent(ac.name or ac.id, ac.type, cfg, service)
        for k in self.required:
            if cfg.get(k) is None or (isinstance(cfg.get(k), str) and not cfg[k].strip()):
                raise ValueError(f"Found error on agent configuration (agent: '{ac.name or ac.id}', type: "
                                 f"'{ac.type}'). Property '{k}' is required")
        if self.configure is not None:
            cfg = self.configure(ac, cfg, module, pipeline, plan)
        return cfg

    def disks(self, ac: AgentConfiguration) -> Dict[str, DiskSpec]:
        return self.disk_fn(ac) if self.disk_fn else {}


def _genai_configure(ac, cfg, module, pipeline, plan):
    from .genai import build_genai_configuration
    return build_genai_configuration(ac, cfg, plan.application)


def _datasource_configure(ac, cfg, module, pipeline, plan):
    from .genai import resolve_datasource
    ds = cfg.get("datasource")
    if ds is not None and isinstance(ds, str):
        cfg["datasource"] = resolve_datasource(ds, plan.application)
    return cfg


def _webcrawler_disks(ac: AgentConfiguration) -> Dict[str, DiskSpec]:
    if str((ac.configuration or {}).get("state-storage", "s3")) == "disk":
        res = ac.resources
        d = res.disk if res is not None and res.disk is not None else DiskSpec(enabled=True)
        return {ac.id: d}
    return {}


def _vector_sink_disks(ac: AgentConfiguration) -> Dict[str, DiskSpec]:
    """The local GPU vector store keeps its WAL + snapshots on the agent's disk (durable
    by default); remote-database sinks need none."""
    ds = (ac.configuration or {}).get("datasource")
    if isinstance(ds, dict) and str(ds.get("service", "local")) not in ("local", "local-gpu"):
        return {}
    res = ac.resources
    return {ac.id: res.disk if res is not None and res.disk is not None else DiskSpec(enabled=True)}


P, S, K, V = ComponentType.PROCESSOR, ComponentType.SOURCE, ComponentType.SINK, ComponentType.SERVICE

_SPECS = [
    AgentSpec(GENAI_STEPS, P, runtime="ai-tools", configure=_genai_configure,
              description="GenAI toolkit step (host transforms, GPU embeddings / completions, queries)"),
    AgentSpec(("re-rank",), P, description="MMR re-rank (BM25 relevance + cosine diversity)"),
    AgentSpec(("flare-controller",), P, required=("loop-topic",), description="FLARE active retrieval loop"),
    AgentSpec(("query-vector-db",), P, required=("datasource", "query"), configure=_datasource_configure),
    AgentSpec(("vector-db-sink",), K, required=("datasource",), configure=_datasource_configure,
              disk_fn=_vector_sink_disks),
    AgentSpec(("text-extractor", "language-detector", "text-splitter", "text-normaliser", "document-to-json"), P),
    AgentSpec(("dispatch", "trigger-event", "log-event"), P),
    AgentSpec(("timer-source",), S),
    AgentSpec(("http-request",), P, required=("url",)),
    AgentSpec(("langserve-invoke",), P, required=("url",)),
    AgentSpec(("webcrawler-source",), S, disk_fn=_webcrawler_disks),
    AgentSpec(("s3-source",), S),
    AgentSpec(("azure-blob-storage-source",), S, required=("endpoint",)),
    AgentSpec(("camel-source",), S, required=("component-uri",)),
    AgentSpec(("python-source",), S, required=("className",)),
    AgentSpec(("python-processor", "python-function"), P, required=("className",)),
    AgentSpec(("python-sink",), K, required=("className",)),
    AgentSpec(("python-service",), V, required=("className",)),
    AgentSpec(("sink",), K, composable=False, description="Kafka Connect sink"),
    AgentSpec(("source",), S, composable=False, description="Kafka Connect source"),
    AgentSpec(("identity", "noop"), P),
    AgentSpec((COMPOSITE_AGENT,), P),
]

AGENT_CATALOG: Dict[str, AgentSpec] = {}
for _s in _SPECS:
    for _t in _s.types:
        AGENT_CATALOG[_t] = _s


def agent_spec(agent_type: str) -> AgentSpec:
    s = AGENT_CATALOG.get(agent_type)
    if s is None:
        raise ValueError(f"Agent type {agent_type} is not supported; known types: {sorted(AGENT_CATALOG)}")
    return s


def register_agent_type(spec: AgentSpec) -> None:
    """Plugin hook (the NAR-index analogue): add agent types at runtime."""
    for t in spec.types:
        AGENT_CATALOG[t] = spec
