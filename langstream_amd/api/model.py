"""Application model: the in-memory form of the LangStream YAML DSL.

Parity: reference ``langstream-api/src/main/java/ai/langstream/api/model/*``
(Application.java:23-51, Module.java:23-105, Pipeline.java:23-51,
AgentConfiguration.java:21-33, TopicDefinition.java:25-122, AssetDefinition.java:24-94,
ResourcesSpec.java:23-36, ErrorsSpec.java:25-47, DiskSpec.java:24-86, Gateway.java:30-162,
Instance/StreamingCluster/ComputeCluster/Secrets/Dependency).
Field names follow the YAML (kebab-case) spelling; Python attributes are snake_case.
"""
from __future__ import annotations

import copy
import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

DEFAULT_MODULE = "default"

# ---------------------------------------------------------------- errors / resources / disks
FAIL = "fail"
SKIP = "skip"
DEAD_LETTER = "dead-letter"
ON_FAILURE_VALUES = (FAIL, SKIP, DEAD_LETTER)


@dataclass
class ErrorsSpec:
    retries: Optional[int] = None
    on_failure: Optional[str] = None

    def with_defaults_from(self, higher: "ErrorsSpec | None") -> "ErrorsSpec":
        if higher is None:
            return self
        return ErrorsSpec(
            retries=self.retries if self.retries is not None else higher.retries,
            on_failure=self.on_failure if self.on_failure is not None else higher.on_failure,
        )

    @staticmethod
    def from_dict(d: Optional[dict]) -> Optional["ErrorsSpec"]:
        if d is None:
            return None
        return ErrorsSpec(retries=d.get("retries"), on_failure=d.get("on-failure", d.get("onFailure")))

    def to_dict(self) -> dict:
        return {"retries": self.retries, "on-failure": self.on_failure}


ErrorsSpec.DEFAULT = ErrorsSpec(retries=0, on_failure=FAIL)  # type: ignore[attr-defined]


@dataclass
class DiskSpec:
    enabled: bool = False
    type: str = "default"
    size: str = "256M"

    @staticmethod
    def from_dict(d):
        if d is None:
            return None
        return DiskSpec(enabled=bool(d.get("enabled", True)), type=d.get("type", "default"),
                        size=str(d.get("size", "256M")))


@dataclass
class ResourcesSpec:
    parallelism: Optional[int] = None
    size: Optional[int] = None
    disk: Optional[DiskSpec] = None

    def with_defaults_from(self, higher: "ResourcesSpec | None") -> "ResourcesSpec":
        if higher is None:
            return self
        return ResourcesSpec(
            parallelism=self.parallelism if self.parallelism is not None else higher.parallelism,
            size=self.size if self.size is not None else higher.size,
            disk=self.disk if self.disk is not None else higher.disk,
        )

    @staticmethod
    def from_dict(d):
        if d is None:
            return None
        return ResourcesSpec(parallelism=d.get("parallelism"), size=d.get("size"),
                             disk=DiskSpec.from_dict(d.get("disk")))

    def to_dict(self):
        return {"parallelism": self.parallelism, "size": self.size,
                "disk": dataclasses.asdict(self.disk) if self.disk else None}


ResourcesSpec.DEFAULT = ResourcesSpec(parallelism=1, size=1)  # type: ignore[attr-defined]


# ---------------------------------------------------------------- topics / assets / schemas
CREATE_IF_NOT_EXISTS = "create-if-not-exists"
CREATION_NONE = "none"
DELETE = "delete"


@dataclass
class SchemaDefinition:
    type: str
    schema: Optional[str] = None
    name: Optional[str] = None

    @staticmethod
    def from_dict(d):
        if d is None:
            return None
        return SchemaDefinition(type=d.get("type"), schema=d.get("schema"), name=d.get("name"))


@dataclass
class TopicDefinition:
    name: str
    creation_mode: str = CREATION_NONE
    deletion_mode: str = CREATION_NONE
    implicit: bool = False
    partitions: int = 0
    key_schema: Optional[SchemaDefinition] = None
    value_schema: Optional[SchemaDefinition] = None
    options: Dict[str, Any] = field(default_factory=dict)
    config: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if self.creation_mode is None:
            self.creation_mode = CREATION_NONE
        if self.deletion_mode is None:
            self.deletion_mode = CREATION_NONE
        if self.creation_mode not in (CREATION_NONE, CREATE_IF_NOT_EXISTS):
            raise ValueError(f"Invalid creation mode {self.creation_mode}, only "
                             f"{CREATION_NONE}, {CREATE_IF_NOT_EXISTS} are allowed")
        if self.deletion_mode not in (CREATION_NONE, DELETE):
            raise ValueError(f"Invalid deletion mode {self.deletion_mode}, only {CREATION_NONE}, {DELETE} are allowed")
        if self.partitions is None:
            self.partitions = 0
        if self.partitions < 0:
            raise ValueError("Invalid partitions: " + str(self.partitions))
        self.options = dict(self.options or {})
        self.config = dict(self.config or {})

    @staticmethod
    def from_dict(d: dict) -> "TopicDefinition":
        return TopicDefinition(
            name=d["name"],
            creation_mode=d.get("creation-mode", CREATION_NONE),
            deletion_mode=d.get("deletion-mode", CREATION_NONE),
            implicit=bool(d.get("implicit", False)),
            partitions=int(d.get("partitions", 0) or 0),
            key_schema=SchemaDefinition.from_dict(d.get("keySchema", d.get("key-schema"))),
            value_schema=SchemaDefinition.from_dict(d.get("schema", d.get("valueSchema"))),
            options=d.get("options") or {},
            config=d.get("config") or {},
        )

    @staticmethod
    def from_name(name: str) -> "TopicDefinition":
        return TopicDefinition(name=name)

    def copy(self) -> "TopicDefinition":
        return copy.deepcopy(self)

    def identity(self) -> tuple:
        return (self.name, self.creation_mode, self.deletion_mode, self.partitions, self.key_schema,
                self.value_schema, repr(sorted(self.options.items())), repr(sorted(self.config.items())))


@dataclass
class AssetDefinition:
    id: str
    name: str
    creation_mode: str = CREATION_NONE
    deletion_mode: str = CREATION_NONE
    asset_type: Optional[str] = None
    config: Dict[str, Any] = field(default_factory=dict)

    @staticmethod
    def from_dict(d: dict) -> "AssetDefinition":
        aid = d.get("id") or d.get("name")
        if not aid:
            raise ValueError("Asset id or name are required")
        return AssetDefinition(id=aid, name=d.get("name") or aid,
                               creation_mode=d.get("creation-mode", CREATION_NONE) or CREATION_NONE,
                               deletion_mode=d.get("deletion-mode", CREATION_NONE) or CREATION_NONE,
                               asset_type=d.get("asset-type"), config=d.get("config") or {})


# ---------------------------------------------------------------- connections / agents
@dataclass(frozen=True)
class Connection:
    """An agent input/output: either an explicit topic or another agent (implicit topic)."""
    connection_type: str  # "TOPIC" | "AGENT"
    definition: str       # topic name or agent id
    enable_dead_letter_queue: bool = False

    @staticmethod
    def from_topic(topic: TopicDefinition) -> "Connection":
        return Connection("TOPIC", topic.name)

    @staticmethod
    def from_agent(agent: "AgentConfiguration") -> "Connection":
        return Connection("AGENT", agent.id)

    def with_deadletter(self, enabled: bool) -> "Connection":
        return Connection(self.connection_type, self.definition, enabled)


@dataclass
class AgentConfiguration:
    id: Optional[str] = None
    name: Optional[str] = None
    type: Optional[str] = None
    input: Optional[Connection] = None
    output: Optional[Connection] = None
    configuration: Dict[str, Any] = field(default_factory=dict)
    resources: Optional[ResourcesSpec] = None
    errors: Optional[ErrorsSpec] = None
    executor: Optional[str] = None  # reserved: named executor group


@dataclass
class Pipeline:
    id: str
    module: str
    name: Optional[str] = None
    resources: ResourcesSpec = field(default_factory=lambda: ResourcesSpec.DEFAULT)
    errors: ErrorsSpec = field(default_factory=lambda: ErrorsSpec.DEFAULT)
    agents: List[AgentConfiguration] = field(default_factory=list)

    def add_agent_configuration(self, a: AgentConfiguration) -> None:
        self.agents.append(a)

    def get_agent(self, agent_id: str) -> Optional[AgentConfiguration]:
        for a in self.agents:
            if a.id == agent_id:
                return a
        return None


@dataclass
class Module:
    id: str
    pipelines: Dict[str, Pipeline] = field(default_factory=dict)
    topics: Dict[str, TopicDefinition] = field(default_factory=dict)
    assets: List[AssetDefinition] = field(default_factory=list)

    def add_pipeline(self, pid: str) -> Pipeline:
        if pid in self.pipelines:
            raise ValueError(f"Pipeline {pid} already exists")
        p = Pipeline(id=pid, module=self.id)
        self.pipelines[pid] = p
        return p

    def add_topic(self, t: TopicDefinition) -> TopicDefinition:
        existing = self.topics.get(t.name)
        if existing is not None:
            if existing.identity() != t.identity():
                raise ValueError(f"Topic {t.name} is defined twice with different definitions")
            return existing
        self.topics[t.name] = t
        return t

    def add_asset(self, a: AssetDefinition) -> None:
        for e in self.assets:
            if e.id == a.id:
                if e != a:
                    raise ValueError(f"Asset {a.id} is defined twice with different definitions")
                return
        self.assets.append(a)

    def resolve_topic(self, name: str) -> TopicDefinition:
        t = self.topics.get(name)
        if t is None:
            raise ValueError(f"Topic {name} is not defined, only {sorted(self.topics)} are defined")
        return t


# ---------------------------------------------------------------- resources / instance / secrets
@dataclass
class Resource:
    id: str
    name: str
    type: str
    configuration: Dict[str, Any] = field(default_factory=dict)


@dataclass
class Dependency:
    name: str
    url: str
    sha512sum: Optional[str] = None
    type: str = "java-library"


@dataclass
class StreamingCluster:
    type: str
    configuration: Dict[str, Any] = field(default_factory=dict)


@dataclass
class ComputeCluster:
    type: str
    configuration: Dict[str, Any] = field(default_factory=dict)


@dataclass
class Instance:
    streaming_cluster: Optional[StreamingCluster] = None
    compute_cluster: Optional[ComputeCluster] = None
    globals: Dict[str, Any] = field(default_factory=dict)


@dataclass
class Secret:
    id: str
    name: Optional[str] = None
    data: Dict[str, Any] = field(default_factory=dict)


@dataclass
class Secrets:
    secrets: Dict[str, Secret] = field(default_factory=dict)


# ---------------------------------------------------------------- gateways
@dataclass
class KeyValueComparison:
    key: Optional[str] = None
    value: Optional[str] = None
    value_from_parameters: Optional[str] = None
    value_from_authentication: Optional[str] = None

    def __post_init__(self):
        n = sum(x is not None for x in (self.value, self.value_from_parameters, self.value_from_authentication))
        if n == 0:
            raise ValueError("Must specify one of value, value-from-parameters, or value-from-authentication")
        if n > 1:
            raise ValueError("Only one of 'value', 'valueFromParameters' or 'valueFromAuthentication' can be "
                             "specified for filter")
        # a missing key is named after the value / parameter / authentication field
        # (Gateway.KeyValueComparison's canonical constructor, Gateway.java:97-108; the
        # ModelBuilderTest expectations go through the same constructor)
        if self.key is None:
            self.key = self.value if self.value is not None else (
                self.value_from_parameters if self.value_from_parameters is not None
                else self.value_from_authentication)

    @staticmethod
    def from_dict(d: dict) -> "KeyValueComparison":
        return KeyValueComparison(
            key=d.get("key"), value=d.get("value"),
            value_from_parameters=d.get("value-from-parameters", d.get("valueFromParameters")),
            value_from_authentication=d.get("value-from-authentication", d.get("valueFromAuthentication")))


def _kvs(lst):
    return [KeyValueComparison.from_dict(x) for x in (lst or [])]


@dataclass
class GatewayAuthentication:
    provider: Optional[str] = None
    configuration: Dict[str, Any] = field(default_factory=dict)
    allow_test_mode: bool = True


@dataclass
class ChatOptions:
    questions_topic: Optional[str] = None
    answers_topic: Optional[str] = None
    headers: List[KeyValueComparison] = field(default_factory=list)


@dataclass
class ServiceOptions:
    agent_id: Optional[str] = None
    input_topic: Optional[str] = None
    output_topic: Optional[str] = None
    headers: List[KeyValueComparison] = field(default_factory=list)


@dataclass
class Gateway:
    id: str
    type: str  # produce | consume | chat | service
    topic: Optional[str] = None
    authentication: Optional[GatewayAuthentication] = None
    parameters: List[str] = field(default_factory=list)
    produce_options: Optional[List[KeyValueComparison]] = None       # produce-options.headers
    consume_options: Optional[List[KeyValueComparison]] = None       # consume-options.filters.headers
    chat_options: Optional[ChatOptions] = None
    service_options: Optional[ServiceOptions] = None
    events_topic: Optional[str] = None
    _raw_keys: tuple = ()

    TYPES = ("produce", "consume", "chat", "service")

    @staticmethod
    def from_dict(d: dict) -> "Gateway":
        auth = d.get("authentication")
        a = None
        if auth is not None:
            a = GatewayAuthentication(provider=auth.get("provider"), configuration=auth.get("configuration") or {},
                                      allow_test_mode=bool(auth.get("allow-test-mode", True)))
        po = d.get("produce-options", d.get("produceOptions"))
        co = d.get("consume-options", d.get("consumeOptions"))
        ch = d.get("chat-options")
        so = d.get("service-options")
        t = d.get("type")
        if t is not None and t not in Gateway.TYPES:
            raise ValueError(f"Invalid gateway type {t}")
        return Gateway(
            id=d.get("id"), type=t, topic=d.get("topic"), authentication=a,
            parameters=list(d.get("parameters") or []),
            produce_options=_kvs((po or {}).get("headers")) if po is not None else None,
            consume_options=_kvs(((co or {}).get("filters") or {}).get("headers")) if co is not None else None,
            chat_options=ChatOptions(questions_topic=ch.get("questions-topic"), answers_topic=ch.get("answers-topic"),
                                     headers=_kvs(ch.get("headers"))) if ch is not None else None,
            service_options=ServiceOptions(agent_id=so.get("agent-id"), input_topic=so.get("input-topic"),
                                           output_topic=so.get("output-topic"),
                                           headers=_kvs(so.get("headers"))) if so is not None else None,
            events_topic=d.get("events-topic"),
        )


# ---------------------------------------------------------------- application
@dataclass
class Application:
    resources: Dict[str, Resource] = field(default_factory=dict)
    modules: Dict[str, Module] = field(default_factory=dict)
    dependencies: List[Dependency] = field(default_factory=list)
    gateways: List[Gateway] = field(default_factory=list)
    instance: Optional[Instance] = None
    secrets: Optional[Secrets] = None

    def get_module(self, mid: str) -> Module:
        m = self.modules.get(mid)
        if m is None:
            m = Module(id=mid)
            self.modules[mid] = m
        return m

    def get_gateway(self, gid: str) -> Optional[Gateway]:
        for g in self.gateways:
            if g.id == gid:
                return g
        return None

    def all_agents(self):
        for m in self.modules.values():
            for p in m.pipelines.values():
                for a in p.agents:
                    yield m, p, a

    def copy(self) -> "Application":
        return copy.deepcopy(self)
