"""Agent SPI (parity: API/runner/code/AgentCode.java:25-72, AgentSource.java:22-54,
AgentProcessor.java:22-46, AgentSink.java:22-47, AgentService.java, AbstractAgentCode.java:27-103,
SingleRecordAgentProcessor.java:27-53, AgentContext.java:25-67, AgentStatusResponse.java).

Asynchrony uses ``concurrent.futures.Future`` (the CompletableFuture analogue): sinks
return futures, processors emit results through a RecordSink callback that may be
invoked from any thread and must never raise.
"""
from __future__ import annotations

import enum
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from .record import Record, RecordSink, SourceRecordAndResult


class ComponentType(str, enum.Enum):
    SOURCE = "SOURCE"
    PROCESSOR = "PROCESSOR"
    SINK = "SINK"
    SERVICE = "SERVICE"


@dataclass
class AgentStatusResponse:
    agent_id: str
    agent_type: str
    component_type: str
    info: Dict[str, Any] = field(default_factory=dict)
    metrics: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> dict:
        return {"agent-id": self.agent_id, "agent-type": self.agent_type, "component-type": self.component_type,
                "info": self.info, "metrics": self.metrics}


class AgentCode:
    """Lifecycle: set_metadata -> init(config) -> set_context(ctx) -> start -> ... -> close."""

    _agent_id: str = "?"
    _agent_type: str = "?"
    _started_at: int = 0
    context: "AgentContext | None" = None

    def set_metadata(self, agent_id: str, agent_type: str, started_at: int) -> None:
        self._agent_id = agent_id
        self._agent_type = agent_type
        self._started_at = started_at

    def agent_id(self) -> str:
        return self._agent_id

    def agent_type(self) -> str:
        return self._agent_type

    def component_type(self) -> ComponentType:
        raise NotImplementedError

    def init(self, configuration: Dict[str, Any]) -> None:
        pass

    def set_context(self, context: "AgentContext") -> None:
        self.context = context

    def start(self) -> None:
        pass

    def close(self) -> None:
        pass

    def restart(self) -> None:
        pass

    def get_agent_status(self) -> List[AgentStatusResponse]:
        return [AgentStatusResponse(self._agent_id, self._agent_type, self.component_type().value, {}, {})]


class AbstractAgentCode(AgentCode):
    """Keeps identity plus the ``total-in``/``total-out`` counters."""

    def __init__(self):
        self._total_in = 0
        self._total_out = 0
        self._last_processed_at = 0
        self._started_at = int(time.time() * 1000)

    def processed(self, n_in: int, n_out: int) -> None:
        self._total_in += n_in
        self._total_out += n_out
        self._last_processed_at = int(time.time() * 1000)

    def build_additional_info(self) -> Dict[str, Any]:
        return {}

    def get_agent_status(self) -> List[AgentStatusResponse]:
        return [AgentStatusResponse(
            self._agent_id, self._agent_type, self.component_type().value, self.build_additional_info(),
            {"total-in": self._total_in, "total-out": self._total_out, "started-at": self._started_at,
             "last-processed-at": self._last_processed_at})]


class AgentSource(AbstractAgentCode):
    def component_type(self) -> ComponentType:
        return ComponentType.SOURCE

    def read(self) -> List[Record]:
        """Return a (possibly empty) batch; should block briefly when idle."""
        raise NotImplementedError

    def commit(self, records: List[Record]) -> None:
        pass

    def permanent_failure(self, record: Record, error: BaseException) -> None:
        """Called when a record fails permanently; default rethrows (fail the pipeline)."""
        raise error


class AgentProcessor(AbstractAgentCode):
    def component_type(self) -> ComponentType:
        return ComponentType.PROCESSOR

    def process(self, records: List[Record], sink: RecordSink) -> None:
        raise NotImplementedError


class SingleRecordAgentProcessor(AgentProcessor):
    """Adapter: implement ``process_record(record) -> list[Record]``; exceptions become
    ``emit(error)`` for that record."""

    def process_record(self, record: Record) -> List[Record]:
        raise NotImplementedError

    def process(self, records: List[Record], sink: RecordSink) -> None:
        for r in records:
            try:
                out = self.process_record(r) or []
                self.processed(1, len(out))
                sink(SourceRecordAndResult(r, list(out), None))
            except Exception as e:  # noqa: BLE001
                sink(SourceRecordAndResult(r, None, e))


class AgentSink(AbstractAgentCode):
    def component_type(self) -> ComponentType:
        return ComponentType.SINK

    def write(self, record: Record) -> Future:
        raise NotImplementedError

    def handles_commit(self) -> bool:
        return False

    def commit(self) -> None:
        pass


class AgentService(AbstractAgentCode):
    def component_type(self) -> ComponentType:
        return ComponentType.SERVICE

    def join(self) -> None:
        raise NotImplementedError


def completed(value: Any = None) -> Future:
    f: Future = Future()
    f.set_result(value)
    return f


def failed(error: BaseException) -> Future:
    f: Future = Future()
    f.set_exception(error)
    return f


class BadRecordHandler:
    """skip / dead-letter / fail handling of a record that failed permanently."""

    def __init__(self, fn: Callable[[Record, BaseException, Callable[[], None]], None]):
        self._fn = fn

    def handle(self, record: Record, error: BaseException, cleanup: Callable[[], None] = lambda: None) -> None:
        self._fn(record, error, cleanup)


class AgentContext:
    """What the runtime gives an agent (AgentContext.java:25-67)."""

    def __init__(self, *, agent_id: str, global_agent_id: str, tenant: str = "default", consumer=None,
                 producer=None, topic_admin=None, topic_connection_provider=None, metrics_reporter=None,
                 bad_record_handler: Optional[BadRecordHandler] = None,
                 critical_failure: Optional[Callable[[BaseException], None]] = None, code_directory: str = "",
                 persistent_state_directory: Optional[str] = None, resources: Optional[Dict[str, Any]] = None,
                 services: Optional[Any] = None):
        self.agent_id = agent_id
        self.global_agent_id = global_agent_id
        self.tenant = tenant
        self.consumer = consumer
        self.producer = producer
        self.topic_admin = topic_admin
        self.topic_connection_provider = topic_connection_provider
        self.metrics_reporter = metrics_reporter
        self.bad_record_handler = bad_record_handler
        self._critical = critical_failure
        self.code_directory = code_directory
        self._state_dir = persistent_state_directory
        self.resources = resources or {}
        self.services = services  # GPU service registry (engines), see langstream_amd.services

    def critical_failure(self, error: BaseException) -> None:
        if self._critical is not None:
            self._critical(error)
        else:
            raise error

    def get_persistent_state_directory(self) -> Optional[str]:
        return self._state_dir

    def get_persistent_state_directory_for_agent(self, agent_id: str) -> Optional[str]:
        import os
        if self._state_dir is None:
            return None
        p = os.path.join(self._state_dir, agent_id)
        os.makedirs(p, exist_ok=True)
        return p
