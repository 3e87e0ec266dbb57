"""Agent API contracts for user Python code."""
from __future__ import annotations

from abc import ABC, abstractmethod
from concurrent.futures import Future
from typing import Any, Dict, List, Optional, Tuple, Union


class Record(ABC):
    @abstractmethod
    def key(self): ...

    @abstractmethod
    def value(self): ...

    @abstractmethod
    def origin(self) -> str: ...

    @abstractmethod
    def timestamp(self) -> int: ...

    @abstractmethod
    def headers(self) -> List[Tuple[str, Any]]: ...


RecordType = Union[Record, dict, list, tuple]


class AgentContext(ABC):
    @abstractmethod
    def get_persistent_state_directory(self) -> Optional[str]: ...


class Agent(ABC):
    def init(self, config: Dict[str, Any], context: AgentContext):
        pass

    def start(self):
        pass

    def close(self):
        pass

    def agent_info(self) -> Dict[str, Any]:
        return {}


class Source(Agent):
    @abstractmethod
    def read(self) -> List[RecordType]:
        """Records as Record objects, dicts (value/key/headers/origin/timestamp) or
        tuples (value, key, headers, origin, timestamp)."""

    def commit(self, record: Record):
        pass

    def permanent_failure(self, record: Record, error: Exception):
        raise error


class Processor(Agent):
    @abstractmethod
    def process(self, record: Record) -> Union[List[RecordType], "Future[List[RecordType]]"]:
        """Records for one input record (or a Future of them)."""


class Sink(Agent):
    @abstractmethod
    def write(self, record: Record) -> Optional["Future[None]"]:
        """None on success (raise on failure), or a Future."""


class Service(Agent):
    @abstractmethod
    def main(self):
        """Run forever."""
