"""Topic SPI (parity: API/runner/topics/TopicConnectionsRuntime.java:24-63,
TopicConsumer.java, TopicProducer.java, TopicReader.java, TopicOffsetPosition.java,
TopicConnectionsRuntimeRegistry.java:32-135) and the streaming-runtime registry."""
from __future__ import annotations

import base64
import json
import threading
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from .record import Record


@dataclass
class TopicOffsetPosition:
    """Reader start position: LATEST, EARLIEST, or ABSOLUTE (opaque bytes, base64 in APIs)."""
    position: str  # "latest" | "earliest" | "absolute"
    offset: Optional[bytes] = None

    LATEST: "TopicOffsetPosition" = None  # type: ignore[assignment]
    EARLIEST: "TopicOffsetPosition" = None  # type: ignore[assignment]

    @staticmethod
    def absolute(offset: bytes) -> "TopicOffsetPosition":
        return TopicOffsetPosition("absolute", offset)

    @staticmethod
    def parse(s: Optional[str]) -> "TopicOffsetPosition":
        if s is None or s == "" or s == "latest":
            return TopicOffsetPosition.LATEST
        if s == "earliest":
            return TopicOffsetPosition.EARLIEST
        return TopicOffsetPosition.absolute(base64.b64decode(s))


TopicOffsetPosition.LATEST = TopicOffsetPosition("latest")
TopicOffsetPosition.EARLIEST = TopicOffsetPosition("earliest")


@dataclass
class TopicReadResult:
    records: List[Record]
    offset: Optional[bytes]  # position after the last record (resume token)


class TopicConsumer:
    def start(self) -> None: ...
    def close(self) -> None: ...
    def read(self) -> List[Record]: raise NotImplementedError
    def commit(self, records: List[Record]) -> None: ...
    def get_info(self) -> Dict[str, Any]: return {}
    def get_total_out(self) -> int: return 0
    def get_native_consumer(self): return None


class BatchWriteError(Exception):
    """A ``write_many`` where some records failed: ``errors[i]`` is record i's error, or
    None when record i was delivered (only the failed ones go to retry / skip / DLQ)."""

    def __init__(self, errors: List[Optional[BaseException]]):
        first = next(e for e in errors if e is not None)
        super().__init__(f"{sum(e is not None for e in errors)} of {len(errors)} records failed: {first!r}")
        self.errors = errors


def per_item(futures: List[Future]) -> Future:
    """One future for a batch of record writes: its result is None when every write
    succeeded, else it fails with a ``BatchWriteError`` listing each record's error."""
    out: Future = Future()
    if not futures:
        out.set_result(None)
        return out
    left = [len(futures)]
    lock = threading.Lock()

    def one(_f: Future) -> None:
        with lock:
            left[0] -= 1
            last = left[0] == 0
        if last:
            errs = [f.exception() for f in futures]
            if any(e is not None for e in errs):
                out.set_exception(BatchWriteError(errs))
            else:
                out.set_result(None)
    for f in futures:
        f.add_done_callback(one)
    return out


def all_of(futures: List[Future]) -> Future:
    """One future for many: done when all are, failed with the first failure (in list
    order) if any failed."""
    out: Future = Future()
    if not futures:
        out.set_result(None)
        return out
    left = [len(futures)]
    lock = threading.Lock()

    def one(_f: Future) -> None:
        with lock:
            left[0] -= 1
            last = left[0] == 0
        if last:
            err = next((f.exception() for f in futures if f.exception() is not None), None)
            if err is not None:
                out.set_exception(err)
            else:
                out.set_result(None)
    for f in futures:
        f.add_done_callback(one)
    return out


class TopicProducer:
    def start(self) -> None: ...
    def close(self) -> None: ...
    def write(self, record: Record) -> Future: raise NotImplementedError

    def write_many(self, records: List[Record]) -> Future:
        """Write records in order; one future for all of them, failing with a
        ``BatchWriteError`` (per-record errors) if any write failed (a runtime with a
        batching client overrides this to queue them as one unit)."""
        return per_item([self.write(r) for r in records])
    def get_info(self) -> Dict[str, Any]: return {}
    def get_total_in(self) -> int: return 0
    def get_native_producer(self): return None


class TopicReader:
    def start(self) -> None: ...
    def close(self) -> None: ...
    def read(self) -> TopicReadResult: raise NotImplementedError


class TopicAdmin:
    def start(self) -> None: ...
    def close(self) -> None: ...
    def get_native_topic_admin(self): return None


class TopicConnectionsRuntime:
    """Runner-side streaming adapter."""

    def init(self, streaming_cluster) -> None: ...
    def deploy(self, plan) -> None: ...
    def delete(self, plan) -> None: ...
    def close(self) -> None: ...

    def create_consumer(self, agent_id: str, streaming_cluster, configuration: Dict[str, Any]) -> TopicConsumer:
        raise NotImplementedError

    def create_reader(self, streaming_cluster, configuration: Dict[str, Any],
                      initial_position: TopicOffsetPosition) -> TopicReader:
        raise NotImplementedError

    def create_producer(self, agent_id: str, streaming_cluster, configuration: Dict[str, Any]) -> TopicProducer:
        raise NotImplementedError

    def create_deadletter_topic_producer(self, agent_id: str, streaming_cluster,
                                         configuration: Dict[str, Any]) -> Optional[TopicProducer]:
        dl = configuration.get("deadLetterTopicProducer")
        if not dl:
            return None
        return self.create_producer(agent_id, streaming_cluster, dl)

    def create_topic_admin(self, agent_id: str, streaming_cluster, configuration: Dict[str, Any]) -> TopicAdmin:
        return TopicAdmin()


class TopicConnectionsRuntimeRegistry:
    """streaming-cluster type -> TopicConnectionsRuntime factory."""

    _factories: Dict[str, Callable[[], TopicConnectionsRuntime]] = {}
    _lock = threading.Lock()

    @classmethod
    def register(cls, type_: str, factory: Callable[[], TopicConnectionsRuntime]) -> None:
        cls._factories[type_] = factory

    _plugins_loaded = False

    @classmethod
    def _load_plugins(cls) -> None:
        """Streaming runtimes of installed bundles: entry-point group ``langstream_amd.topics``
        (the reference's META-INF/ai.langstream.streamingClusters.index)."""
        if cls._plugins_loaded:
            return
        cls._plugins_loaded = True
        try:
            from importlib.metadata import entry_points
            for ep in entry_points().select(group="langstream_amd.topics"):
                try:
                    ep.load()
                except Exception:  # noqa: BLE001
                    import logging
                    logging.getLogger(__name__).exception("failed to load streaming plugin %s", ep.name)
        except Exception:  # noqa: BLE001
            pass

    @classmethod
    def get(cls, streaming_cluster) -> TopicConnectionsRuntime:
        from .. import topics as _topics  # noqa: F401  (registers built-in runtimes)
        t = streaming_cluster.type if streaming_cluster is not None else "noop"
        f = cls._factories.get(t)
        if f is None:
            cls._load_plugins()
            f = cls._factories.get(t)
        if f is None:
            raise ValueError(f"No TopicConnectionsRuntime found for type {t}; known: {sorted(cls._factories)}")
        rt = f()
        rt.init(streaming_cluster)
        return rt

    @classmethod
    def types(cls) -> List[str]:
        from .. import topics as _topics  # noqa: F401
        return sorted(cls._factories)


class TopicConnectionProvider:
    """Given to agents so they can open extra producers/consumers (AgentContext)."""

    def __init__(self, runtime: TopicConnectionsRuntime, streaming_cluster):
        self.runtime = runtime
        self.streaming_cluster = streaming_cluster

    def create_consumer(self, agent_id: str, config: Dict[str, Any]) -> TopicConsumer:
        return self.runtime.create_consumer(agent_id, self.streaming_cluster, config)

    def create_producer(self, agent_id: str, topic: str, config: Optional[Dict[str, Any]] = None) -> TopicProducer:
        cfg = dict(config or {})
        cfg["topic"] = topic
        return self.runtime.create_producer(agent_id, self.streaming_cluster, cfg)


def encode_offsets(offsets: Dict[int, int]) -> bytes:
    """Per-partition reader position -> opaque bytes (JSON {partition: offset})."""
    return json.dumps({str(k): v for k, v in sorted(offsets.items())}).encode()


def decode_offsets(b: bytes) -> Dict[int, int]:
    return {int(k): int(v) for k, v in json.loads(b.decode()).items()}
