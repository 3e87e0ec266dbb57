"""Configuration helpers and batching executors.

Parity: API/util/ConfigurationUtils.java:46-322, API/util/BatchExecutor.java:30-95,
API/util/OrderedAsyncBatchExecutor.java:39-177.
"""
from __future__ import annotations

import copy
import logging
import os
import threading
from collections import deque
from concurrent.futures import Future
from typing import Any, Callable, Dict, Generic, List, Optional, TypeVar

log = logging.getLogger(__name__)
T = TypeVar("T")

DEVELOPMENT_MODE = os.environ.get("LANGSTREAM_DEVELOPMENT_MODE", "false").lower() == "true"


def is_development_mode() -> bool:
    return DEVELOPMENT_MODE or os.environ.get("langstream.development.mode", "false").lower() == "true"


# ---------------------------------------------------------------- typed getters
def get_string(key: str, default: Optional[str], cfg: Dict[str, Any]) -> Optional[str]:
    v = cfg.get(key)
    if v is None:
        return default
    return v if isinstance(v, str) else str(v)


def get_int(key: str, default: int, cfg: Dict[str, Any]) -> int:
    v = cfg.get(key)
    if v is None or v == "":
        return default
    return int(float(v)) if isinstance(v, str) else int(v)


def get_long(key: str, default: int, cfg: Dict[str, Any]) -> int:
    return get_int(key, default, cfg)


def get_double(key: str, default: Optional[float], cfg: Dict[str, Any]) -> Optional[float]:
    v = cfg.get(key)
    if v is None or v == "":
        return default
    return float(v)


def get_boolean(key: str, default: bool, cfg: Dict[str, Any]) -> bool:
    v = cfg.get(key)
    if v is None:
        return default
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() == "true"


def get_list(key: str, cfg: Dict[str, Any]) -> List[Any]:
    v = cfg.get(key)
    if v is None:
        return []
    if isinstance(v, list):
        return v
    if isinstance(v, str):
        return [x.strip() for x in v.split(",") if x.strip()]
    return [v]


def get_map(key: str, default: Optional[dict], cfg: Dict[str, Any]) -> Dict[str, Any]:
    v = cfg.get(key)
    if v is None:
        return dict(default or {})
    if not isinstance(v, dict):
        raise ValueError(f"{key} must be a map, got {type(v).__name__}")
    return v


def required_field(cfg: Dict[str, Any], key: str, description: str = "") -> Any:
    v = cfg.get(key)
    if v is None or (isinstance(v, str) and not v.strip()):
        raise ValueError(f"Missing required field '{key}'{(' in ' + description) if description else ''}")
    return v


def required_non_empty_field(cfg: Dict[str, Any], key: str, description: str = "") -> Any:
    v = required_field(cfg, key, description)
    if isinstance(v, (list, dict)) and not v:
        raise ValueError(f"Field '{key}' must not be empty{(' in ' + description) if description else ''}")
    return v


_SECRET_KEYS = ("password", "secret", "access-key", "accesskey", "token", "credentials", "api-key", "apikey")


def redact_secrets(v: Any) -> Any:
    """Deep copy with secret-looking values replaced by '<redacted>'."""
    if isinstance(v, dict):
        out = {}
        for k, x in v.items():
            if isinstance(k, str) and any(s in k.lower() for s in _SECRET_KEYS) and not isinstance(x, (dict, list)):
                out[k] = "<redacted>"
            else:
                out[k] = redact_secrets(x)
        return out
    if isinstance(v, list):
        return [redact_secrets(x) for x in v]
    return copy.copy(v)


# ---------------------------------------------------------------- batch executors
def java_hash(v: Any) -> int:
    """``java.util.Objects.hashCode`` of a record key as the JVM computes it: String ->
    String.hashCode over UTF-16 code units, Integer / Long / Boolean / Double per their
    hashCode, null -> 0; byte[] keys hash by content (Arrays.hashCode).  Bucket choices of
    the ordered batch executors depend on it (OrderedAsyncBatchExecutor.java:94-105)."""
    def s32(h: int) -> int:
        h &= 0xFFFFFFFF
        return h - (1 << 32) if h >= 1 << 31 else h
    if v is None:
        return 0
    if isinstance(v, bool):
        return 1231 if v else 1237
    if isinstance(v, int):
        return s32(v) if -(1 << 31) <= v < (1 << 31) else s32(v ^ (v >> 32))
    if isinstance(v, float):
        import struct
        bits = struct.unpack(">q", struct.pack(">d", v))[0]
        return s32(bits ^ (bits >> 32))
    if isinstance(v, (bytes, bytearray)):
        h = 1
        for b in v:
            h = (31 * h + (b - 256 if b > 127 else b)) & 0xFFFFFFFF
        return s32(h)
    s = v if isinstance(v, str) else str(v)
    h = 0
    data = s.encode("utf-16-be")
    for i in range(0, len(data), 2):
        h = (31 * h + ((data[i] << 8) | data[i + 1])) & 0xFFFFFFFF
    return s32(h)


class _Scheduler:
    """A tiny shared timer thread (ScheduledExecutorService analogue)."""

    def __init__(self):
        self._cv = threading.Condition()
        self._tasks: list = []  # (deadline, seq, fn, interval)
        self._seq = 0
        self._thread = threading.Thread(target=self._run, name="langstream-timer", daemon=True)
        self._thread.start()

    def schedule_fixed_delay(self, fn: Callable[[], None], interval_s: float):
        import time
        with self._cv:
            self._seq += 1
            handle = [True]
            self._tasks.append((time.monotonic() + interval_s, self._seq, fn, interval_s, handle))
            self._cv.notify()
        return handle

    @staticmethod
    def cancel(handle) -> None:
        handle[0] = False

    def _run(self) -> None:
        import time
        while True:
            with self._cv:
                while not self._tasks:
                    self._cv.wait()
                self._tasks.sort(key=lambda t: t[0])
                deadline, seq, fn, interval, handle = self._tasks[0]
                now = time.monotonic()
                if now < deadline:
                    self._cv.wait(deadline - now)
                    continue
                self._tasks.pop(0)
            if not handle[0]:
                continue
            try:
                fn()
            except Exception:  # noqa: BLE001
                log.exception("scheduled task failed")
            with self._cv:
                if handle[0]:
                    self._tasks.append((time.monotonic() + interval, seq, fn, interval, handle))


_scheduler: Optional[_Scheduler] = None
_sched_lock = threading.Lock()


def scheduler() -> _Scheduler:
    global _scheduler
    with _sched_lock:
        if _scheduler is None:
            _scheduler = _Scheduler()
        return _scheduler


class BatchExecutor(Generic[T]):
    """Flush a batch when it reaches ``batch_size`` or after ``flush_interval_ms`` idle."""

    def __init__(self, batch_size: int, processor: Callable[[List[T]], None], flush_interval_ms: int):
        self.batch_size = max(1, batch_size)
        self.processor = processor
        self.flush_interval_ms = flush_interval_ms
        self._batch: List[T] = []
        self._lock = threading.Lock()
        self._handle = None

    def start(self) -> None:
        if self.flush_interval_ms > 0:
            self._handle = scheduler().schedule_fixed_delay(self.flush, self.flush_interval_ms / 1000.0)

    def stop(self) -> None:
        if self._handle is not None:
            _Scheduler.cancel(self._handle)
        self.flush()

    def add(self, item: T) -> None:
        to_run = None
        with self._lock:
            self._batch.append(item)
            if len(self._batch) >= self.batch_size or self.flush_interval_ms <= 0:
                to_run, self._batch = self._batch, []
        if to_run:
            self.processor(to_run)

    def flush(self) -> None:
        with self._lock:
            to_run, self._batch = self._batch, []
        if to_run:
            self.processor(to_run)


class OrderedAsyncBatchExecutor(Generic[T]):
    """Hash items into ``num_buckets`` buckets; each bucket runs at most ONE async batch
    at a time and queues the rest, so per-key order is preserved while the bucket count
    bounds concurrency.  ``processor(batch, future)`` must complete ``future``."""

    def __init__(self, batch_size: int, processor: Callable[[List[T], Future], None], flush_interval_ms: int,
                 num_buckets: int, hash_fn: Callable[[T], int]):
        self.batch_size = max(1, batch_size)
        self.processor = processor
        self.flush_interval_ms = flush_interval_ms
        self.num_buckets = max(1, num_buckets)
        self.hash_fn = hash_fn
        self._buckets = [_Bucket(self) for _ in range(self.num_buckets)]
        self._handle = None

    def start(self) -> None:
        if self.flush_interval_ms > 0:
            self._handle = scheduler().schedule_fixed_delay(self.flush, self.flush_interval_ms / 1000.0)

    def stop(self) -> None:
        if self._handle is not None:
            _Scheduler.cancel(self._handle)
        self.flush()

    def flush(self) -> None:
        for b in self._buckets:
            b.flush()

    def add(self, item: T) -> None:
        h = self.hash_fn(item)
        b = self._buckets[0] if self.num_buckets == 1 else self._buckets[abs(h) % self.num_buckets]
        b.add(item)


class _Bucket:
    def __init__(self, owner: OrderedAsyncBatchExecutor):
        self.owner = owner
        self.pending: deque = deque()
        self.current: list = []
        self.processing = False
        self.lock = threading.RLock()

    def add(self, item) -> None:
        with self.lock:
            self.current.append(item)
            if len(self.current) >= self.owner.batch_size or self.owner.flush_interval_ms <= 0:
                self._schedule_current()

    def flush(self) -> None:
        with self.lock:
            self._schedule_current()

    def _schedule_current(self) -> None:
        if not self.current:
            return
        batch, self.current = self.current, []
        if not self.processing:
            self._execute(batch)
        else:
            self.pending.append(batch)

    def _execute(self, batch) -> None:
        self.processing = True
        fut: Future = Future()

        def done(_f):
            with self.lock:
                self.processing = False
                if self.pending:
                    self._execute(self.pending.popleft())

        fut.add_done_callback(done)
        try:
            self.owner.processor(batch, fut)
        except Exception as e:  # noqa: BLE001
            log.exception("batch processor raised")
            if not fut.done():
                fut.set_exception(e)


class MicroBatcher(Generic[T]):
    """Opportunistic batching without added latency: a worker thread takes the first
    queued item and everything else already queued (up to ``max_batch``), runs
    ``fn(items) -> results`` once, and resolves each item's Future.  Under load calls
    coalesce into large batches (one GPU launch); when idle an item runs alone at once."""

    def __init__(self, fn: Callable[[List[T]], List[Any]], max_batch: int = 64, name: str = "micro-batcher"):
        import queue as _q
        self.fn = fn
        self.max_batch = max(1, max_batch)
        self._q: "_q.Queue" = _q.Queue()
        self._thread = threading.Thread(target=self._run, name=name, daemon=True)
        self._thread.start()

    def submit(self, item: T) -> Future:
        f: Future = Future()
        self._q.put((item, f))
        return f

    def _run(self) -> None:
        import queue as _q
        from ..utils.profiling import ThreadProfiler
        prof = ThreadProfiler(self._thread.name)
        while True:
            prof.tick()
            first = self._q.get()
            batch = [first]
            while len(batch) < self.max_batch:
                try:
                    batch.append(self._q.get_nowait())
                except _q.Empty:
                    break
            try:
                res = self.fn([b[0] for b in batch])
                for (_, f), r in zip(batch, res):
                    f.set_result(r)
            except BaseException as e:  # noqa: BLE001
                for _, f in batch:
                    if not f.done():
                        f.set_exception(e)
