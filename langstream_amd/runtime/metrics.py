"""Metrics (RT/agent/metrics/PrometheusMetricsReporter.java:24-108): one global counter
per (sanitised) metric name labelled by ``agent_id``; exposed as Prometheus text on
``/metrics``.  Also holds latency histograms used by the benchmarks."""
from __future__ import annotations

import re
import threading
from typing import Dict, Optional

try:
    import prometheus_client as prom
except ImportError:  # pragma: no cover
    prom = None

_SAN = re.compile(r"[^a-zA-Z0-9_]")


def sanitize(name: str) -> str:
    n = _SAN.sub("_", name)
    return n if not n[:1].isdigit() else "_" + n


class _Counter:
    def __init__(self, c, labels):
        self._c = c
        self._labels = labels
        self._child = c.labels(**labels) if c is not None else None   # resolved once, not per inc
        self.value = 0.0
        self._lock = threading.Lock()

    def inc(self, n: float = 1.0) -> None:
        with self._lock:
            self.value += n
        if self._child is not None:
            self._child.inc(n)

    def count(self) -> float:
        return self.value


class MetricsReporter:
    _global: Optional["MetricsReporter"] = None
    _glock = threading.Lock()

    def __init__(self, prefix: str = "langstream", agent_id: Optional[str] = None,
                 registry=None, pod: Optional[str] = None):
        self.prefix = prefix
        self.agent_id = agent_id
        self.pod = pod
        self.registry = registry if registry is not None else (prom.CollectorRegistry() if prom else None)
        self._counters: Dict[str, object] = {}
        self._lock = threading.Lock()
        self._children: Dict[tuple, _Counter] = {}

    @classmethod
    def global_reporter(cls) -> "MetricsReporter":
        with cls._glock:
            if cls._global is None:
                cls._global = MetricsReporter()
            return cls._global

    def with_agent(self, agent_id: str) -> "MetricsReporter":
        child = MetricsReporter.__new__(MetricsReporter)
        child.__dict__ = dict(self.__dict__)
        child.agent_id = agent_id
        child._root = getattr(self, "_root", self)
        return child

    def counter(self, name: str, agent_id: Optional[str] = None, help_: str = "") -> _Counter:
        root = getattr(self, "_root", self)
        agent = agent_id or self.agent_id or "unknown"
        full = sanitize(f"{self.prefix}_{name}")
        with root._lock:
            key = (full, agent)
            c = root._children.get(key)
            if c is not None:
                return c
            pc = root._counters.get(full)
            labels = ["agent_id"] + (["pod"] if self.pod else [])
            if pc is None and prom is not None:
                pc = prom.Counter(full, help_ or name, labels, registry=root.registry)
                root._counters[full] = pc
            lv = {"agent_id": agent}
            if self.pod:
                lv["pod"] = self.pod
            c = _Counter(pc, lv)
            root._children[key] = c
            return c

    def exposition(self) -> bytes:
        root = getattr(self, "_root", self)
        if prom is None or root.registry is None:
            lines = [f"{n}{{agent_id=\"{a}\"}} {c.value}" for (n, a), c in root._children.items()]
            return ("\n".join(lines) + "\n").encode()
        return prom.generate_latest(root.registry)
