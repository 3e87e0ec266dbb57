"""Runtime agent-code registry: agent type -> AgentCode factory.

The reference discovers implementations through NAR index files and ServiceLoader
(CORE/nar/NarFileHandler.java, API/runner/code/AgentCodeProvider.java).  Here modules
register factories on import; third-party plugins can call :func:`register_agent` or
expose an entry point ``langstream_amd.agents``.
"""
from __future__ import annotations

import importlib
import logging
import threading
from typing import Callable, Dict

log = logging.getLogger(__name__)

_FACTORIES: Dict[str, Callable[[], object]] = {}
_loaded = False
_lock = threading.Lock()

_BUILTIN_MODULES = (
    "langstream_amd.agents.builtin",
    "langstream_amd.agents.genai.agent",
    "langstream_amd.agents.text",
    "langstream_amd.agents.flow",
    "langstream_amd.agents.vector",
    "langstream_amd.agents.rerank",
    "langstream_amd.agents.flare",
    "langstream_amd.agents.http",
    "langstream_amd.agents.webcrawler",
    "langstream_amd.agents.storage",
    "langstream_amd.agents.python_agents",
    "langstream_amd.agents.kafka_connect",
)


def register_agent(*types: str):
    """Decorator/func: register an AgentCode class (or factory) for agent types."""
    def deco(factory):
        for t in types:
            _FACTORIES[t] = factory
        return factory
    return deco


def _load_builtins() -> None:
    global _loaded
    with _lock:
        if _loaded:
            return
        for m in _BUILTIN_MODULES:
            try:
                importlib.import_module(m)
            except ImportError as e:
                log.debug("agent module %s unavailable: %s", m, e)
        try:
            from importlib.metadata import entry_points
            for ep in entry_points().select(group="langstream_amd.agents"):
                try:
                    ep.load()
                except Exception:  # noqa: BLE001
                    log.exception("failed to load agent plugin %s", ep.name)
        except Exception:  # noqa: BLE001
            pass
        _loaded = True


def create_agent(agent_type: str):
    _load_builtins()
    f = _FACTORIES.get(agent_type)
    if f is None:
        raise ValueError(f"No agent code registered for type {agent_type}; known: {sorted(_FACTORIES)}")
    return f()


def known_agent_types():
    _load_builtins()
    return sorted(_FACTORIES)
