"""Local application runner -- the ``langstream docker run`` equivalent.

Parity: TESTER/LocalApplicationRunner.java:79-297 and TESTER/Main.java:53-205: parse
the application, plan it, set up topics/assets, and run every agent "pod" in-process.
Unlike the reference (one thread per agent, ``parallelism`` ignored), every replica of
an agent gets its own runner thread and they share the agent's consumer group, so
``resources.parallelism`` is honoured (replica data-parallelism over partitions).
The GPU services (LLM / embedding engines, vector store) are process-wide singletons
shared by all agents (``langstream_amd.services``).
"""
from __future__ import annotations

import logging
import os
import tempfile
import threading
import time
from typing import Any, Dict, List, Optional

from ..api.model import Application, Instance, StreamingCluster, ComputeCluster
from ..api.record import Header, Record, SimpleRecord
from ..api.topics import TopicConnectionsRuntimeRegistry, TopicOffsetPosition
from ..core.deployer import ApplicationDeployer, pod_configuration
from ..core.parser import build_application_instance, build_from_directory
from ..utils import gctune
from ..core.planner import ExecutionPlan
from .runner import AgentRunner

log = logging.getLogger(__name__)


class LocalApplicationRunner:
    def __init__(self, application: Application, application_id: str = "app", tenant: str = "default",
                 code_directory: str = "", state_dir: Optional[str] = None, services=None,
                 agents: Optional[List[str]] = None):
        if application.instance is None or application.instance.streaming_cluster is None:
            g = application.instance.globals if application.instance else {}
            application.instance = Instance(StreamingCluster("memory", {}), ComputeCluster("none", {}), g)
        self.application = application
        self.application_id = application_id
        self.tenant = tenant
        self.code_directory = code_directory
        self.state_dir = state_dir or tempfile.mkdtemp(prefix="langstream-state-")
        self.deployer = ApplicationDeployer()
        self.plan: ExecutionPlan = self.deployer.create_implementation(application_id, application)
        self.only_agents = agents
        if services is None:
            from ..services import ServiceRegistry
            services = ServiceRegistry.default()
        self.services = services
        self.runners: List[AgentRunner] = []
        self.threads: List[threading.Thread] = []
        self.errors: List[BaseException] = []
        self._topic_rt = None

    # ------------------------------------------------------------------ construction helpers
    @staticmethod
    def from_directory(app_dir: str, instance_file: Optional[str] = None, secrets_file: Optional[str] = None,
                       **kw) -> "LocalApplicationRunner":
        info = build_from_directory(app_dir, instance_file, secrets_file)
        kw.setdefault("code_directory", app_dir)
        return LocalApplicationRunner(info.application, **kw)

    @staticmethod
    def from_yaml(files: Dict[str, str], instance: Optional[str] = None, secrets: Optional[str] = None,
                  **kw) -> "LocalApplicationRunner":
        info = build_application_instance(files, instance, secrets)
        return LocalApplicationRunner(info.application, **kw)

    # ------------------------------------------------------------------ lifecycle
    @property
    def streaming_cluster(self):
        return self.plan.application.instance.streaming_cluster

    @property
    def topic_runtime(self):
        if self._topic_rt is None:
            self._topic_rt = TopicConnectionsRuntimeRegistry.get(self.streaming_cluster)
        return self._topic_rt

    def start(self, wait: float = 10.0) -> "LocalApplicationRunner":
        self.deployer.setup(self.tenant, self.plan)
        for key, node in self.plan.agents.items():
            if self.only_agents and node.id not in self.only_agents:
                continue
            replicas = max(1, int(node.resources.parallelism or 1))
            for rep in range(replicas):
                pod = pod_configuration(self.plan, node, self.tenant, self.code_directory,
                                        os.path.join(self.state_dir, node.id), rep)
                os.makedirs(pod.persistent_state_directory, exist_ok=True)
                runner = AgentRunner(pod, services=self.services)
                runner.build()
                t = threading.Thread(target=self._run, args=(runner,), name=f"agent-{node.id}-{rep}", daemon=True)
                self.runners.append(runner)
                self.threads.append(t)
        for t in self.threads:
            t.start()
        deadline = time.time() + wait
        for r in self.runners:
            r.started.wait(max(0.0, deadline - time.time()))
        gctune.tune()   # startup heap -> permanent generation, rare full collections
        return self

    def _run(self, runner: AgentRunner) -> None:
        try:
            runner.run()
        except BaseException as e:  # noqa: BLE001
            log.exception("agent %s failed", runner.pod.agent_id)
            self.errors.append(e)

    def stop(self, timeout: float = 30.0) -> None:
        for r in self.runners:
            r.stop()
        deadline = time.time() + timeout
        for t in self.threads:
            t.join(max(0.1, deadline - time.time()))

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()

    # ------------------------------------------------------------------ topic helpers (tests / CLI)
    def _conn(self, topic: str, producer: bool) -> Dict[str, Any]:
        """The plan topic's connection configuration (schemas / serde), as an agent gets it."""
        t = self.plan.get_topic(topic)
        if t is None:
            return {"topic": topic}
        return t.producer_configuration() if producer else t.consumer_configuration()

    def producer(self, topic: str):
        p = self.topic_runtime.create_producer("local-client", self.streaming_cluster, self._conn(topic, True))
        p.start()
        return p

    def produce(self, topic: str, value: Any, key: Any = None, headers: Optional[Dict[str, Any]] = None) -> None:
        hs = [Header(k, v) for k, v in (headers or {}).items()]
        self.producer(topic).write(SimpleRecord.of(key, value, hs)).result(10)

    def reader(self, topic: str, position: TopicOffsetPosition = TopicOffsetPosition.EARLIEST):
        r = self.topic_runtime.create_reader(self.streaming_cluster, self._conn(topic, False), position)
        r.start()
        return r

    def consume(self, topic: str, n: int, timeout: float = 30.0,
                position: TopicOffsetPosition = TopicOffsetPosition.EARLIEST) -> List[Record]:
        rd = self.reader(topic, position)
        out: List[Record] = []
        deadline = time.time() + timeout
        while len(out) < n and time.time() < deadline:
            if self.errors:
                raise self.errors[0]
            out.extend(rd.read().records)
        return out

    def agent_info(self) -> Dict[str, Any]:
        return {f"{r.pod.agent_id}-{r.pod.replica}": r.agent_info() for r in self.runners}
