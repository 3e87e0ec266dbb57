"""Local application runner -- the ``langstream docker run`` equivalent.

Parity: TESTER/LocalApplicationRunner.java:79-297 and TESTER/Main.java:53-205: parse
the application, plan it, set up topics/assets, and run every agent "pod" in-process.
Unlike the reference (one thread per agent, ``parallelism`` ignored), every replica of
an agent gets its own runner thread and they share the agent's consumer group, so
``resources.parallelism`` is honoured (replica data-parallelism over partitions).
The GPU services (LLM / embedding engines, vector store) are process-wide singletons
shared by all agents (``langstream_amd.services``).

``replica_processes=True`` (or ``LANGSTREAM_REPLICA_PROCESSES=1``) runs each replica of
an agent with ``parallelism`` > 1 as its own agent-pod process instead
(``python -m langstream_amd.runtime.pod``, the process a StatefulSet replica runs), when
the streaming cluster is reachable from other processes (kafka / pulsar / shm): each
replica then has its own interpreter -- and GIL -- and its own engines on the same GPU,
which is what scales a host-bound agent (per-record Python work) on one device.
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
                 agents: Optional[List[str]] = None, replica_processes: Optional[bool] = None):
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
        if replica_processes is None:
            replica_processes = os.environ.get("LANGSTREAM_REPLICA_PROCESSES", "") == "1"
        self.replica_processes = replica_processes
        self.processes: List["_PodProcess"] = []

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
            if replicas > 1 and self.replica_processes and self._cross_process():
                for rep in range(replicas):
                    self.processes.append(_PodProcess(self, node, rep))
                continue
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
        for p in self.processes:
            # engines load in every replica process: allow them longer than a thread
            p.wait_started(max(wait, 300.0))
        if self.processes:
            threading.Thread(target=self._watch_processes, name="replica-watch", daemon=True).start()
        gctune.tune()   # startup heap -> permanent generation, rare full collections
        return self

    def _run(self, runner: AgentRunner) -> None:
        try:
            runner.run()
        except BaseException as e:  # noqa: BLE001
            log.exception("agent %s failed", runner.pod.agent_id)
            self.errors.append(e)

    def _cross_process(self) -> bool:
        sc = self.streaming_cluster
        return sc is not None and sc.type in ("kafka", "pulsar", "shm")

    def _watch_processes(self) -> None:
        while self.processes and not all(p.stopping for p in self.processes):
            for p in self.processes:
                rc = p.proc.poll()
                if rc is not None and not p.stopping and not p.reported:
                    p.reported = True
                    self.errors.append(RuntimeError(f"agent {p.agent_id} replica {p.replica} exited with {rc}"))
            time.sleep(0.5)

    def stop(self, timeout: float = 30.0) -> None:
        for r in self.runners:
            r.stop()
        for p in self.processes:
            p.terminate()
        deadline = time.time() + timeout
        for t in self.threads:
            t.join(max(0.1, deadline - time.time()))
        for p in self.processes:
            p.join(max(0.1, deadline - time.time()))

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


class _PodProcess:
    """One agent replica as an agent-pod process (runtime/pod.py) on this host."""

    def __init__(self, owner: LocalApplicationRunner, node, replica: int):
        import json
        from ..core.k8s import agent_pod_configuration
        self.agent_id, self.replica = node.id, replica
        self.stopping = self.reported = False
        d = os.path.join(owner.state_dir, node.id, f"replica-{replica}")
        os.makedirs(d, exist_ok=True)
        cfg = os.path.join(d, "pod-configuration.json")
        with open(cfg, "w") as f:
            json.dump(agent_pod_configuration(owner.plan, node, owner.tenant), f, default=str)
        self.ready = os.path.join(d, "started")
        if os.path.exists(self.ready):
            os.remove(self.ready)
        from ..utils.procs import spawn_module
        # a replica pod uses the GPU (its own engines on the parent's device); torchrun's
        # ranks of the parent are not this pod's TP group
        self.proc = spawn_module("langstream_amd.runtime.pod", [cfg], gpu=True, pipes=False, env={
            "HOSTNAME": f"{node.id}-{replica}",              # the StatefulSet ordinal
            "LANGSTREAM_AGENT_HTTP_PORT": "0",
            "LANGSTREAM_AGENT_READY_FILE": self.ready,
            "LANGSTREAM_FATAL_WAIT_S": "0",
            "LANGSTREAM_AGENT_RUNNER_CODE_PATH": owner.code_directory or "",
            "LANGSTREAM_AGENT_RUNNER_PERSISTENT_STATE_DIRECTORY": d,
            "LOCAL_RANK": os.environ.get("LOCAL_RANK", "0")})

    def wait_started(self, timeout: float) -> None:
        deadline = time.time() + timeout
        while not os.path.exists(self.ready):
            if self.proc.poll() is not None:
                raise RuntimeError(f"agent {self.agent_id} replica {self.replica} exited with {self.proc.returncode}")
            if time.time() > deadline:
                raise TimeoutError(f"agent {self.agent_id} replica {self.replica} did not start in {timeout:.0f}s")
            time.sleep(0.05)

    def terminate(self) -> None:
        self.stopping = True
        if self.proc.poll() is None:
            self.proc.terminate()

    def join(self, timeout: float) -> None:
        try:
            self.proc.wait(timeout)
        except Exception:  # noqa: BLE001
            self.proc.kill()
            self.proc.wait(5)
