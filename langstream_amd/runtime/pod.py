"""Agent pod entrypoint + agent HTTP API.

Parity: ``RT/agent/AgentRunnerStarter.java:40-135`` (pod configuration from argv or
``LANGSTREAM_AGENT_RUNNER_POD_CONFIGURATION``, code dir ``LANGSTREAM_AGENT_RUNNER_CODE_PATH``,
persistent state dir ``LANGSTREAM_AGENT_RUNNER_PERSISTENT_STATE_DIRECTORY``; a fatal
error waits 60 s then exits non-zero so the StatefulSet restarts the pod),
``RT/agent/api/AgentAPIController.java:27-87`` (``GET /metrics`` Prometheus text,
``GET /info`` list of AgentStatusResponse, ``POST /commands/restart``).

The pod configuration is the JSON written by ``core.k8s.agent_pod_configuration``.
Replica index: the StatefulSet ordinal (``HOSTNAME`` suffix) or ``RANK``.  Under
``torchrun`` (tensor-parallel chat agents) rank 0 runs the agent loop and the other
ranks serve the LLM engine's TP worker loop (``services.ServiceRegistry``).
"""
from __future__ import annotations

import json
import logging
import os
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, Tuple

from .metrics import MetricsReporter
from .runner import AgentRunner, RuntimePodConfiguration

log = logging.getLogger(__name__)


class AgentAPIServer:
    """/metrics, /info, /commands/restart for a set of runners (one pod, or every
    agent thread in local mode -- the docker-run agent-control port 8790)."""

    def __init__(self, runners: List[AgentRunner], host: str = "0.0.0.0", port: int = 8080,
                 metrics: Optional[MetricsReporter] = None):
        self.runners = runners
        self.metrics = metrics or MetricsReporter.global_reporter()
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body: bytes, ctype="application/json"):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):
                if self.path.startswith("/metrics"):
                    self._send(200, outer.metrics.exposition(), "text/plain; version=0.0.4")
                elif self.path.startswith("/info"):
                    info = []
                    for r in outer.runners:
                        try:
                            info += r.agent_info()
                        except Exception as e:  # noqa: BLE001
                            info.append({"agent-id": r.pod.agent_id, "error": str(e)})
                    self._send(200, json.dumps(info, default=str).encode())
                else:
                    self._send(404, b"{}")

            def do_POST(self):
                if self.path.startswith("/commands/restart"):
                    for r in outer.runners:
                        r.restart()
                    self._send(200, b"{}")
                else:
                    self._send(404, b"{}")

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="agent-api")

    def start(self) -> "AgentAPIServer":
        self.thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()


def load_pod_configuration(path: str, code_dir: str = "", state_dir: Optional[str] = None,
                           replica: int = 0) -> RuntimePodConfiguration:
    from ..api.model import StreamingCluster
    with open(path) as f:
        c = json.load(f)
    a = c["agent"]
    sc = c.get("streamingCluster")
    eh = a.get("errorHandlerConfiguration") or {}
    return RuntimePodConfiguration(
        agent_id=a["agentId"], agent_type=a["agentType"], component_type=a.get("componentType", "PROCESSOR"),
        application_id=a["applicationId"], tenant=a.get("tenant", "default"), configuration=a.get("configuration")
        or {}, input=c.get("input") or {}, output=c.get("output") or {},
        streaming_cluster=StreamingCluster(sc["type"], sc.get("configuration") or {}) if sc else None,
        errors={"retries": eh.get("retries", 0), "onFailure": eh.get("onFailure", "fail")},
        code_directory=code_dir, persistent_state_directory=state_dir, replica=replica)


def _replica_index() -> int:
    host = os.environ.get("HOSTNAME", "")
    tail = host.rsplit("-", 1)[-1]
    if tail.isdigit():
        return int(tail)
    if int(os.environ.get("WORLD_SIZE", "1") or 1) > 1:
        return 0   # torchrun ranks of a TP pod are one replica
    return int(os.environ.get("RANK", "0"))


def chat_engine_request(configuration: Dict[str, Any]) -> Tuple[Optional[str], Dict[str, Any]]:
    """(model, local-engine config) of a planned ai-chat/text-completions agent: the
    GenAI planner stores ``{steps: [{type, model, ...}], <service-key>: resource}``."""
    steps = configuration.get("steps") or [configuration]
    model = steps[0].get("model")
    for key in ("local", "openai"):
        res = configuration.get(key)
        if isinstance(res, dict) and (key == "local" or res.get("provider") == "local"):
            return model, res
    raise ValueError("tensor-parallel pods need a local-gpu-configuration chat agent")


def serve_tp_worker(configuration: Dict[str, Any], services=None) -> int:
    """TP ranks > 0: build the same engine as rank 0 (weights shard, KV pool, lock-step
    graph capture) and mirror its steps until rank 0 stops the engine."""
    from ..services import ServiceRegistry
    reg = services or ServiceRegistry.default()
    model, res = chat_engine_request(configuration)
    eng = reg.llm_engine(model, res)
    eng.worker_loop()
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    logging.basicConfig(level=os.environ.get("LANGSTREAM_LOG_LEVEL", "INFO"),
                        format="%(asctime)s %(levelname)s %(threadName)s %(name)s %(message)s")
    cfg = argv[0] if argv else os.environ.get("LANGSTREAM_AGENT_RUNNER_POD_CONFIGURATION")
    if not cfg:
        print("usage: python -m langstream_amd.runtime.pod <pod-configuration.json>", file=sys.stderr)
        return 2
    code = os.environ.get("LANGSTREAM_AGENT_RUNNER_CODE_PATH", "")
    state = os.environ.get("LANGSTREAM_AGENT_RUNNER_PERSISTENT_STATE_DIRECTORY")
    tp_world = int(os.environ.get("WORLD_SIZE", "1") or 1)
    if tp_world > 1:
        # torchrun inside one pod = one tensor-parallel chat agent replica
        from ..parallel import init_tensor_parallel
        from ..services import ServiceRegistry
        reg = ServiceRegistry.default()
        reg.tp = init_tensor_parallel(tp_world)
        if reg.tp.rank != 0:
            pod = load_pod_configuration(cfg, code, state, _replica_index())
            return serve_tp_worker(pod.configuration, reg)
    pod = load_pod_configuration(cfg, code, state, _replica_index())
    runner = AgentRunner(pod)
    api = AgentAPIServer([runner], port=int(os.environ.get("LANGSTREAM_AGENT_HTTP_PORT", "8080"))).start()
    stop = threading.Event()
    try:
        import signal
        signal.signal(signal.SIGTERM, lambda *_: (runner.stop(), stop.set()))
    except (ValueError, OSError):
        pass
    from ..utils import gctune
    ready = os.environ.get("LANGSTREAM_AGENT_READY_FILE")

    def on_started():
        runner.started.wait()
        if ready:
            # the local runner's replica processes wait for this (runtime/local.py)
            open(ready, "w").close()
        gctune.tune()
    threading.Thread(target=on_started, name="gc-tune", daemon=True).start()
    try:
        runner.run()
        return 0
    except Exception as e:  # noqa: BLE001
        log.exception("agent %s failed: %s", pod.agent_id, e)
        # like AgentRunnerStarter: give operators time to read the logs, then exit non-zero
        stop.wait(float(os.environ.get("LANGSTREAM_FATAL_WAIT_S", "60")))
        return 1
    finally:
        api.stop()


if __name__ == "__main__":
    sys.exit(main())
