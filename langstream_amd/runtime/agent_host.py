"""A pre-started process that later runs a subset of an application's agents.

Agents of a LangStream application run in their own pods; on one host the local runner
runs them as threads of one interpreter.  ``AgentHostProcess`` gives selected agents an
interpreter of their own without spawning it late: the child starts EARLY (before the
parent initialises the GPU -- a process that has done so must not fork+exec children on
some hosts), idles, and when told builds a ``LocalApplicationRunner`` for the named
agents on the same (cross-process) streaming cluster.  Used by the config-4 bench for
the webcrawler source (rank 0 otherwise serves the crawl for every rank from the same
interpreter as its query pipeline and engine thread).

Protocol on stdin / stdout, one JSON line each way:
  parent -> {"files": {...}, "instance": "...", "application_id": "...", "agents": [...],
             "state_dir": "..."}          child -> {"started": true} | {"error": "..."}
  parent closes stdin                     child stops the agents and exits
"""
from __future__ import annotations

import json
import sys
import threading
from typing import Dict, List, Optional


def main() -> int:
    line = sys.stdin.readline()
    if not line.strip():
        return 0
    req = json.loads(line)
    try:
        from .local import LocalApplicationRunner
        runner = LocalApplicationRunner.from_yaml(req["files"], instance=req.get("instance"),
                                                  application_id=req.get("application_id", "app"),
                                                  agents=req["agents"], state_dir=req.get("state_dir"))
        runner.start(wait=float(req.get("wait", 60.0)))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"error": f"{type(e).__name__}: {e}"}), flush=True)
        return 1
    print(json.dumps({"started": True}), flush=True)
    done = threading.Event()

    def watch():
        try:
            sys.stdin.read()
        except Exception:  # noqa: BLE001
            pass
        done.set()
    threading.Thread(target=watch, daemon=True).start()
    while not done.wait(0.5):
        if runner.errors:
            print(json.dumps({"error": repr(runner.errors[0])}), flush=True)
            break
    runner.stop(10)
    return 0


class AgentHostProcess:
    def __init__(self, env: Optional[Dict[str, str]] = None):
        from ..utils.procs import spawn_module
        self.proc = spawn_module("langstream_amd.runtime.agent_host", env=env)

    def start(self, files: Dict[str, str], instance: Optional[str], application_id: str, agents: List[str],
              state_dir: Optional[str] = None, wait: float = 60.0) -> None:
        self.proc.stdin.write(json.dumps({"files": files, "instance": instance, "application_id": application_id,
                                          "agents": agents, "state_dir": state_dir, "wait": wait}) + "\n")
        self.proc.stdin.flush()
        reply = self.proc.stdout.readline()
        msg = json.loads(reply) if reply.strip() else {"error": f"agent host exited ({self.proc.poll()})"}
        if not msg.get("started"):
            raise RuntimeError(f"agent host for {agents}: {msg.get('error')}")

    def alive(self) -> bool:
        return self.proc.poll() is None

    def stop(self, timeout: float = 20.0) -> None:
        from ..utils.procs import close_stdin_and_wait
        close_stdin_and_wait(self.proc, timeout)


if __name__ == "__main__":
    raise SystemExit(main())
