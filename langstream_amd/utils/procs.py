"""Child interpreters for the pieces that run beside an agent process on one host: the
in-tree Kafka broker, the bench's load clients and crawl site, agent hosts and agent-pod
replicas.  One place for the environment rules:

* the repository root is put on ``PYTHONPATH`` (the child runs ``-m langstream_amd...``
  from any working directory);
* children that do not use the GPU get ``CUDA_VISIBLE_DEVICES`` / ``HIP_VISIBLE_DEVICES``
  emptied, so importing torch there never touches the device;
* the parent's ``torch.distributed`` rank variables are dropped unless asked for: a child
  is not a rank of the parent's process group.

Start children before the parent initialises the GPU where possible (a process that has
initialised it should not fork + exec on some hosts).
"""
from __future__ import annotations

import os
import subprocess
import sys
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DIST_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "MASTER_ADDR", "MASTER_PORT",
             "TORCHELASTIC_RUN_ID")


def child_env(gpu: bool = False, keep_dist: bool = False, extra: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([ROOT, env.get("PYTHONPATH", "")]).rstrip(os.pathsep)
    if not gpu:
        env["CUDA_VISIBLE_DEVICES"] = ""
        env["HIP_VISIBLE_DEVICES"] = ""
    if not keep_dist:
        for k in DIST_VARS:
            env.pop(k, None)
    env.update(extra or {})
    return env


def spawn_module(module: str, args: List[str] = (), *, gpu: bool = False, keep_dist: bool = False,
                 env: Optional[Dict[str, str]] = None, pipes: bool = True) -> subprocess.Popen:
    """``python -m module args...`` with text-mode stdin/stdout pipes (the control channel)."""
    kw = dict(stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True) if pipes else {}
    return subprocess.Popen([sys.executable, "-m", module, *args], env=child_env(gpu, keep_dist, env), **kw)


def read_tagged(proc: subprocess.Popen, prefix: str, what: str) -> str:
    """The child's first stdout line, which must start with ``prefix`` (its readiness
    message); the child is killed otherwise."""
    line = proc.stdout.readline().strip()
    if not line.startswith(prefix):
        proc.kill()
        raise RuntimeError(f"{what} failed to start: {line!r} (exit {proc.poll()})")
    return line[len(prefix):]


def close_stdin_and_wait(proc: subprocess.Popen, timeout: float = 10.0) -> None:
    """Children watch their stdin: closing it is their stop signal."""
    if proc.poll() is not None:
        return
    try:
        if proc.stdin is not None:
            proc.stdin.close()
        proc.wait(timeout)
    except Exception:  # noqa: BLE001
        proc.kill()
        proc.wait(5)
