"""Per-rank heartbeats and a stall detector for multi-process jobs (bench.py, TP pods).

A multi-GPU job whose one rank hangs -- in a collective, a kernel that never finishes, a
dead peer -- otherwise leaves every other rank blocked in its next collective until an
outer timeout kills the whole job with no hint of where it stopped.  Each rank here
publishes ``(phase, beat count, time)`` in the job's c10d store whenever it makes
progress (``phase()`` / ``beat()`` from the main loop, never from a timer, so a hung rank
stops beating), and a daemon thread on every rank checks its OWN last beat against the
phase's limit.  When it is exceeded the thread reads every rank's last beat, prints one
JSON line naming the phase and the suspect rank (the rank the others are waiting for: one
that never beat, else one not blocked in a collective -- ``arrive()`` marks a rank about
to block -- oldest beat first), and ends the process with ``exit_code`` -- every rank of a
stalled job exits non-zero within one limit instead of hanging.

The thread runs while the main thread waits inside RCCL / gloo / a device synchronize
(they release the GIL).  ``LS_WATCHDOG=0`` disables it.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from typing import Any, Dict, Optional


class RankWatchdog:
    def __init__(self, rank: int, world: int, store=None, poll_s: float = 2.0, exit_code: int = 3,
                 prefix: str = "lsw", out=None, exit_fn=None):
        self.rank, self.world = rank, world
        self.store = store if store is not None else _default_store()
        self.poll_s = poll_s
        self.exit_code = exit_code
        self.prefix = prefix
        self.out = out or sys.stderr
        self._exit = exit_fn or os._exit
        self._phase = "start"
        self._limit = float("inf")
        self._last = time.time()
        self._beats = 0
        self._waiting: Optional[str] = None
        self._pub = 0.0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.fired: Optional[Dict[str, Any]] = None

    # ------------------------------------------------------------------ main-thread API
    def start(self) -> "RankWatchdog":
        if os.environ.get("LS_WATCHDOG", "1") == "0":
            return self
        self._publish(force=True)
        self._thread = threading.Thread(target=self._run, name=f"rank-watchdog-{self.rank}", daemon=True)
        self._thread.start()
        return self

    def phase(self, name: str, limit_s: float) -> None:
        """Enter ``name``: this rank must beat (or change phase) at least every ``limit_s``."""
        self._phase, self._limit = name, float(limit_s)
        self._waiting = None
        self.beat(force=True)

    def beat(self, force: bool = False) -> None:
        self._last = time.time()
        self._beats += 1
        self._waiting = None
        self._publish(force)

    def arrive(self, what: str) -> None:
        """About to block in a collective / barrier ``what``: a rank that stalls while the
        others have all arrived is the one they wait for (the report's suspect)."""
        self._waiting = what
        self._publish(force=True)

    def stop(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ internals
    def _key(self, r: int) -> str:
        return f"{self.prefix}/{r}"

    def _publish(self, force: bool = False) -> None:
        now = time.time()
        if not force and now - self._pub < 1.0:      # at most one store round trip per second
            return
        self._pub = now
        try:
            self.store.set(self._key(self.rank), json.dumps({"phase": self._phase, "beats": self._beats,
                                                              "t": self._last, "waiting": self._waiting}))
        except Exception:  # noqa: BLE001  (the store's host may be the one that died)
            pass

    def _snapshot(self) -> Dict[int, Any]:
        out: Dict[int, Any] = {}
        now = time.time()
        for r in range(self.world):
            try:
                if not self.store.check([self._key(r)]):
                    out[r] = None
                    continue
                d = json.loads(self.store.get(self._key(r)))
                out[r] = {"phase": d["phase"], "beats": d["beats"], "age_s": round(now - d["t"], 1),
                          "waiting": d.get("waiting")}
            except Exception as e:  # noqa: BLE001
                out[r] = {"error": repr(e)}
        return out

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            stalled = time.time() - self._last
            if stalled <= self._limit:
                continue
            ranks = self._snapshot()
            known = {r: v for r, v in ranks.items() if isinstance(v, dict) and "age_s" in v}
            missing = [r for r, v in ranks.items() if v is None]
            # the rank the others wait for: one that never published, else one not blocked
            # in a collective (stuck in its own work), oldest beat first
            busy = {r: v for r, v in known.items() if not v.get("waiting")}
            pool = busy or known
            suspect = missing[0] if missing else (max(pool, key=lambda r: pool[r]["age_s"]) if pool else None)
            self.fired = {"error": "rank stalled", "rank": self.rank, "phase": self._phase,
                          "stalled_s": round(stalled, 1), "limit_s": self._limit, "suspect_rank": suspect,
                          "suspect_phase": (known.get(suspect) or {}).get("phase") if suspect is not None else None,
                          "ranks": ranks}
            try:
                print(json.dumps(self.fired), file=self.out, flush=True)
            finally:
                self._exit(self.exit_code)
            return


def _default_store():
    import torch.distributed as dist
    from torch.distributed import distributed_c10d as c10d
    if not dist.is_initialized():
        raise RuntimeError("RankWatchdog needs an initialised default process group (or an explicit store)")
    return c10d._get_default_store()
