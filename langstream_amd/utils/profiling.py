"""Opt-in per-thread cProfile for long-running service threads.

``LANGSTREAM_PROFILE_THREADS="llm-engine,query-batcher"`` (or ``*``) profiles the named
threads; each dumps cumulative stats to ``$LANGSTREAM_PROFILE_DIR/<thread>.txt``
(default ``gpurun_out/``) every ``LANGSTREAM_PROFILE_EVERY_S`` seconds from inside
the thread (cProfile is per-thread, so enable/disable must happen there).

Usage in a thread body::

    prof = ThreadProfiler("query-batcher")
    while True:
        ...work...
        prof.tick()
"""
from __future__ import annotations

import os
import time


class ThreadProfiler:
    def __init__(self, name: str):
        sel = os.environ.get("LANGSTREAM_PROFILE_THREADS", "")
        self.name = name
        self.on = bool(sel) and (sel == "*" or name in {s.strip() for s in sel.split(",")})
        self.pr = None
        if self.on:
            import cProfile
            self.out_dir = os.environ.get("LANGSTREAM_PROFILE_DIR", "gpurun_out")
            self.every = float(os.environ.get("LANGSTREAM_PROFILE_EVERY_S", "10"))
            self.last = time.monotonic()
            self.pr = cProfile.Profile()
            self.pr.enable()

    def tick(self, force: bool = False) -> None:
        if not self.on or (not force and time.monotonic() - self.last < self.every):
            return
        import pstats
        self.pr.disable()
        try:
            os.makedirs(self.out_dir, exist_ok=True)
            with open(os.path.join(self.out_dir, f"{self.name}.txt"), "w") as f:
                pstats.Stats(self.pr, stream=f).sort_stats("cumulative").print_stats(70)
        except Exception:  # noqa: BLE001
            pass
        self.last = time.monotonic()
        self.pr.enable()
