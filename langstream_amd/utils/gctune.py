"""Garbage-collector policy for a running application process.

An agent process allocates millions of small objects per second (records, headers,
token lists) on top of a large, long-lived startup heap (loaded models' Python-side
state, vector-store metadata, plan objects).  CPython's default thresholds (700, 10, 10)
then run a full (gen-2) collection every few seconds that walks the whole startup heap
while holding the GIL, and every agent thread -- including the LLM engine's scheduler,
whose next GPU step waits for it -- stalls for 100+ ms (the RAG bench measured 419 ms of
GC pause per 9.7 s, 3 full collections; `bench.py` reports `gc_rank0`).

`tune()` (called once the application's agents are running):
  * `gc.freeze()` moves everything alive at that point to the permanent generation, so
    later collections never traverse the startup heap;
  * thresholds (50000, 20, 100): young collections every 50k net allocations, full
    collections rarely.
Cycles are still collected.  LANGSTREAM_GC=default keeps CPython's policy;
LANGSTREAM_GC_GEN0 overrides the young-generation threshold.  (Round 3, one box,
alternating runs: 400000 removes the two ~30 ms young collections of 3 RAG steps but
measured 118.3 / 119.0 records/s against 122.0 / 121.3 at 50000 -- profiles/gc_r3c/.)
"""
from __future__ import annotations

import gc
import os
import sys

_done = False


def tune() -> bool:
    global _done
    if _done or os.environ.get("LANGSTREAM_GC", "tuned") == "default":
        return False
    gc.collect()
    gc.freeze()
    gc.set_threshold(int(os.environ.get("LANGSTREAM_GC_GEN0", "50000")), 20, 100)
    sw = os.environ.get("LANGSTREAM_SWITCH_MS")
    if sw:
        # GIL hand-off interval: a thread coming back from a GIL-released native call
        # (a GPU step, a socket read) waits up to this long for a Python-busy thread
        sys.setswitchinterval(float(sw) / 1000.0)
    _done = True
    return True
