"""Per-thread CPU accounting (Linux ``/proc``): which threads of this process burn CPU.

Used to diagnose GIL contention in the streaming runtime: the engine threads must not
be starved by agent threads.  ``snapshot()`` returns {thread name: cpu seconds}; diff
two snapshots around a measured region.
"""
from __future__ import annotations

import os
import threading
from typing import Dict

_CLK = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100


def snapshot() -> Dict[str, float]:
    names = {t.native_id: t.name for t in threading.enumerate() if t.native_id is not None}
    out: Dict[str, float] = {}
    base = f"/proc/{os.getpid()}/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/stat") as f:
                stat = f.read()
            with open(f"{base}/{tid}/comm") as f:
                comm = f.read().strip()
        except OSError:
            continue
        fields = stat[stat.rfind(")") + 2:].split()
        cpu = (int(fields[11]) + int(fields[12])) / _CLK  # utime + stime
        name = names.get(int(tid), f"native:{comm}")
        out[name] = out.get(name, 0.0) + cpu
    return out


def diff(a: Dict[str, float], b: Dict[str, float], top: int = 20) -> Dict[str, float]:
    d = {k: round(b.get(k, 0.0) - a.get(k, 0.0), 2) for k in set(a) | set(b)}
    return dict(sorted(((k, v) for k, v in d.items() if v > 0), key=lambda kv: -kv[1])[:top])
