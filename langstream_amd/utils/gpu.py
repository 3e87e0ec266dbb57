"""GPU helpers shared by the auxiliary (non-LLM) GPU services.

The LLM engine keeps the default HIP stream of its device busy with back-to-back
steps (lookahead keeps two queued).  Latency-sensitive side work -- query embeddings,
vector-store kNN, upserts -- must not queue behind those steps, so it runs on ONE
high-priority auxiliary stream per device and overlaps the LLM's kernels on the
remaining CUs.  Results come back through pinned buffers and a *blocking* event, so
the waiting thread sleeps instead of spinning a core.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Dict, List, Optional

import torch

_lock = threading.Lock()
_aux: Dict[int, "torch.cuda.Stream"] = {}
_search: Dict[int, "torch.cuda.Stream"] = {}


def _hp_stream(table, device) -> Optional["torch.cuda.Stream"]:
    device = torch.device(device)
    if device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    with _lock:
        s = table.get(idx)
        if s is None:
            lo, hi = torch.cuda.Stream.priority_range()
            s = torch.cuda.Stream(device=idx, priority=min(lo, hi))
            # everything enqueued on the device so far (weights, setup) happens-before
            s.wait_stream(torch.cuda.current_stream(idx))
            table[idx] = s
    return s


def aux_stream(device) -> Optional["torch.cuda.Stream"]:
    """Embeddings and vector-store writes."""
    return _hp_stream(_aux, device)


def search_stream(device) -> Optional["torch.cuda.Stream"]:
    """Vector-store searches: their own high-priority stream, so a query's kNN never
    queues behind a large ingest embedding batch on the auxiliary stream (searches wait
    only for the store's last write, VectorStore._write_ev)."""
    return _hp_stream(_search, device)


@contextlib.contextmanager
def on_aux(device):
    s = aux_stream(device)
    if s is None:
        yield None
        return
    with torch.cuda.stream(s):
        yield s


@contextlib.contextmanager
def on_search(device):
    s = search_stream(device)
    if s is None:
        yield None
        return
    with torch.cuda.stream(s):
        yield s


def to_host_async(*tensors: torch.Tensor):
    """(pinned host copies, event): the D2H copies enqueued on the current stream; the
    caller synchronises the event before reading the copies (possibly after releasing a
    lock).  CPU tensors pass through with event None."""
    if not tensors or not tensors[0].is_cuda:
        return list(tensors), None
    outs = []
    for t in tensors:
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        outs.append(h)
    ev = torch.cuda.Event(blocking=True)
    ev.record()
    return outs, ev


def to_host(*tensors: torch.Tensor) -> List[torch.Tensor]:
    """D2H copies of the given device tensors (enqueued on the current stream) into
    pinned buffers; waits with a blocking event.  CPU tensors pass through."""
    if not tensors or not tensors[0].is_cuda:
        return list(tensors)
    outs = []
    for t in tensors:
        h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
        h.copy_(t, non_blocking=True)
        outs.append(h)
    ev = torch.cuda.Event(blocking=True)
    ev.record()
    ev.synchronize()
    return outs
