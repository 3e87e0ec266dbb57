"""Collective self-check before a multi-GPU job serves or measures anything.

A first 8-GPU run whose all-reduce hangs or returns garbage would otherwise show up as a
timeout or as NaN logits deep inside serving.  ``check_collectives`` runs, on the job's
process group, the collectives the job will use and compares each result with the sum
computed on the host from the known per-rank inputs:

* ``eager``: one all-reduce (and one all-gather) issued directly -- RCCL over xGMI on
  GPUs, gloo on CPU;
* ``graph``: the same all-reduce captured into a HIP graph and replayed (the default TP
  decode path: c10d all-reduces inside the runner's captured decode graphs,
  ``ops/csrc/runner.hip``);
* ``oneshot``: the one-shot IPC all-reduce of ``ops/csrc/allreduce.hip`` when
  ``LS_ONESHOT_AR=1`` enables it for serving.

A wrong eager (or one-shot) result raises ``CollectiveCheckError`` with the phase and
the first mismatching element -- the caller exits non-zero with that message.  A graph
capture that fails or replays a wrong sum only disables graphs: the result says so and
the engine falls back to eager RCCL steps.  A rank that never arrives is caught by the
``RankWatchdog`` (bounded time, names the missing rank and the phase).

Inputs are small integers times (rank + 1), exact in bf16 and f32, so the expected sums
are exact.  Fault injection for the CPU tests: ``LS_BRINGUP_FAULT=wrong-sum@<rank>`` (that
rank adds 1 to its contribution) or ``stall@<rank>`` (that rank sleeps before the first
collective).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

log = logging.getLogger(__name__)

N_ELEMS = 4096 + 7      # a ragged tail past the 8-element vectors


class CollectiveCheckError(RuntimeError):
    pass


def _fault(rank: int) -> Optional[str]:
    f = os.environ.get("LS_BRINGUP_FAULT", "")
    if "@" not in f:
        return None
    kind, _, r = f.partition("@")
    return kind if r.strip().isdigit() and int(r) == rank else None


def _inputs(rank: int, world: int, device, dtype):
    base = (torch.arange(N_ELEMS, dtype=torch.float32) % 4) + 1          # 1..4
    mine = base * (rank + 1)
    want = base * (world * (world + 1) // 2)                               # <= 4 * 36 = 144: exact in bf16
    return mine.to(device=device, dtype=dtype), want


def _compare(phase: str, got: torch.Tensor, want: torch.Tensor) -> None:
    g = got.detach().float().cpu()
    bad = (g != want).nonzero()
    if bad.numel():
        i = int(bad[0, 0])
        raise CollectiveCheckError(f"collective self-check failed in phase '{phase}': element {i} = "
                                   f"{float(g[i])}, expected {float(want[i])} ({bad.numel()} of {g.numel()} wrong)")


def check_collectives(group=None, device: Optional[str] = None, graphs: bool = True, oneshot: Optional[bool] = None,
                      dtype: Optional[torch.dtype] = None, watchdog=None, limit_s: float = 120.0) -> Dict[str, bool]:
    """Run the self-check on ``group`` (default: the default group).  Returns
    {"eager": True, "graph": bool, "oneshot": bool or None}; raises CollectiveCheckError
    on a wrong eager / one-shot result."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if device is None:
        device = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() and \
            dist.get_backend(group) == "nccl" else "cpu"
    on_gpu = str(device).startswith("cuda")
    dtype = dtype or (torch.bfloat16 if on_gpu else torch.float32)
    res: Dict[str, Optional[bool]] = {"eager": False, "graph": False, "oneshot": None}
    fault = _fault(rank)

    def phase(name):
        if watchdog is not None:
            watchdog.phase(f"bringup:{name}", limit_s)

    def arrive(what):
        if watchdog is not None:
            watchdog.arrive(what)

    if fault == "stall":
        phase("eager-allreduce")
        time.sleep(10 * limit_s)
    # ---- eager all-reduce + all-gather
    phase("eager-allreduce")
    x, want = _inputs(rank, world, device, dtype)
    if fault == "wrong-sum":
        x = x + 1
    arrive("all_reduce")
    dist.all_reduce(x, group=group)
    _compare("eager all-reduce", x, want)
    phase("eager-allgather")
    mine = torch.full((8,), float(rank + 1), device=device, dtype=dtype)
    parts = [torch.empty_like(mine) for _ in range(world)]
    arrive("all_gather")
    dist.all_gather(parts, mine, group=group)
    _compare("eager all-gather", torch.stack(parts), torch.arange(1, world + 1, dtype=torch.float32)[:, None]
             .expand(world, 8))
    res["eager"] = True
    # ---- graph-captured all-reduce (GPU only)
    if graphs and on_gpu:
        phase("graph-allreduce")

        def agree(ok: bool) -> bool:
            # every rank must agree before the next step: a replay while a peer gave up
            # on its capture would wait for it forever
            flag = torch.tensor([1 if ok else 0], device=device, dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
            return bool(flag.item())

        y, want_g = _inputs(rank, world, device, dtype)
        src = y.clone()
        g = None
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                dist.all_reduce(y, group=group)          # warm the communicator on this stream
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                dist.all_reduce(y, group=group)
        except Exception as e:  # noqa: BLE001
            log.warning("capturing an all-reduce into a graph failed (%s)", e)
            g = None
        ok = False
        if agree(g is not None):
            y.copy_(src)
            g.replay()
            torch.cuda.synchronize()
            try:
                _compare("graph all-reduce", y, want_g)
                ok = True
            except CollectiveCheckError as e:
                log.warning("%s", e)
        res["graph"] = agree(ok)
        if not res["graph"]:
            log.warning("graph-captured all-reduce failed the self-check: serving with eager steps")
    # ---- one-shot IPC all-reduce
    if oneshot is None:
        oneshot = os.environ.get("LS_ONESHOT_AR", "0") not in ("", "0")
    if oneshot and on_gpu:
        phase("oneshot-allreduce")
        from .. import ops
        z, want_o = _inputs(rank, world, device, torch.bfloat16)
        if fault == "wrong-sum":
            z = z + 1
        err = ops.hip().oneshot_allreduce_selftest(group or dist.group.WORLD, z)
        if err:
            raise CollectiveCheckError("collective self-check failed in phase 'one-shot all-reduce': a peer "
                                       "never arrived (the spin wait timed out)")
        _compare("one-shot all-reduce", z, want_o)
        res["oneshot"] = True
    phase("bringup-done")
    return res
