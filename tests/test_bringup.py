"""Multi-rank bring-up that cannot hang or silently corrupt (VERDICT r5 'next round' 4):
the collective self-check (parallel/bringup.py) and the per-rank watchdog
(parallel/watchdog.py), on gloo with world size 2 -- a correct group passes, an injected
wrong sum ends every rank non-zero with the failing phase, an injected stalled rank ends
every rank with exit 3 within the watchdog limit, naming the stalled rank and phase; and
bench.py --gpus 2 stops before timing anything when its self-check fails."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

RANK_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import torch.distributed as dist
from langstream_amd.parallel.bringup import CollectiveCheckError, check_collectives
from langstream_amd.parallel.watchdog import RankWatchdog
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
wd = RankWatchdog(rank, world, poll_s=0.2).start()
try:
    res = check_collectives(watchdog=wd, limit_s=float(os.environ.get("LIMIT", "30")))
except CollectiveCheckError as e:
    print(json.dumps({"rank": rank, "error": str(e)}), flush=True)
    os._exit(2)
print(json.dumps({"rank": rank, "result": res}), flush=True)
wd.stop()
dist.destroy_process_group()
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ranks(world=2, timeout=120, **env):
    port = _port()
    procs = []
    for r in range(world):
        e = dict(os.environ, REPO=REPO, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r),
                 WORLD_SIZE=str(world), LOCAL_RANK=str(r), **{k: str(v) for k, v in env.items()})
        procs.append(subprocess.Popen([sys.executable, "-c", RANK_SCRIPT], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    out = []
    t0 = time.time()
    for p in procs:
        try:
            so, se = p.communicate(timeout=max(1, timeout - (time.time() - t0)))
        except subprocess.TimeoutExpired:
            p.kill()
            so, se = p.communicate()
        out.append((p.returncode, so, se))
    return out, time.time() - t0


def test_selfcheck_passes_on_a_healthy_group():
    res, _ = _ranks()
    for rc, so, se in res:
        assert rc == 0, se[-2000:]
        got = json.loads(so.strip().splitlines()[-1])["result"]
        assert got == {"eager": True, "graph": False, "oneshot": None}   # CPU: no graphs / one-shot


def test_selfcheck_wrong_sum_fails_every_rank_with_the_phase():
    res, _ = _ranks(LS_BRINGUP_FAULT="wrong-sum@1")
    for rc, so, se in res:
        assert rc == 2, (rc, se[-2000:])
        err = json.loads(so.strip().splitlines()[-1])["error"]
        assert "phase 'eager all-reduce'" in err and "expected" in err


def test_stalled_rank_ends_every_rank_naming_it():
    """rank 1 hangs before its first collective: rank 0 waits in the all-reduce, its
    watchdog fires after LIMIT s; rank 1's own watchdog fires too (it stopped beating)."""
    res, dt = _ranks(LS_BRINGUP_FAULT="stall@1", LIMIT=3, timeout=60)
    assert dt < 45
    for rank, (rc, so, se) in enumerate(res):
        assert rc == 3, (rank, rc, se[-2000:])
        line = next(json.loads(x) for x in se.splitlines() if x.startswith("{") and "rank stalled" in x)
        assert line["rank"] == rank and line["phase"] == "bringup:eager-allreduce"
        assert line["stalled_s"] >= 3
        if rank == 0:
            assert line["suspect_rank"] == 1 and line["suspect_phase"] == "bringup:eager-allreduce"


def test_watchdog_unit_reports_oldest_rank():
    import torch.distributed as dist  # noqa: F401
    from torch.distributed import TCPStore
    from langstream_amd.parallel.watchdog import RankWatchdog
    store = TCPStore("127.0.0.1", 0, 3, True, wait_for_workers=False)
    fired = []
    a = RankWatchdog(0, 3, store=store, poll_s=0.05, exit_fn=fired.append, out=open(os.devnull, "w"))
    b = RankWatchdog(1, 3, store=store, poll_s=10)
    b.phase("timed", 100)
    time.sleep(0.3)
    a.start()
    a.phase("timed", 0.2)
    deadline = time.time() + 5
    while not fired and time.time() < deadline:
        time.sleep(0.05)
    assert fired == [3]
    assert a.fired["suspect_rank"] == 2          # rank 2 never published a beat
    assert a.fired["ranks"][2] is None and a.fired["ranks"][1]["phase"] == "timed"
    a.stop()


def test_bench_multi_rank_stops_on_a_failed_selfcheck(tmp_path):
    """bench.py --gpus 2 (gloo on CPU): the injected wrong sum ends the run non-zero with
    the self-check's message, before setup and timing."""
    env = dict(os.environ, LS_BRINGUP_FAULT="wrong-sum@1", PYTHONPATH=REPO)
    t0 = time.time()
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--corpus", "100", "--batch", "2", "--docs", "0", "--also-stream", "0"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert p.returncode != 0
    assert "collective self-check failed" in p.stderr and "eager all-reduce" in p.stderr
    assert '"metric"' not in p.stdout
    assert time.time() - t0 < 240
