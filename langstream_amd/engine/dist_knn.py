"""Global top-k over the vector-store shards of all data-parallel replicas (SURVEY
§2.10 C-DP).

With one process per GPU every replica of the ingest pipeline writes the chunks it
consumed into ITS OWN HBM store, so each store holds a shard of the corpus.  A
``query-vector-db`` lookup must still see the whole corpus, as it does against the
reference's shared database (VEC/QueryVectorDBAgent.java:27-93 over one datasource).

``ShardedKnn`` runs a background thread on every rank that executes lock-step search
rounds (every rank takes part in every round, so collectives always match):

1. all-gather of a small JSON header (gloo, CPU): each rank's pending requests
   ``(collection, n_queries, k, include_vector, dim)`` and its stop flag; an empty round
   sleeps ``tick`` and repeats;
2. per collection: all-gather of the query vectors ``[W*Qmax, d]`` over the data group
   (RCCL over xGMI on the GPU), the fused MFMA kNN kernel of the LOCAL shard on every
   rank for all ``W*Qmax`` queries, then one all-to-all of ``(score, row)`` candidates
   ``[W, Qmax, k]`` back to the ranks that asked;
3. merge on the device: top-k of the ``W*k`` candidates per query -> ``(owner, row)``;
4. two-phase payload fetch over gloo: each rank asks every owner only for the rows in
   its merged top-k (``k/W`` per query on average) and the owners answer with the
   metadata (and vectors when ``include-vector``) -- bandwidth-optimal for the text
   payloads that stay on the host.

Store locks are held on each rank from its local search to its payload answer, so row
indices cannot be moved by a concurrent delete in between.
"""
from __future__ import annotations

import json
import logging
import os
import threading
import time
from concurrent.futures import Future
from typing import Any, Dict, List, Optional

import msgpack
import numpy as np
import torch
import torch.distributed as dist

from ..utils.gpu import on_search, to_host
from .vector_store import VectorStoreRegistry

log = logging.getLogger(__name__)

_service: Optional["ShardedKnn"] = None


def active() -> Optional["ShardedKnn"]:
    return _service


def start(device=None, tick_s: float = 0.001) -> "ShardedKnn":
    """Start the process-wide service (collective: every rank of the default group)."""
    global _service
    if _service is None:
        _service = ShardedKnn(device=device, tick_s=tick_s)
    return _service


def stop() -> None:
    global _service
    s, _service = _service, None
    if s is not None:
        s.close()


class _Req:
    __slots__ = ("coll", "q", "k", "inc", "fut")

    def __init__(self, coll, q, k, inc):
        self.coll, self.q, self.k, self.inc = coll, q, k, inc
        self.fut: Future = Future()


class ShardedKnn:
    def __init__(self, device=None, tick_s: float = 0.001, max_queries_per_round: int = 4096):
        if not dist.is_initialized():
            raise RuntimeError("ShardedKnn needs an initialised default process group")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        backend = dist.get_backend()
        self.device = torch.device(device or ("cuda" if backend == "nccl" else "cpu"))
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        # separate groups so the service never interleaves with the caller's collectives
        self.meta = dist.new_group(backend="gloo")
        # LS_KNN_DATA=gloo|nccl: which group carries a round's queries and partial results.
        # They are KB-sized and latency-bound: on host (gloo) they never queue behind the
        # LLM's decode graphs on a shared hardware queue; measured in profiles/.
        data_backend = os.environ.get("LS_KNN_DATA", "gloo") if backend == "nccl" else "gloo"
        if data_backend == "nccl":
            # high-priority RCCL streams: a round's collectives must not queue behind the
            # LLM engine's decode graphs on a shared hardware queue
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = os.environ.get("LS_KNN_HIPRI", "1") != "0"
            self.data = dist.new_group(backend="nccl", pg_options=opts)
        else:
            self.data = dist.new_group(backend="gloo")
        self.data_dev = self.device if data_backend == "nccl" else torch.device("cpu")
        self.tick_s = tick_s
        self.max_idle_s = max(tick_s, 0.004)
        self.max_q = max_queries_per_round
        self._pending: List[_Req] = []
        self._cv = threading.Condition()
        self._stop = False
        self.rounds = 0
        self.stats = {"rounds": 0, "queries": 0, "search_s": 0.0, "payload_s": 0.0, "round_s": 0.0,
                      "header_s": 0.0}
        # LS_KNN_PROFILE=1: synchronise after each phase of a round's search (diagnosis only)
        self._prof = os.environ.get("LS_KNN_PROFILE") == "1" and self.device.type == "cuda"
        self._replicate = max(1, int(os.environ.get("LS_KNN_REPLICATE", "1") or 1))
        if self._prof:
            self.stats.update(upload_s=0.0, gather_s=0.0, topk_s=0.0, a2a_s=0.0)
        self._thread = threading.Thread(target=self._loop, name="sharded-knn", daemon=True)
        self._thread.start()

    # ------------------------------------------------------------------ client API
    def search(self, collection: str, queries, k: int, with_vectors: bool = False) -> Future:
        """Global top-k for the rows of ``queries`` ([Q, d]) -> Future[List[List[dict]]]
        in the local store's result format (id, similarity, metadata[, vector])."""
        q = np.array(queries.cpu() if isinstance(queries, torch.Tensor) else queries, dtype=np.float32, ndmin=2)
        q = q / np.maximum(np.linalg.norm(q, axis=-1, keepdims=True), 1e-12)
        r = _Req(collection, q, int(k), bool(with_vectors))
        if r.k < 1:
            r.fut.set_exception(ValueError("top-k must be >= 1"))
            return r.fut
        with self._cv:
            if self._stop:
                r.fut.set_exception(RuntimeError("sharded kNN service stopped"))
                return r.fut
            self._pending.append(r)
            self._cv.notify()
        return r.fut

    def close(self, timeout: float = 30.0) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout)

    # ------------------------------------------------------------------ collectives
    _SLOT = 2048   # round headers fit in one fixed-size all-gather slot almost always

    # Host-side buffers are numpy arrays handed to the collectives through
    # torch.from_numpy: a torch op releases and re-takes the GIL, and on a rank whose agents
    # keep the GIL busy every re-take waits up to the switch interval while the other
    # ranks wait in the next collective (tests/test_distributed_cpu.py slow-rank test).
    def _allgather_bytes(self, b: bytes) -> List[bytes]:
        """All-gather of variable-length byte strings over the gloo group: ONE collective
        with a fixed 2 KiB slot per rank (4-byte length + payload); only when some rank's
        payload is longer do all ranks (who all see every length) run a second round."""
        slot = np.zeros(self._SLOT, dtype=np.uint8)
        n = len(b)
        slot[:4] = np.array([n], dtype=np.int32).view(np.uint8)
        if 0 < n <= self._SLOT - 4:
            slot[4: 4 + n] = np.frombuffer(b, dtype=np.uint8)
        o = np.empty(self.world * self._SLOT, dtype=np.uint8)
        dist.all_gather_into_tensor(torch.from_numpy(o), torch.from_numpy(slot), group=self.meta)
        lens = o.reshape(self.world, self._SLOT)[:, :4].copy().view(np.int32)[:, 0].tolist()
        if max(lens) <= self._SLOT - 4:
            return [o[i * self._SLOT + 4: i * self._SLOT + 4 + lens[i]].tobytes() for i in range(self.world)]
        m = max(lens)
        buf = np.zeros(m, dtype=np.uint8)
        if b:
            buf[:n] = np.frombuffer(b, dtype=np.uint8)
        o = np.empty(self.world * m, dtype=np.uint8)
        dist.all_gather_into_tensor(torch.from_numpy(o), torch.from_numpy(buf), group=self.meta)
        return [o[i * m: i * m + lens[i]].tobytes() for i in range(self.world)]

    def _alltoall_bytes(self, per_dest: List[bytes]) -> List[bytes]:
        send_n = np.array([len(b) for b in per_dest], dtype=np.int64)
        recv_n = np.empty(self.world, dtype=np.int64)
        dist.all_to_all_single(torch.from_numpy(recv_n), torch.from_numpy(send_n), group=self.meta)
        flat = b"".join(per_dest)
        send = np.frombuffer(flat, dtype=np.uint8).copy() if flat else np.zeros(0, dtype=np.uint8)
        o = np.empty(int(recv_n.sum()), dtype=np.uint8)
        dist.all_to_all_single(torch.from_numpy(o), torch.from_numpy(send), recv_n.tolist(), send_n.tolist(),
                               group=self.meta)
        out, p = [], 0
        for n in recv_n.tolist():
            out.append(o[p: p + n].tobytes())
            p += n
        return out

    # ------------------------------------------------------------------ service loop
    def _loop(self) -> None:
        import sys
        # A round hands the GIL back and forth ~10 times (each gloo collective releases
        # it); on a rank whose agents are busy in Python every hand-off waits up to the
        # switch interval, and the OTHER ranks wait in the collective for it.  1 ms (the
        # LLM engine's setting) bounds a slow rank's cost to the rest of the world.
        sys.setswitchinterval(min(sys.getswitchinterval(), 0.001))
        try:
            if self.device.type == "cuda":
                torch.cuda.set_device(self.device.index if self.device.index is not None
                                      else torch.cuda.current_device())
                # Every device op of a round -- the H2D query copy, the kNN kernel and the
                # D2H copies (plus the RCCL collectives under LS_KNN_DATA=nccl, which order
                # themselves after the CURRENT stream) -- runs on the one high-priority search
                # stream: they queue neither behind the LLM engine's steps nor behind ingest
                # embedding batches, and the store's writes share the stream.
                with on_search(self.device):
                    self._serve()
            else:
                self._serve()
        except BaseException as e:  # noqa: BLE001  (setup failed: fail what is pending)
            log.exception("sharded kNN service failed")
            with self._cv:
                self._stop = True
                pend, self._pending = self._pending, []
            for r in pend:
                if not r.fut.done():
                    r.fut.set_exception(e if isinstance(e, Exception) else RuntimeError(str(e)))

    def _serve(self) -> None:
        idle = 0
        try:
            while True:
                with self._cv:
                    take, n = [], 0
                    while self._pending and (not take or n + self._pending[0].q.shape[0] <= self.max_q):
                        r = self._pending.pop(0)
                        take.append(r)
                        n += r.q.shape[0]
                    stopping = self._stop and not take and not self._pending
                hdr = {"s": stopping, "r": [[r.coll, int(r.q.shape[0]), r.k, r.inc, int(r.q.shape[1])] for r in take]}
                t_h = time.perf_counter()
                hdrs = [json.loads(b) for b in self._allgather_bytes(json.dumps(hdr).encode())]
                dt_h = time.perf_counter() - t_h
                if all(h["s"] for h in hdrs):
                    return
                if not any(h["r"] for h in hdrs):
                    self.stats["idle_header_s"] = self.stats.get("idle_header_s", 0.0) + dt_h
                    # idle: back off (tick, 2 tick, ... up to max_idle_s) so an idle service
                    # does not run a collective every millisecond next to the engines; a
                    # local request wakes this rank at once, remote ones within the backoff
                    idle = min(idle + 1, 16)
                    with self._cv:
                        if not self._pending:
                            self._cv.wait(min(self.max_idle_s, self.tick_s * (1 << min(idle, 10))))
                    continue
                idle = 0
                self.stats["header_s"] += dt_h   # rounds with work only (idle polls: idle_header_s)
                self.rounds += 1
                self.stats["rounds"] += 1
                self.stats["queries"] += sum(int(r.q.shape[0]) for r in take)
                t_r = time.perf_counter()
                try:
                    self._round(take, hdrs)
                    self.stats["round_s"] += time.perf_counter() - t_r
                except Exception as e:  # noqa: BLE001  (a local failure after the collectives)
                    log.exception("sharded kNN round failed")
                    for r in take:
                        if not r.fut.done():
                            r.fut.set_exception(e)
        except Exception as e:  # noqa: BLE001  (a collective failed: the service is dead)
            log.exception("sharded kNN service stopped")
            with self._cv:
                self._stop = True
                pend, self._pending = self._pending, []
            for r in pend:
                r.fut.set_exception(e)

    def _phase(self, key: str, t0: float) -> float:
        """LS_KNN_PROFILE: charge the time since ``t0`` (after a device sync) to ``key``;
        the remainder of the search keeps accruing to search_s."""
        if not self._prof:
            return t0
        torch.cuda.current_stream().synchronize()   # the search stream, not the LLM's
        t = time.perf_counter()
        self.stats[key] += t - t0
        self.stats["search_s"] += t - t0
        return t

    def _round(self, take: List[_Req], hdrs: List[Dict[str, Any]]) -> None:
        W, me = self.world, self.rank
        colls = sorted({r[0] for h in hdrs for r in h["r"]})
        stores = {c: VectorStoreRegistry.get(c) for c in colls if VectorStoreRegistry.exists(c)}
        locks = [stores[c].lock for c in sorted(stores)]
        for lk in locks:
            lk.acquire()
        # Every rank must run the SAME collective sequence in a round (the headers decide
        # it, and every rank sees the same headers).  A local failure (OOM in the kNN, a
        # store error, a bad payload) is therefore recorded here and substituted with an
        # empty contribution; the round's collectives all still run, and the requests it
        # touched fail afterwards with the recorded error.
        errs: Dict[str, BaseException] = {}       # collection -> local failure
        try:
            hits: Dict[int, List[List[tuple]]] = {}   # id(req) -> per query [(score, owner, row)]
            need: List[Dict[str, set]] = [dict() for _ in range(W)]
            vec_colls = set()
            for coll in colls:
                reqs_all = [(h_i, r) for h_i, h in enumerate(hdrs) for r in h["r"] if r[0] == coll]
                dims = {r[4] for _, r in reqs_all}
                mine = [r for r in take if r.coll == coll]
                if len(dims) != 1:   # every rank sees the same headers -> all skip consistently
                    for r in mine:
                        r.fut.set_exception(ValueError(f"collection {coll}: queries of different dims {dims}"))
                    continue
                dim = dims.pop()
                counts = [sum(r[1] for hi, r in reqs_all if hi == i) for i in range(W)]
                kmax = max(r[2] for _, r in reqs_all)
                if any(r[3] for _, r in reqs_all):
                    vec_colls.add(coll)
                qmax = max(counts)
                t_s = time.perf_counter()
                host = self.data_dev.type == "cpu"
                if host:
                    qloc_np = np.zeros((qmax, dim), dtype=np.float32)
                    if mine:
                        qloc_np[: counts[me]] = np.concatenate([r.q for r in mine])
                    qall_np = np.empty((W * qmax, dim), dtype=np.float32)
                    dist.all_gather_into_tensor(torch.from_numpy(qall_np), torch.from_numpy(qloc_np), group=self.data)
                    qall = torch.from_numpy(qall_np)
                else:
                    qloc = torch.zeros(qmax, dim, dtype=torch.float32, pin_memory=True)
                    if mine:
                        qloc[: counts[me]] = torch.from_numpy(np.concatenate([r.q for r in mine]))
                    qloc = qloc.to(self.data_dev, non_blocking=True)   # pinned: async, no staging copy
                    t_s = self._phase("upload_s", t_s)
                    qall = torch.empty(W * qmax, dim, dtype=torch.float32, device=self.data_dev)
                    dist.all_gather_into_tensor(qall, qloc, group=self.data)
                t_s = self._phase("gather_s", t_s)
                store = stores.get(coll)
                s = idx = None
                if store is not None and store.dim == dim and len(store):
                    try:
                        # LS_KNN_REPLICATE=R (diagnosis): search the gathered queries R times
                        # over, i.e. the per-round load of R x W ranks, and keep the first copy
                        qs = qall if self._replicate <= 1 else qall.repeat(self._replicate, 1)
                        if store.device.type == "cuda" and self.data_dev.type == "cpu":
                            s, idx = to_host(*store.topk_rows(qs.pin_memory().to(
                                store.device, non_blocking=True).to(store.dtype), kmax))
                        else:
                            s, idx = store.topk_rows(qs.to(store.device, store.dtype), kmax)
                            s, idx = s.to(self.data_dev), idx.to(self.data_dev)
                        s, idx = s[: W * qmax], idx[: W * qmax]
                    except Exception as e:  # noqa: BLE001 - contribute nothing, keep the collectives
                        log.exception("sharded kNN: local search of %s failed", coll)
                        errs[coll] = e
                        s = idx = None
                if host:
                    # [W*qmax, k, 2] float32 pairs (score, row bits), exchanged in numpy
                    send_np = np.empty((W * qmax, kmax, 2), dtype=np.float32)
                    if s is None:
                        send_np[..., 0] = -np.inf
                        send_np[..., 1] = np.array([-1], dtype=np.int32).view(np.float32)[0]
                    else:
                        s_np = s.float().numpy() if isinstance(s, torch.Tensor) else np.asarray(s, np.float32)
                        i_np = idx.int().numpy() if isinstance(idx, torch.Tensor) else np.asarray(idx, np.int32)
                        send_np[..., 0] = s_np
                        send_np[..., 1] = i_np.view(np.float32)
                    t_s = self._phase("topk_s", t_s)
                    recv_np = np.empty_like(send_np)
                    dist.all_to_all_single(torch.from_numpy(recv_np), torch.from_numpy(send_np), group=self.data)
                else:
                    if s is None:
                        s = torch.full((W * qmax, kmax), float("-inf"), device=self.data_dev)
                        idx = torch.full((W * qmax, kmax), -1, dtype=torch.int32, device=self.data_dev)
                    send = torch.stack([s.float(), idx.int().view(torch.float32)], -1).contiguous()  # [W*qmax,k,2]
                    t_s = self._phase("topk_s", t_s)
                    recv = torch.empty_like(send)
                    dist.all_to_all_single(recv, send, group=self.data)
                    recv_np = recv.cpu().numpy()
                t_s = self._phase("a2a_s", t_s)
                n_me = counts[me]
                if n_me == 0:
                    continue
                try:
                    # merge the W shards' candidates of this rank's queries on the host
                    rv = recv_np.reshape(W, qmax, kmax, 2)[:, :n_me]            # [W, n_me, k, 2]
                    cs = rv[..., 0].transpose(1, 0, 2).reshape(n_me, W * kmax)
                    ci = np.ascontiguousarray(rv[..., 1]).view(np.int32).transpose(1, 0, 2).reshape(n_me, W * kmax)
                    sel = np.argsort(-cs, axis=1, kind="stable")[:, :kmax]
                    top_s = np.take_along_axis(cs, sel, 1).tolist()
                    rows = np.take_along_axis(ci, sel, 1).tolist()
                    owners = (sel // kmax).tolist()
                except Exception as e:  # noqa: BLE001 - local merge only, no collective inside
                    log.exception("sharded kNN: merge of %s failed", coll)
                    errs.setdefault(coll, e)
                    continue
                self.stats["search_s"] += time.perf_counter() - t_s
                qi = 0
                for r in mine:
                    per_q = []
                    for j in range(qi, qi + r.q.shape[0]):
                        lst = [(sc, o, rw) for sc, o, rw in zip(top_s[j][: r.k], owners[j][: r.k], rows[j][: r.k])
                               if rw >= 0 and sc != float("-inf")]
                        for _, o, rw in lst:
                            need[o].setdefault(coll, set()).add(rw)
                        per_q.append(lst)
                    hits[id(r)] = per_q
                    qi += r.q.shape[0]
            # phase 2: payloads of the merged top-k rows, asked from their owners; the rows
            # this rank owns are served directly (no serialisation, no exchange)
            t_p = time.perf_counter()

            def serve(asked, as_bytes=True):
                # vectors: one gathered float32 block per collection; remote askers get each
                # row's bytes, this rank's own results keep the numpy row (no round trip)
                ans = {}
                for coll, rws in asked.items():
                    st = stores.get(coll)
                    if st is None:
                        continue
                    try:
                        rws = [rw for rw in sorted(rws) if 0 <= rw < len(st)]
                        vecs = {}
                        if coll in vec_colls and rws:
                            flat, arr = st.row_vectors_array(rws)
                            vecs = {rw: (arr[i].tobytes() if as_bytes else arr[i]) for i, rw in enumerate(flat)}
                        ans[coll] = {rw: (st.row_payload(rw), vecs.get(rw)) for rw in rws}
                    except Exception as e:  # noqa: BLE001 - tell the asker instead of skipping the exchange
                        log.exception("sharded kNN: payloads of %s failed", coll)
                        ans.setdefault("__errors__", {})[coll] = f"{type(e).__name__}: {e}"
                return ans

            local = serve(need[me], as_bytes=False)
            asks = [b"" if d == me else msgpack.packb({c: sorted(v) for c, v in need[d].items()}) for d in range(W)]
            got_asks = [msgpack.unpackb(b, strict_map_key=False) if b else {} for b in self._alltoall_bytes(asks)]
            answers = [b"" if src == me else msgpack.packb(serve(got_asks[src]), use_bin_type=True)
                       for src in range(W)]
        finally:
            for lk in reversed(locks):
                lk.release()
        payload = [msgpack.unpackb(b, raw=False, strict_map_key=False) if b else {}
                   for b in self._alltoall_bytes(answers)]
        payload[me] = local
        for src, ans in enumerate(payload):
            for coll, msg in (ans.get("__errors__") or {}).items():
                errs.setdefault(coll, RuntimeError(f"kNN shard {src} could not serve {coll}: {msg}"))
        self.stats["payload_s"] += time.perf_counter() - t_p
        for r in take:
            if r.fut.done():
                continue
            if r.coll in errs:
                r.fut.set_exception(errs[r.coll])
                continue
            out = []
            for lst in hits.get(id(r), [[] for _ in range(r.q.shape[0])]):
                res = []
                for sc, o, rw in lst:
                    p = payload[o].get(r.coll, {}).get(rw)
                    if p is None:
                        continue
                    d = dict(p[0])
                    d["similarity"] = sc
                    if r.inc and p[1] is not None:
                        v = p[1]
                        d["vector"] = (v if isinstance(v, np.ndarray) else np.frombuffer(v, np.float32)).tolist()
                    res.append(d)
                out.append(res)
            r.fut.set_result(out)
