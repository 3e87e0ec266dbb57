"""HBM-resident vector store with brute-force kNN on the GPU.

Rows are L2-normalised bf16 vectors in one device tensor ``[capacity, dim]`` (dense:
deletes move tail rows into the holes, so ``[0, n)`` is always valid and the kNN kernel
never scans dead rows).  Search is the fused MFMA GEMM + top-k kernel
(``ops.knn_topk``), so cosine similarity over 10^6-10^7 rows per GPU is one kernel pass
over HBM.  Metadata (arbitrary JSON-able dicts: text, source, ...) stays on the host.
Capacity doubles on demand; at 384 dims a 288 GB GPU holds >10^8 rows.

Limits are explicit: the kernel covers embedding dims ``KERNEL_DIMS`` and k <= 64; any
other dim or a larger k runs the exact chunked GEMM + ``torch.topk`` path (logged once
when the collection is created) instead of being clamped.

Durability (parity: the reference writers persist to a database before the source
offset is committed, VEC/jdbc/JdbcWriter.java:33-208): with a persistence directory
(``VectorStoreRegistry.configure(persist_dir=...)``, the vector-database resource's
``persist-directory`` or ``$LANGSTREAM_VECTOR_STORE_DIR``) every upsert / delete is
appended to a write-ahead log before it returns -- so before the sink's future
completes and the runner commits the offset -- and the collection is restored from
``snapshot + WAL`` when it is first opened after a restart.  The WAL is compacted into
a new snapshot once it outgrows it.

Used by ``vector-db-sink`` (upsert/delete) and ``query-vector-db`` (search), by the
JDBC-compatible SQL datasource for ``ORDER BY cosine_similarity(...) DESC LIMIT k``, and
by ``engine/dist_knn.py`` for the global top-k over the shards of all DP replicas.
"""
from __future__ import annotations

import json
import logging
import os
import re
import threading
import time
from typing import Any, Dict, List, Optional, Sequence, Tuple

import msgpack
import numpy as np
import torch

from .. import ops
from ..utils.gpu import aux_stream, on_search, to_host, to_host_async

log = logging.getLogger(__name__)

KERNEL_DIMS = (128, 256, 384, 512, 768, 1024, 1536, 2048)
KERNEL_MAX_K = 64


def _safe(name: str) -> str:
    return re.sub(r"[^A-Za-z0-9_.-]", "_", name)[:200]


class _Persistence:
    """Snapshot + write-ahead log of one collection.

    Crash safety:
    * the snapshot is ONE file (``snapshot.lsv``: magic, JSON header with dim / dtype /
      ids / metadata, then the raw vector rows) written to a temp file and swapped in with
      a single ``os.replace`` -- a crash leaves either the old or the new snapshot, never
      a vector file whose row count disagrees with its ids;
    * the WAL is length-prefixed msgpack entries; ``load`` stops at a torn or corrupt
      tail entry and TRUNCATES the log there before anything is appended, so entries
      written after a restart are never parsed across the garbage;
    * replaying WAL entries over a snapshot that already contains them is idempotent
      (upserts by id, deletes of present ids), so a crash between the snapshot swap and
      the WAL reset loses nothing."""

    MAGIC = b"LSVS0001"

    def __init__(self, directory: str, fsync: bool = False):
        self.dir = directory
        self.fsync = fsync
        os.makedirs(directory, exist_ok=True)
        self.wal_path = os.path.join(directory, "wal.log")
        self.snap_path = os.path.join(directory, "snapshot.lsv")
        # pre-r3 layout (two files, swapped separately): read if present, never written
        self.old_meta = os.path.join(directory, "snapshot.json")
        self.old_vec = os.path.join(directory, "snapshot.vec")
        self._wal = None

    def _open_wal(self) -> None:
        if self._wal is None:
            self._wal = open(self.wal_path, "ab")

    def _append(self, entry) -> None:
        self.append_packed(self.pack(entry))

    @staticmethod
    def pack(entry) -> bytes:
        b = msgpack.packb(entry, use_bin_type=True)
        return len(b).to_bytes(4, "little") + b

    def append_packed(self, b: bytes) -> None:
        self._open_wal()
        self._wal.write(b)
        self._wal.flush()
        if self.fsync:
            os.fsync(self._wal.fileno())

    @classmethod
    def pack_upsert(cls, ids, vecs_f32: np.ndarray, metas) -> bytes:
        return cls.pack(("u", list(ids), vecs_f32.astype(np.float32).tobytes(), list(metas)))

    def log_upsert(self, ids, vecs_f32: np.ndarray, metas) -> None:
        self.append_packed(self.pack_upsert(ids, vecs_f32, metas))

    def log_delete(self, ids) -> None:
        self._append(("d", list(ids)))

    def wal_bytes(self) -> int:
        self._open_wal()
        return self._wal.tell()

    @classmethod
    def read_snapshot_header(cls, path: str) -> Optional[Tuple[dict, int]]:
        """(header, byte offset of the vector rows) of a snapshot file, or None."""
        if not os.path.exists(path):
            return None
        with open(path, "rb") as f:
            head = f.read(16)
            if len(head) < 16 or head[:8] != cls.MAGIC:
                raise ValueError(f"{path}: not a vector-store snapshot")
            n = int.from_bytes(head[8:16], "little")
            return json.loads(f.read(n).decode()), 16 + n

    def load(self):
        """-> (dim or None, ids, metas, vectors torch [n, dim] or None, wal entries)."""
        ids, metas, vec, dim = [], [], None, None
        hdr = self.read_snapshot_header(self.snap_path)
        if hdr is not None:
            m, off = hdr
            dim, ids, metas = m["dim"], m["ids"], m["meta"]
            bf = m.get("dtype") == "bfloat16"
            raw = np.fromfile(self.snap_path, dtype=np.int16 if bf else np.float32, offset=off)
            vec = torch.from_numpy(raw[: len(ids) * dim].reshape(len(ids), dim).copy())
            if bf:
                vec = vec.view(torch.bfloat16)
        elif os.path.exists(self.old_meta) and os.path.exists(self.old_vec):
            with open(self.old_meta) as f:
                m = json.load(f)
            dim, ids, metas = m["dim"], m["ids"], m["meta"]
            raw = np.fromfile(self.old_vec, dtype=np.int16 if m.get("dtype") == "bfloat16" else np.float32)
            if raw.size != len(ids) * dim:
                raise ValueError(f"{self.dir}: legacy snapshot.vec holds {raw.size} values for {len(ids)} ids")
            vec = torch.from_numpy(raw.reshape(len(ids), dim).copy())
            if m.get("dtype") == "bfloat16":
                vec = vec.view(torch.bfloat16)
        entries = []
        data = b""
        if os.path.exists(self.wal_path):
            with open(self.wal_path, "rb") as f:
                data = f.read()
        i = 0
        while i + 4 <= len(data):
            n = int.from_bytes(data[i:i + 4], "little")
            if i + 4 + n > len(data):
                break  # torn tail write: everything before it was acknowledged
            try:
                entries.append(msgpack.unpackb(data[i + 4:i + 4 + n], raw=False, strict_map_key=False))
            except Exception:  # noqa: BLE001 - a corrupt entry ends the valid log like a torn one
                break
            i += 4 + n
        if i != len(data):
            log.warning("vector store %s: dropping %d bytes of torn WAL tail", self.dir, len(data) - i)
            if self._wal is not None:
                self._wal.close()
                self._wal = None
            with open(self.wal_path, "r+b") as f:
                f.truncate(i)
                f.flush()
                os.fsync(f.fileno())
        return dim, ids, metas, vec, entries

    def snapshot(self, dim: int, ids, metas, vec: torch.Tensor) -> None:
        tmp = self.snap_path + ".tmp"
        bf16 = vec.dtype == torch.bfloat16
        hdr = json.dumps({"dim": dim, "dtype": "bfloat16" if bf16 else "float32", "ids": list(ids),
                          "meta": list(metas)}).encode()
        with open(tmp, "wb") as f:
            f.write(self.MAGIC + len(hdr).to_bytes(8, "little") + hdr)
            (vec.view(torch.int16) if bf16 else vec.float()).numpy().tofile(f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, self.snap_path)      # the single atomic swap
        for old in (self.old_meta, self.old_vec):
            if os.path.exists(old):
                os.remove(old)
        try:
            dfd = os.open(self.dir, os.O_RDONLY)
            try:
                os.fsync(dfd)
            finally:
                os.close(dfd)
        except OSError:
            pass
        if self._wal is not None:
            self._wal.close()
        self._wal = open(self.wal_path, "wb")

    def close(self) -> None:
        if self._wal is not None:
            self._wal.close()
            self._wal = None


# Optional search tracer (benchmarks): when a list, every search appends (enter, lock
# taken, top-k on the host, results built, number of queries) as time.time() stamps.
SEARCH_TRACE: Optional[list] = None
SEARCH_RETRIES = 3   # lock-free top-k attempts a renumbering delete may invalidate before one under the lock


class VectorStore:
    def __init__(self, dim: int, device="cuda", capacity: int = 1024, dtype=torch.bfloat16, name: str = "default",
                 persist_dir: Optional[str] = None, fsync: bool = False):
        self.dim = dim
        self.name = name
        self.device = torch.device(device)
        self.dtype = dtype
        self.kernel_dim = dim in KERNEL_DIMS
        if not self.kernel_dim:
            log.warning("vector collection %s: dim %d has no kNN kernel instantiation %s; searches use the exact "
                        "GEMM + torch.topk path", name, dim, KERNEL_DIMS)
        with on_search(self.device):  # every GPU op of the store runs on the search stream
            self._vecs = torch.zeros(max(16, capacity), dim, device=self.device, dtype=dtype)
        self._n = 0
        self._ids: List[Any] = []
        self._meta: List[Dict[str, Any]] = []
        self._row: Dict[Any, int] = {}
        self.lock = threading.RLock()
        self._write_ev = None   # recorded on the store stream after every device write
        self._gen = 0           # bumped when deletes renumber rows (search re-resolves)
        self.search_retries = 0
        self._persist = _Persistence(persist_dir, fsync) if persist_dir else None
        if self._persist is not None:
            with on_search(self.device), self.lock:
                self._restore()
                self._mark_written()

    def __len__(self) -> int:
        return self._n

    @property
    def persistent(self) -> bool:
        return self._persist is not None

    def attach_persistence(self, persist_dir: str, fsync: bool = False) -> bool:
        """Make a store created without persistence durable: restore what the directory
        holds and WAL-log every later write.  Only an EMPTY store can be attached (its
        in-memory rows would otherwise exist in no WAL); returns False when it is not."""
        with on_search(self.device), self.lock:
            if self._persist is not None:
                return True
            if self._n:
                return False
            self._persist = _Persistence(persist_dir, fsync)
            self._restore()
            self._mark_written()
            return True

    # ------------------------------------------------------------------ mutation
    def _grow(self, need: int) -> None:
        cap = self._vecs.shape[0]
        if need <= cap:
            return
        while cap < need:
            cap *= 2
        nv = torch.zeros(cap, self.dim, device=self.device, dtype=self.dtype)
        nv[: self._n] = self._vecs[: self._n]
        self._vecs = nv

    def _normalize(self, v) -> torch.Tensor:
        t = torch.as_tensor(v, dtype=torch.float32)
        if t.dim() == 1:
            t = t[None]
        if t.shape[-1] != self.dim:
            raise ValueError(f"vector dim {t.shape[-1]} != collection {self.name} dim {self.dim}")
        t = t.to(self.device)
        return torch.nn.functional.normalize(t, dim=-1, eps=1e-12).to(self.dtype)

    def upsert(self, ids: Sequence[Any], vectors, metadata: Optional[Sequence[Dict[str, Any]]] = None) -> None:
        metadata = list(metadata) if metadata is not None else [{} for _ in ids]
        if len(metadata) != len(ids):
            raise ValueError("ids and metadata lengths differ")
        if not (isinstance(vectors, torch.Tensor) and vectors.is_cuda):
            self._upsert_host(ids, vectors, metadata)
            return
        with on_search(self.device), self.lock:
            # device vectors come from the embedding engine's auxiliary stream
            torch.cuda.current_stream().wait_stream(aux_stream(self.device))
            vecs = self._normalize(vectors)
            if vecs.shape[0] != len(ids):
                raise ValueError("ids and vectors lengths differ")
            if self._persist is not None:
                self._persist.log_upsert(ids, to_host(vecs.float())[0].numpy(), metadata)
            self._apply_upsert(ids, vecs, metadata)
            self._mark_written()
            self._maybe_compact()

    def _upsert_host(self, ids, vectors, metadata) -> None:
        """Host vectors (lists from records): normalisation, the store-dtype rounding, the
        WAL entry and the pinned upload are prepared before the store lock is taken, so
        the lock covers only the WAL append and the device scatter -- a search waits for
        a few calls instead of the whole upsert (every torch call is a GIL hand-off, and
        on a busy process each hand-off can wait behind other threads)."""
        host = self._normalize_host(vectors)
        if host.shape[0] != len(ids):
            raise ValueError("ids and vectors lengths differ")
        t = torch.from_numpy(np.ascontiguousarray(host, dtype=np.float32)).to(self.dtype)
        entry = (_Persistence.pack_upsert(ids, t.float().numpy(), metadata)
                 if self._persist is not None else None)
        with on_search(self.device):
            if self.device.type == "cuda":
                t = t.pin_memory().to(self.device, non_blocking=True)
            with self.lock:
                if entry is not None:
                    self._persist.append_packed(entry)
                self._apply_upsert(ids, t, metadata)
                self._mark_written()
                self._maybe_compact()

    def _apply_upsert(self, ids, vecs: torch.Tensor, metadata) -> None:
        new_rows = {i for i in ids if i not in self._row}
        self._grow(self._n + len(new_rows))
        rows = []
        for k, md in zip(ids, metadata):
            r = self._row.get(k)
            if r is None:
                r = self._n
                self._n += 1
                self._row[k] = r
                self._ids.append(k)
                self._meta.append(md)
            else:
                self._meta[r] = md
            rows.append(r)
        # duplicate ids in one batch: the last occurrence wins (index_copy_ order is unspecified)
        last: Dict[int, int] = {}
        for j, r in enumerate(rows):
            last[r] = j
        src = list(last.values())
        dst = torch.tensor(list(last.keys()), device=self.device, dtype=torch.long)
        self._vecs.index_copy_(0, dst, vecs[torch.tensor(src, device=self.device, dtype=torch.long)]
                               if len(src) != len(rows) else vecs)

    def delete(self, ids: Sequence[Any]) -> int:
        with on_search(self.device), self.lock:
            present = [k for k in dict.fromkeys(ids) if k in self._row]
            if not present:
                return 0
            if self._persist is not None:
                self._persist.log_delete(present)
            n = self._apply_delete(present)
            self._mark_written()
            self._maybe_compact()
            return n

    def _apply_delete(self, ids) -> int:
        """Remove rows in one device copy: the surviving tail rows fill the holes."""
        self._gen += 1   # row numbers change: a search between its top-k and its payloads redoes
        dead = {self._row.pop(k) for k in ids}
        m = len(dead)
        keep_n = self._n - m
        holes = sorted(r for r in dead if r < keep_n)
        fillers = [r for r in range(keep_n, self._n) if r not in dead]
        if holes:
            src = torch.tensor(fillers, device=self.device, dtype=torch.long)
            dst = torch.tensor(holes, device=self.device, dtype=torch.long)
            self._vecs.index_copy_(0, dst, self._vecs.index_select(0, src))
            for h, f in zip(holes, fillers):
                self._ids[h] = self._ids[f]
                self._meta[h] = self._meta[f]
                self._row[self._ids[h]] = h
        del self._ids[keep_n:]
        del self._meta[keep_n:]
        self._n = keep_n
        return m

    # ------------------------------------------------------------------ persistence
    def _restore(self) -> None:
        dim, ids, metas, vec, entries = self._persist.load()
        if dim is not None and dim != self.dim:
            raise ValueError(f"persisted collection {self.name} has dim {dim}, opened with {self.dim}")
        if ids:
            self._apply_upsert(ids, vec.to(device=self.device, dtype=self.dtype), metas)
        for e in entries:
            if e[0] == "u":
                vf = np.frombuffer(e[2], dtype=np.float32).reshape(len(e[1]), self.dim).copy()
                self._apply_upsert(e[1], self._normalize(vf), e[3])
            elif e[0] == "d":
                present = [k for k in e[1] if k in self._row]
                if present:
                    self._apply_delete(present)
        if self._n:
            log.info("vector collection %s restored: %d rows (%d WAL entries)", self.name, self._n, len(entries))

    def _mark_written(self) -> None:
        """(caller holding the lock) order later reads on other streams after the device
        writes just enqueued on the store's stream."""
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
            self._write_ev = ev

    def _order_read(self) -> None:
        """(caller holding the lock, on the stream that will read) wait for the last
        write and keep the row buffer alive for this stream."""
        if self.device.type == "cuda":
            if self._write_ev is not None:
                torch.cuda.current_stream().wait_event(self._write_ev)
            self._vecs.record_stream(torch.cuda.current_stream())

    def _maybe_compact(self) -> None:
        p = self._persist
        if p is None or p.wal_bytes() < max(64 << 20, self._n * self.dim * 2):
            return
        self.snapshot()

    def snapshot(self) -> None:
        """Write a snapshot of the collection and truncate the WAL."""
        if self._persist is None:
            return
        with on_search(self.device), self.lock:
            v = to_host(self._vecs[: self._n].contiguous())[0]
            self._persist.snapshot(self.dim, self._ids, self._meta, v)

    def close(self) -> None:
        if self._persist is not None:
            self._persist.close()

    # ------------------------------------------------------------------ lookup
    def get(self, key: Any) -> Optional[Dict[str, Any]]:
        with self.lock:
            r = self._row.get(key)
            return None if r is None else dict(self._meta[r])

    def vector(self, key: Any) -> Optional[List[float]]:
        with self.lock:
            r = self._row.get(key)
            if r is None:
                return None
            with on_search(self.device):
                return to_host(self._vecs[r].float())[0].tolist()

    # ------------------------------------------------------------------ search
    def topk_rows(self, q: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Device top-k over the live rows (caller holds ``lock``; any stream -- the read
        is ordered after the store's last write).  q: normalised [Q, dim] in the store dtype.  Returns (scores f32 [Q,k],
        rows int32 [Q,k]); missing entries are (-inf, -1)."""
        n = self._n
        Qn = q.shape[0]
        if n == 0 or Qn == 0:
            return (torch.full((Qn, k), float("-inf"), device=self.device),
                    torch.full((Qn, k), -1, device=self.device, dtype=torch.int32))
        self._order_read()
        X = self._vecs[:n]
        if self.device.type == "cuda" and self.kernel_dim and k <= KERNEL_MAX_K:
            return ops.knn_topk(X, q.contiguous(), k)
        return _exact_topk(X, q, k)

    def search(self, queries, k: int = 10, with_vectors: bool = False) -> List[List[Dict[str, Any]]]:
        """queries: [Q, dim] (list or tensor).  Returns per query a list of
        {"id", "similarity", **metadata} sorted by decreasing cosine similarity."""
        if k < 1:
            raise ValueError("top-k must be >= 1")
        tr = SEARCH_TRACE
        t_in = time.time() if tr is not None else 0.0
        # host preparation outside the lock: numpy conversion + normalisation, then one
        # pinned H2D copy on the search stream (the sharded service's path, which measured
        # 26 ms per round in the RAG bench where this one took 30-170 ms per batch:
        # profiles/r5/bench_stage_trace_r5j.log vs knn_w8load_r5o.log)
        qn = self._normalize_host(queries)
        # The lock is held while work is ENQUEUED, not while the GPU runs it: the top-k and
        # its D2H copy are enqueued under the lock and waited for outside it; the row
        # numbers are then resolved under the lock again, unless a delete renumbered the
        # rows in between (generation check -> search again).  Writes go to the same
        # search stream, so the device reads are ordered against them either way.
        with on_search(self.device):
            q = self._to_device_query(qn)
            for attempt in range(SEARCH_RETRIES + 1):
                if attempt == SEARCH_RETRIES:
                    # a steady stream of deletes kept renumbering rows: the last attempt
                    # holds the lock from the top-k through the row resolution, so the
                    # search always finishes
                    with self.lock:
                        t_lk = time.time() if tr is not None else 0.0
                        (hs, hi), ev = to_host_async(*self.topk_rows(q, k))
                        if ev is not None:
                            ev.synchronize()
                        s, idx = hs.tolist(), hi.tolist()
                        t_gpu = time.time() if tr is not None else 0.0
                        hits = [[(sc, r, self.row_payload(r)) for sc, r in zip(srow, irow) if 0 <= r < self._n]
                                for srow, irow in zip(s, idx)]
                        pend = (self._gather_rows_async({r for row in hits for _, r, _ in row})
                                if with_vectors else None)
                    break
                with self.lock:
                    t_lk = time.time() if tr is not None else 0.0
                    gen = self._gen
                    (hs, hi), ev = to_host_async(*self.topk_rows(q, k))
                if ev is not None:
                    ev.synchronize()
                s, idx = hs.tolist(), hi.tolist()
                t_gpu = time.time() if tr is not None else 0.0
                with self.lock:
                    if self._gen != gen:
                        self.search_retries += 1
                        continue
                    hits = [[(sc, r, self.row_payload(r)) for sc, r in zip(srow, irow) if 0 <= r < self._n]
                            for srow, irow in zip(s, idx)]
                    pend = (self._gather_rows_async({r for row in hits for _, r, _ in row})
                            if with_vectors else None)
                break
            vec_rows = None
            if pend is not None:
                flat, outs, ev = pend
                if ev is not None:
                    ev.synchronize()
                vec_rows = (flat, outs[0].numpy() if flat else np.zeros((0, self.dim), np.float32))
        # the result objects are built after the lock is released
        out = self._build_results(hits, vec_rows)
        if tr is not None:
            tr.append((t_in, t_lk, t_gpu, time.time(), len(out)))
        return out

    def _normalize_host(self, v) -> np.ndarray:
        if isinstance(v, torch.Tensor):
            a = v.detach().float().cpu().numpy()
        else:
            a = np.asarray(v, dtype=np.float32)
        if a.ndim == 1:
            a = a[None]
        if a.shape[-1] != self.dim:
            raise ValueError(f"vector dim {a.shape[-1]} != collection {self.name} dim {self.dim}")
        return a / np.maximum(np.linalg.norm(a, axis=-1, keepdims=True), 1e-12)

    def _to_device_query(self, a: np.ndarray) -> torch.Tensor:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t.to(self.dtype)

    @staticmethod
    def _build_results(hits, vec_rows) -> List[List[Dict[str, Any]]]:
        vecs = {}
        if vec_rows is not None and vec_rows[0]:
            from ..utils.fastjson import f32_rows   # native rows of float32 values
            vecs = dict(zip(vec_rows[0], f32_rows(vec_rows[1])))
        out = []
        for row in hits:
            res = []
            for sc, r, d in row:
                d["similarity"] = sc
                if vec_rows is not None:
                    d["vector"] = vecs.get(r)
                res.append(d)
            out.append(res)
        return out

    def rows_to_results(self, scores, rows, with_vectors: bool) -> List[List[Dict[str, Any]]]:
        """Host results for row indices (caller holds ``lock``)."""
        vec_rows = self.row_vectors({i for row in rows for i in row if 0 <= i < self._n}) if with_vectors else None
        out = []
        for srow, irow in zip(scores, rows):
            res = []
            for sc, r in zip(srow, irow):
                if r < 0 or r >= self._n:
                    continue
                d = self.row_payload(r)
                d["similarity"] = sc
                if vec_rows is not None:
                    d["vector"] = vec_rows[r]
                res.append(d)
            out.append(res)
        return out

    def row_payload(self, r: int) -> Dict[str, Any]:
        d = dict(self._meta[r])
        d["id"] = self._ids[r]
        return d

    def row_vectors(self, rows) -> Dict[int, List[float]]:
        flat, arr = self.row_vectors_array(rows)
        if not flat:
            return {}
        from ..utils.fastjson import f32_rows   # native rows of float32 values
        return dict(zip(flat, f32_rows(arr)))

    def _gather_rows_async(self, rows):
        """(sorted rows, [pinned f32 copy], event) of the given rows: the device gather and
        its D2H copy enqueued on the search stream (caller holds ``lock``)."""
        flat = sorted(rows)
        if not flat:
            return flat, [], None
        with on_search(self.device):
            self._order_read()
            outs, ev = to_host_async(self._vecs[torch.tensor(flat, device=self.device)].float())
        return flat, outs, ev

    def row_vectors_array(self, rows):
        """(sorted rows, float32 numpy [n, dim]): one device gather + one D2H copy, no
        per-float Python objects (the sharded kNN ships these rows as bytes)."""
        flat = sorted(rows)
        if not flat:
            return flat, np.zeros((0, self.dim), np.float32)
        with on_search(self.device):
            self._order_read()
            arr = to_host(self._vecs[torch.tensor(flat, device=self.device)].float())[0].numpy()
        return flat, arr


def _exact_topk(X: torch.Tensor, q: torch.Tensor, k: int, chunk: int = 1 << 20):
    """Exact top-k by chunked GEMM + torch.topk (dims / k outside the kernel)."""
    Qn = q.shape[0]
    best_s = torch.full((Qn, 0), float("-inf"), device=X.device)
    best_i = torch.full((Qn, 0), -1, device=X.device, dtype=torch.long)
    qf = q.float()
    for s0 in range(0, X.shape[0], chunk):
        sc = qf @ X[s0: s0 + chunk].float().t()
        kk = min(k, sc.shape[1])
        v, i = torch.topk(sc, kk, dim=-1)
        best_s = torch.cat([best_s, v], 1)
        best_i = torch.cat([best_i, i + s0], 1)
        if best_s.shape[1] > k:
            best_s, sel = torch.topk(best_s, k, dim=-1)
            best_i = torch.gather(best_i, 1, sel)
    if best_s.shape[1] < k:
        pad = k - best_s.shape[1]
        best_s = torch.cat([best_s, best_s.new_full((Qn, pad), float("-inf"))], 1)
        best_i = torch.cat([best_i, best_i.new_full((Qn, pad), -1)], 1)
    return best_s, best_i.int()


class VectorStoreRegistry:
    """Process-wide named stores (one per collection/table), shared by sink and query agents."""

    _stores: Dict[str, VectorStore] = {}
    _lock = threading.Lock()
    persist_dir: Optional[str] = os.environ.get("LANGSTREAM_VECTOR_STORE_DIR") or None
    fsync: bool = False
    # collection -> directory bound by the sink that owns it (``bind``): the zero-config
    # default, each local vector-db-sink persisting ITS collection in ITS own state dir
    _bound: Dict[str, str] = {}

    @classmethod
    def _dir_of(cls, name: str) -> Optional[str]:
        """Where ``name`` persists: the process-wide directory when one is configured
        (persist-directory / $LANGSTREAM_VECTOR_STORE_DIR), else its sink's binding."""
        if cls.persist_dir:
            return os.path.join(cls.persist_dir, _safe(name))
        return cls._bound.get(name)

    @classmethod
    def bind(cls, name: str, directory: str) -> None:
        """Persist collection ``name`` under ``directory`` (a sink's persistent state
        directory) when no process-wide directory is configured.  Only that collection
        is affected: a second sink of another collection binds its own directory, and
        no sink's directory becomes a default for the others."""
        with cls._lock:
            if cls.persist_dir:
                return
            old = cls._bound.get(name)
            if old and old != directory:
                log.warning("vector collection %s is already persisted under %s; ignoring %s", name, old, directory)
                return
            cls._bound[name] = directory
            s = cls._stores.get(name)
            if s is not None and not s.persistent and not s.attach_persistence(directory, cls.fsync):
                log.warning("vector collection %s was created without persistence and already holds "
                            "%d rows: they are NOT durable (bind persistence before the first write)",
                            name, len(s))

    @classmethod
    def configure(cls, persist_dir: Optional[str] = None, fsync: Optional[bool] = None) -> None:
        """Set the persistence directory (and fsync policy) for collections.  Collections
        that already exist without persistence -- e.g. a query agent that started before
        the sink -- are made durable when still empty, and reported otherwise; a collection
        already persisted elsewhere keeps its directory (with a warning)."""
        with cls._lock:
            if fsync is not None:
                cls.fsync = bool(fsync)
            if not persist_dir or persist_dir == cls.persist_dir:
                return
            old = cls.persist_dir
            cls.persist_dir = persist_dir
            for name, s in cls._stores.items():
                if s.persistent:
                    log.warning("vector collection %s keeps its persistence directory under %s; the new "
                                "directory %s applies to collections created from now on", name, old, persist_dir)
                elif not s.attach_persistence(os.path.join(persist_dir, _safe(name)), cls.fsync):
                    log.warning("vector collection %s was created without persistence and already holds "
                                "%d rows: they are NOT durable (configure persistence before the first write)",
                                name, len(s))

    @classmethod
    def _persisted_dim(cls, name: str) -> Optional[int]:
        d = cls._dir_of(name)
        if not d:
            return None
        meta = os.path.join(d, "snapshot.json")
        wal = os.path.join(d, "wal.log")
        hdr = _Persistence.read_snapshot_header(os.path.join(d, "snapshot.lsv"))
        if hdr is not None:
            return int(hdr[0]["dim"])
        if os.path.exists(meta):
            with open(meta) as f:
                return int(json.load(f)["dim"])
        if os.path.exists(wal) and os.path.getsize(wal) > 4:
            with open(wal, "rb") as f:
                n = int.from_bytes(f.read(4), "little")
                e = msgpack.unpackb(f.read(n), raw=False, strict_map_key=False)
            if e[0] == "u" and e[1]:
                return len(e[2]) // 4 // len(e[1])
        return None

    @classmethod
    def get(cls, name: str, dim: Optional[int] = None, device=None, persist: bool = True) -> VectorStore:
        """The collection ``name`` (created with ``dim`` if new; restored from the
        persistence directory when one is configured and ``persist``)."""
        with cls._lock:
            s = cls._stores.get(name)
            if s is None:
                if dim is None and persist:
                    dim = cls._persisted_dim(name)
                if dim is None:
                    raise KeyError(f"vector collection {name} does not exist")
                if device is None:
                    device = "cuda" if torch.cuda.is_available() else "cpu"
                pdir = cls._dir_of(name) if persist else None
                s = VectorStore(dim, device=device, name=name, persist_dir=pdir, fsync=cls.fsync)
                cls._stores[name] = s
            return s

    @classmethod
    def exists(cls, name: str) -> bool:
        if name in cls._stores:
            return True
        return cls._persisted_dim(name) is not None

    @classmethod
    def drop(cls, name: str, purge: bool = False) -> None:
        """Forget the in-memory collection; ``purge`` also deletes its persisted data."""
        with cls._lock:
            s = cls._stores.pop(name, None)
        if s is not None:
            s.close()
        d = cls._dir_of(name) if purge else None
        if d:
            import shutil
            shutil.rmtree(d, ignore_errors=True)

    @classmethod
    def reset(cls) -> None:
        with cls._lock:
            for s in cls._stores.values():
                s.close()
            cls._stores.clear()
            cls._bound.clear()
