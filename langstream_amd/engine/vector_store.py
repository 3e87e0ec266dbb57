"""HBM-resident vector store with brute-force kNN on the GPU.

Rows are L2-normalised bf16 vectors in one device tensor ``[capacity, dim]`` (dense:
deletes swap the last row into the hole, so ``[0, n)`` is always valid and the kNN
kernel never scans dead rows).  Search is the fused MFMA GEMM + top-k kernel
(``ops.knn_topk``), so cosine similarity over 10^6-10^7 rows per GPU is one kernel pass
over HBM.  Metadata (arbitrary JSON-able dicts: text, source, ...) stays on the host.
Capacity doubles on demand; at 384 dims a 288 GB GPU holds >10^8 rows.

Used by ``vector-db-sink`` (upsert/delete) and ``query-vector-db`` (search), and by
the JDBC-compatible SQL datasource for ``ORDER BY cosine_similarity(...) DESC LIMIT k``.
"""
from __future__ import annotations

import threading
from typing import Any, Dict, List, Optional, Sequence

import torch

from .. import ops
from ..utils.gpu import on_aux, to_host


class VectorStore:
    def __init__(self, dim: int, device="cuda", capacity: int = 1024, dtype=torch.bfloat16, name: str = "default"):
        self.dim = dim
        self.name = name
        self.device = torch.device(device)
        self.dtype = dtype
        with on_aux(self.device):  # every GPU op of the store runs on the auxiliary stream
            self._vecs = torch.zeros(max(16, capacity), dim, device=self.device, dtype=dtype)
        self._n = 0
        self._ids: List[Any] = []
        self._meta: List[Dict[str, Any]] = []
        self._row: Dict[Any, int] = {}
        self._lock = threading.RLock()

    def __len__(self) -> int:
        return self._n

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
            raise ValueError(f"vector dim {t.shape[-1]} != store dim {self.dim}")
        t = t.to(self.device)
        return torch.nn.functional.normalize(t, dim=-1, eps=1e-12).to(self.dtype)

    def upsert(self, ids: Sequence[Any], vectors, metadata: Optional[Sequence[Dict[str, Any]]] = None) -> None:
        with on_aux(self.device):
            self._upsert(ids, vectors, metadata)

    def _upsert(self, ids, vectors, metadata) -> None:
        vecs = self._normalize(vectors)
        with self._lock:
            metadata = metadata or [{} for _ in ids]
            new_rows = [i for i in ids if i not in self._row]
            self._grow(self._n + len(set(new_rows)))
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
            self._vecs[torch.tensor(rows, device=self.device, dtype=torch.long)] = vecs

    def delete(self, ids: Sequence[Any]) -> int:
        with on_aux(self.device):
            return self._delete(ids)

    def _delete(self, ids: Sequence[Any]) -> int:
        removed = 0
        with self._lock:
            for k in ids:
                r = self._row.pop(k, None)
                if r is None:
                    continue
                last = self._n - 1
                if r != last:
                    self._vecs[r] = self._vecs[last]
                    self._ids[r] = self._ids[last]
                    self._meta[r] = self._meta[last]
                    self._row[self._ids[r]] = r
                self._ids.pop()
                self._meta.pop()
                self._n -= 1
                removed += 1
        return removed

    def get(self, key: Any) -> Optional[Dict[str, Any]]:
        with self._lock:
            r = self._row.get(key)
            return None if r is None else dict(self._meta[r])

    def vector(self, key: Any) -> Optional[List[float]]:
        with self._lock:
            r = self._row.get(key)
            if r is None:
                return None
            with on_aux(self.device):
                return to_host(self._vecs[r].float())[0].tolist()

    def search(self, queries, k: int = 10, with_vectors: bool = False) -> List[List[Dict[str, Any]]]:
        """queries: [Q, dim] (list or tensor).  Returns per query a list of
        {"id", "similarity", **metadata} sorted by decreasing cosine similarity."""
        with on_aux(self.device):
            return self._search(queries, k, with_vectors)

    def _search(self, queries, k: int, with_vectors: bool) -> List[List[Dict[str, Any]]]:
        q = self._normalize(queries)
        with self._lock:
            n = self._n
            if n == 0:
                return [[] for _ in range(q.shape[0])]
            kk = max(1, min(k, 64, n))
            s, idx = ops.knn_topk(self._vecs[:n], q.contiguous(), kk)
            s, idx = (t.tolist() for t in to_host(s, idx))
            vec_rows = None
            if with_vectors:
                flat = sorted({i for row in idx for i in row if i >= 0})
                if flat:
                    vv = to_host(self._vecs[torch.tensor(flat, device=self.device)].float())[0].tolist()
                    vec_rows = dict(zip(flat, vv))
            out = []
            for qi in range(len(idx)):
                res = []
                for sc, r in zip(s[qi], idx[qi]):
                    if r < 0 or r >= n:
                        continue
                    d = dict(self._meta[r])
                    d["id"] = self._ids[r]
                    d["similarity"] = sc
                    if vec_rows is not None:
                        d["vector"] = vec_rows[r]
                    res.append(d)
                out.append(res)
            return out


class VectorStoreRegistry:
    """Process-wide named stores (one per collection/table), shared by sink and query agents."""

    _stores: Dict[str, VectorStore] = {}
    _lock = threading.Lock()

    @classmethod
    def get(cls, name: str, dim: Optional[int] = None, device=None) -> VectorStore:
        with cls._lock:
            s = cls._stores.get(name)
            if s is None:
                if dim is None:
                    raise KeyError(f"vector collection {name} does not exist")
                if device is None:
                    device = "cuda" if torch.cuda.is_available() else "cpu"
                s = VectorStore(dim, device=device, name=name)
                cls._stores[name] = s
            return s

    @classmethod
    def exists(cls, name: str) -> bool:
        return name in cls._stores

    @classmethod
    def drop(cls, name: str) -> None:
        with cls._lock:
            cls._stores.pop(name, None)

    @classmethod
    def reset(cls) -> None:
        with cls._lock:
            cls._stores.clear()
