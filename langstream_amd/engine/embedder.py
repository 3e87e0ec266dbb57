"""Dynamic-batching embedding engine (compute-ai-embeddings on the GPU).

Any number of agent threads call :meth:`EmbeddingEngine.embed_async`; a single engine
thread drains the queue, tokenizes with the native WordPiece tokenizer (GIL released,
multi-threaded), packs up to ``max_batch_tokens`` tokens padding-free and runs one
encoder forward.  Results resolve ``concurrent.futures.Future`` objects in request
order.  This replaces the reference's one-text-per-predict local path
(``AbstractHuggingFaceEmbeddingService.java:183-207``).
"""
from __future__ import annotations

import logging
import queue
import threading
from concurrent.futures import Future
from typing import List, Optional, Sequence

import torch

from ..models.bert import BertEncoder
from ..utils.fastjson import f32_rows
from ..utils.gpu import on_aux, to_host

log = logging.getLogger(__name__)


class EmbeddingEngine:
    def __init__(self, encoder: BertEncoder, tokenizer, max_batch_tokens: int = 32768, max_len: int = 512,
                 return_tensors: bool = False):
        self.encoder = encoder
        self.tok = tokenizer
        self.max_batch_tokens = max_batch_tokens
        self.max_len = min(max_len, encoder.cfg.max_position)
        self.return_tensors = return_tensors
        self._q: "queue.Queue" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self.stats = {"batches": 0, "texts": 0, "tokens": 0}

    @property
    def dim(self) -> int:
        return self.encoder.cfg.hidden_size

    # ------------------------------------------------------------------ sync api
    def embed(self, texts: Sequence[str]) -> List[List[float]]:
        """Blocking; runs inline on the caller's thread (no engine thread needed)."""
        out = self._embed_batch(list(texts))
        return f32_rows(out) if isinstance(out, torch.Tensor) else out

    def embed_tensor(self, texts: Sequence[str]) -> torch.Tensor:
        """Device tensor, produced on the device's auxiliary stream (consume it there,
        e.g. VectorStore.upsert, or synchronise)."""
        if hasattr(self.tok, "encode_batch_packed"):
            ids, lens = self.tok.encode_batch_packed(list(texts), max_len=self.max_len)
            with on_aux(self.encoder.device):
                return self.encoder.encode_arrays(ids, lens)
        toks = self.tok.encode_batch(list(texts), max_len=self.max_len)
        with on_aux(self.encoder.device):
            return self.encoder.encode_tokens(toks)

    def _embed_batch(self, texts: List[str]):
        """Tokenise once (native, multi-threaded), encode in packed batches of at most
        ``max_batch_tokens`` on the auxiliary stream, one device->host copy at the end."""
        import numpy as np
        if hasattr(self.tok, "encode_batch_packed"):
            ids, lens = self.tok.encode_batch_packed(texts, max_len=self.max_len)
        else:
            tl = self.tok.encode_batch(texts, max_len=self.max_len)
            lens = np.array([len(t) for t in tl], dtype=np.int32)
            ids = np.array([x for t in tl for x in t], dtype=np.int32)
        ends = np.cumsum(lens, dtype=np.int64)
        outs = []
        i, n = 0, len(lens)
        with on_aux(self.encoder.device):  # do not queue behind the LLM engine's steps
            while i < n:
                # as many texts as fit in max_batch_tokens (at least one)
                t0 = ends[i - 1] if i else 0
                j = max(i + 1, int(np.searchsorted(ends, t0 + self.max_batch_tokens, side="right")))
                t1 = ends[j - 1]
                outs.append(self.encoder.encode_arrays(ids[t0:t1], lens[i:j]))
                self.stats["batches"] += 1
                self.stats["texts"] += j - i
                self.stats["tokens"] += int(t1 - t0)
                i = j
            if not outs:
                return torch.zeros(0, self.dim)
            return to_host(outs[0] if len(outs) == 1 else torch.cat(outs))[0]

    # ------------------------------------------------------------------ async api
    def embed_async(self, texts: Sequence[str]) -> Future:
        f: Future = Future()
        self._q.put((list(texts), f))
        if self._thread is None:
            self.start()
        return f

    def start(self) -> None:
        if self._thread is not None:
            return
        self._thread = threading.Thread(target=self._loop, name="embed-engine", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        self._q.put(None)
        if self._thread is not None:
            self._thread.join(timeout=10)
            self._thread = None

    def _loop(self) -> None:
        if self.encoder.device.type == "cuda":
            torch.cuda.set_device(self.encoder.device)
        while not self._stop.is_set():
            item = self._q.get()
            if item is None:
                continue
            pending = [item]
            ntexts = len(item[0])
            # coalesce whatever else is queued (dynamic batching)
            while ntexts < 4096:
                try:
                    nxt = self._q.get_nowait()
                except queue.Empty:
                    break
                if nxt is None:
                    continue
                pending.append(nxt)
                ntexts += len(nxt[0])
            texts = [t for p in pending for t in p[0]]
            try:
                out = self._embed_batch(texts)
                k = 0
                for p_texts, fut in pending:
                    part = out[k: k + len(p_texts)]
                    k += len(p_texts)
                    # float32 rows: serialised at float32 precision (utils/fastjson.py)
                    fut.set_result(part if self.return_tensors else f32_rows(part))
            except Exception as e:  # noqa: BLE001
                log.exception("embedding batch failed")
                for _, fut in pending:
                    if not fut.done():
                        fut.set_exception(e)
