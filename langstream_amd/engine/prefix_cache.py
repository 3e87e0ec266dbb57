"""Automatic prefix KV reuse for the LLM engine (exact: the reused KV is bit-for-bit what
the prompt's own prefill would write for those positions, up to kernel routing).

Prompts built from one template share a token prefix -- the RAG chain's chat template
and system message are ~45 of a ~350-token prompt in the config-4 bench (bench.py APP)
-- and a prefix's KV depends only on the prefix (causal attention, absolute RoPE
positions).  This cache keeps the KV of such prefixes in blocks of its own and starts a
new prompt's prefill at the end of its longest cached prefix, after copying those
blocks into the prompt's own blocks (copy, not share: the prompt's first partial block
receives its own tokens after the prefix).

* Discovery: a new prompt is compared with the heads of the last ``history`` prompts;
  a common prefix of at least ``min_len`` tokens (and ``min_gain`` longer than what the
  cache already holds for it) is captured from this request once its prefill has
  passed it.
* Capture and reuse are KV block copies that ride in the NEXT step's arena
  (``kvcopy``, executed before that step's forward on the step stream --
  ``StepExecutor::run`` / ``PyStepExecutor._run``), so they are ordered after the step
  that computed the prefix and before any step that reads them, and under tensor
  parallelism every rank performs them (the arena is broadcast).
* Full prefix blocks are SHARED: a hit's block table starts with the entry's blocks
  (read-only -- the prompt writes from the prefix end on, which lies past them), so
  only the partial last block is copied, and every sequence of the batch reads the same
  physical prefix KV (cache hits in the decode attention instead of HBM reads).
* At most ``max_entries`` prefixes (LRU); an entry is evicted only when no live request
  shares its blocks and no copy of the step being built reads them.

The vLLM / SGLang production engines do the same (block-hash / radix-tree prefix
caching); the reference delegates generation to remote services (OpenAI prompt caching,
OpenAICompletionService.java:122-404).  ``LS_PREFIX_CACHE=0`` disables it.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np


class _Entry:
    __slots__ = ("ids", "blocks", "last_step", "hits", "refs")

    def __init__(self, ids: np.ndarray, blocks: List[int], step: int):
        self.ids, self.blocks, self.last_step, self.hits = ids, blocks, step, 0
        self.refs = 0   # live requests whose block tables hold this entry's full blocks


class PrefixCache:
    def __init__(self, allocator, block: int, max_entries: int = 8, min_len: int = 32, max_len: int = 512,
                 history: int = 32, min_gain: int = 16, max_copies: int = 2048):
        self.allocator, self.block = allocator, block
        self.max_entries, self.min_len, self.max_len = max_entries, min_len, max_len
        self.min_gain, self.max_copies = min_gain, max_copies
        self.entries: List[_Entry] = []
        # heads of the last `history` prompts, one row each (-1 padded), compared with a
        # new prompt in one vectorised pass
        self._heads = np.full((history, max_len), -1, dtype=np.int64)
        self._nrecent = 0
        self._next = 0
        self.pending: List[Tuple[object, int]] = []      # (request, prefix length) to capture
        self.copies: List[Tuple[int, int]] = []          # (src, dst) block pairs for the next step
        self.stats: Dict[str, int] = {"hit_tokens": 0, "hits": 0, "captures": 0, "evictions": 0}

    # -------------------------------------------------------------- lookups
    def _head(self, r) -> np.ndarray:
        h = getattr(r, "_prefix_head", None)
        if h is None:
            h = np.asarray(r.prompt_ids[: self.max_len], dtype=np.int64)
            r._prefix_head = h
        return h

    def _best(self, head: np.ndarray, n_prompt: int) -> Optional[_Entry]:
        best = None
        for e in self.entries:
            L = len(e.ids)
            if L < n_prompt and L <= len(head) and (best is None or L > len(best.ids)) \
                    and np.array_equal(head[:L], e.ids):
                best = e
        return best

    def observe(self, r) -> None:
        """A request reached the scheduler: look for a shared prefix worth capturing."""
        head = self._head(r)
        n = len(r.prompt_ids)
        lcp = 0
        m = min(len(head), n - 1)
        if self._nrecent and m > 0:
            neq = self._heads[: self._nrecent, :m] != head[:m]       # padding (-1) never matches
            first = np.where(neq.any(axis=1), neq.argmax(axis=1), m)
            lcp = int(first.max())
        row = self._heads[self._next]
        row[:] = -1
        row[: len(head)] = head
        self._next = (self._next + 1) % len(self._heads)
        self._nrecent = min(self._nrecent + 1, len(self._heads))
        if lcp < self.min_len:
            return
        have = self._best(head, n)
        if have is not None and lcp < len(have.ids) + self.min_gain:
            return
        # one pending capture per prefix: a longer one only when it gains min_gain tokens
        for q, L in self.pending:
            k = min(L, lcp)
            if lcp < L + self.min_gain and np.array_equal(self._head(q)[:k], head[:k]):
                return
        self.pending.append((r, lcp))

    def hit(self, r, step: int) -> Tuple[int, Optional[_Entry]]:
        """Longest cached prefix of a fresh request's prompt: (length, entry) or (0, None)."""
        e = self._best(self._head(r), len(r.prompt_ids))
        if e is None:
            return 0, None
        nb = (len(e.ids) + self.block - 1) // self.block
        if len(self.copies) + nb > self.max_copies:
            return 0, None
        return len(e.ids), e

    def apply_hit(self, r, e: _Entry, step: int) -> None:
        """The request took entry e: its block table starts with the entry's full blocks
        (shared, read-only); the partial last prefix block is copied into its own block."""
        nb = (len(e.ids) + self.block - 1) // self.block
        nfull = len(e.ids) // self.block
        self.copies.extend(zip(e.blocks[nfull:nb], r.blocks[nfull:nb]))
        e.refs += 1
        r._prefix_entry = e
        e.last_step = step
        e.hits += 1
        self.stats["hits"] += 1
        self.stats["hit_tokens"] += len(e.ids)

    # -------------------------------------------------------------- captures
    def collect_captures(self, step: int, headroom: int = 0) -> None:
        """Capture every pending prefix whose request has computed past it (its KV is
        written by an earlier step); requests that finished or lost their blocks drop.
        ``headroom``: blocks a capture may not take (one per decoding sequence of the
        step being built, so a capture never starves decoding)."""
        keep = []
        for r, L in self.pending:
            if getattr(r, "finished", False):
                continue
            nb = (L + self.block - 1) // self.block
            if r.num_computed < L or len(r.blocks) < nb:   # not there yet (or preempted)
                keep.append((r, L))
                continue
            if len(self.copies) + nb > self.max_copies:
                keep.append((r, L))
                continue
            if len(self.entries) >= self.max_entries and not self._evict(step):
                continue
            if self.allocator.num_free() - headroom < nb:
                keep.append((r, L))            # the pool is short now: retry at a later step
                continue
            dst = list(self.allocator.allocate(nb))
            self.copies.extend(zip(r.blocks[:nb], dst))
            self.entries.append(_Entry(self._head(r)[:L].copy(), dst, step))
            self.stats["captures"] += 1
        self.pending = keep

    def release(self, r) -> None:
        """A request gave its blocks back (finished or preempted)."""
        e = getattr(r, "_prefix_entry", None)
        if e is not None:
            e.refs -= 1
            r._prefix_entry = None

    def _evict(self, step: int) -> bool:
        # an entry is evictable once no live request shares its blocks and no copy of
        # this step reads them
        cands = [e for e in self.entries if e.last_step != step and e.refs == 0]
        if not cands:
            return False
        e = min(cands, key=lambda x: x.last_step)
        self.entries.remove(e)
        self.allocator.free(e.blocks)
        self.stats["evictions"] += 1
        return True

    def _idle(self, step: int, keep: Optional[_Entry] = None) -> List[_Entry]:
        return [e for e in self.entries if e.refs == 0 and e.last_step != step and e is not keep]

    def reclaimable(self, step: int, keep: Optional[_Entry] = None) -> int:
        """Blocks that ``reclaim`` could give back for the step being built."""
        return sum(len(e.blocks) for e in self._idle(step, keep))

    def reclaim(self, want_free: int, step: int, keep: Optional[_Entry] = None) -> int:
        """KV pool pressure: evict idle entries (no request shares their blocks, no copy of
        step ``step`` reads them), least recently used first, until ``want_free`` blocks
        are free or none is left.  The scheduler calls this before it preempts a sequence,
        skips a decode row or ends a prompt with 'length' -- cached prefixes are an
        optimisation and never hold blocks a sequence needs.  Returns the blocks freed."""
        freed = 0
        while self.allocator.num_free() < want_free:
            cands = self._idle(step, keep)
            if not cands:
                break
            e = min(cands, key=lambda x: x.last_step)
            self.entries.remove(e)
            self.allocator.free(e.blocks)
            freed += len(e.blocks)
            self.stats["evictions"] += 1
            self.stats["reclaimed_blocks"] = self.stats.get("reclaimed_blocks", 0) + len(e.blocks)
        return freed

    def take_copies(self) -> List[Tuple[int, int]]:
        c, self.copies = self.copies, []
        return c

    def clear(self) -> None:
        """Drop every entry no request shares (the rest stay until released)."""
        for e in [e for e in self.entries if e.refs == 0]:
            self.allocator.free(e.blocks)
            self.entries.remove(e)
        self.pending.clear()
        self.copies.clear()
