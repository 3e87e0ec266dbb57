"""Continuous-batching LLM serving engine on MI355X.

Replaces the remote completion services the reference calls from
``ai-chat-completions`` / ``ai-text-completions`` (SURVEY §2.10 K2/K3;
``OpenAICompletionService.java:122-404``, ``OllamaProvider.java:273-311``) with a local
engine:

* paged KV cache (64-token blocks, V stored transposed in 8-key groups; blocks managed by the native
  ``BlockAllocator``), sized from the 288 GB HBM budget;
* unified steps: every step carries one decode token per running sequence plus, when
  prompts are waiting, chunked-prefill tokens (``max_prefill_tokens`` per step), so new
  requests never stall the sequences already decoding;
* the scheduler describes a step in a fixed-layout pinned "arena" through numpy views
  (``engine/arena.py``); the native ``StepExecutor`` runs the whole step -- upload,
  token feedback, forward, logit deltas, sampling, download -- in ONE GIL-released
  call, so the agent threads sharing the interpreter cannot stall the GPU;
* pure-decode steps replay a HIP graph captured per batch-size bucket (one graph serves
  every context length: the split-KV grid is sized for ``max_model_len``); mixed steps
  run eagerly from C++;
* one-step lookahead: the next step's input tokens are gathered ON DEVICE from the
  previous step's sampled tokens, so step N+1 is launched before step N's tokens are
  copied back -- host bookkeeping (detokenisation, streaming callbacks, scheduling)
  overlaps the GPU instead of idling it.  Finishing is detected one step late; that
  step's extra token is discarded;
* sampling on device (temperature / top-k / top-p / seed / penalties / logit-bias,
  log-probs of the sampled token + top-n alternatives for FLARE);
* recompute-preemption when KV blocks run out;
* automatic prefix KV reuse (``engine/prefix_cache.py``): prompts that share a template
  prefix start their prefill after it, its KV copied from a cached copy;
* tensor parallel: rank 0 schedules; its executor broadcasts the device arena over
  RCCL and the other ranks' executors (``worker_loop``, pure C++) mirror every step.
"""
from __future__ import annotations

import itertools
import logging
import os
import collections
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..models.llama import LlamaModel
from ..native import lib
from .prefix_cache import PrefixCache
from .arena import (H_BUCKET, H_KIND, H_ND, H_NCOPY, H_NDELTA, H_NGATHER, H_NPS, H_NROWS, H_NTILES, H_NTOP,
                    H_ROWS_ALL, H_T, KIND_STEP, MAX_KV_COPIES, ArenaLayout, NativeStepExecutor, PyStepExecutor)

log = logging.getLogger(__name__)
BLOCK = ops.KV_BLOCK
NSLOTS = 3          # arena ring: one being filled, one in flight, one being retired
MAX_DELTAS = 1 << 16


@dataclass
class SamplingParams:
    max_tokens: int = 256
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    seed: Optional[int] = None
    stop_token_ids: Sequence[int] = ()
    stop: Sequence[str] = ()
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    logit_bias: Optional[Dict[int, float]] = None
    logprobs: int = 0            # >0: also return this many top alternatives per token
    ignore_eos: bool = False
    min_tokens: int = 0

    @property
    def needs_history(self) -> bool:
        return bool(self.presence_penalty or self.frequency_penalty)


@dataclass
class TokenEvent:
    request_id: int
    token_id: int
    logprob: float
    text: str                    # text delta decoded so far (may be "" for partial UTF-8)
    index: int                   # output position
    finished: bool
    finish_reason: Optional[str] = None
    top: Optional[List[tuple]] = None  # [(token_id, logprob)] alternatives


def _device_index(dev) -> int:
    """Index of a CUDA device given as 'cuda', 'cuda:N' or a torch.device ('cuda' alone:
    the current device)."""
    d = torch.device(dev)
    return d.index if d.index is not None else torch.cuda.current_device()


@dataclass
class Request:
    request_id: int
    prompt_ids: List[int]
    params: SamplingParams
    callback: Optional[Callable[[TokenEvent], None]] = None
    arrival: float = field(default_factory=time.perf_counter)
    # state
    output_ids: List[int] = field(default_factory=list)
    output_logprobs: List[float] = field(default_factory=list)
    blocks: List[int] = field(default_factory=list)
    shared_blocks: int = 0       # blocks[:shared_blocks] belong to a prefix-cache entry (read-only)
    num_computed: int = 0        # tokens whose KV is (or is being) written to the cache
    num_launched: int = 0        # output tokens launched (sampled or in flight)
    finished: bool = False
    finish_reason: Optional[str] = None
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    pending_row: int = -1        # row of this request's in-flight token in the lookahead step
    pending_step: int = -1       # id of the step that holds that token
    _emitted: bytearray = field(default_factory=bytearray)
    _text: str = ""
    _done_event: threading.Event = field(default_factory=threading.Event)
    seed: int = 0

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    def token_at(self, i: int) -> int:
        n = len(self.prompt_ids)
        return self.prompt_ids[i] if i < n else self.output_ids[i - n]

    def tokens(self, s: int, e: int) -> List[int]:
        n = len(self.prompt_ids)
        if e <= n:
            return self.prompt_ids[s:e]
        return (self.prompt_ids[s:] if s < n else []) + self.output_ids[max(0, s - n): e - n]

    @property
    def total_len(self) -> int:
        return len(self.prompt_ids) + self.num_launched

    @property
    def text(self) -> str:
        return self._text

    def wait(self, timeout: Optional[float] = None) -> bool:
        return self._done_event.wait(timeout)


@dataclass
class _InFlight:
    reqs: List[Request]
    slot: int
    n_top: int
    step_id: int
    ready: bool = False          # results already waited for (by the next exec.step)


class LLMEngine:
    def __init__(self, model: LlamaModel, tokenizer=None, *, num_blocks: Optional[int] = None,
                 kv_fraction: float = 0.55, max_model_len: int = 4096, max_batch: int = 256,
                 max_prefill_tokens: int = 8192, use_graphs: bool = True, graph_buckets: Sequence[int] = (),
                 lookahead: bool = True, device=None, prefix_cache: Optional[bool] = None):
        self.model = model
        self.cfg = model.cfg
        self.tok = tokenizer
        self.device = torch.device(device or model.device)
        self.tp = model.tp
        self.max_model_len = min(max_model_len, self.cfg.max_position)
        self.max_blocks_per_seq = (self.max_model_len + BLOCK - 1) // BLOCK
        self.max_batch = max_batch
        self.max_prefill_tokens = max_prefill_tokens
        self.is_gpu = self.device.type == "cuda"
        self.use_graphs = use_graphs and self.is_gpu
        if self.is_gpu:
            ops.enable_decode_gemm_tuning()   # cold-picked GEMM solutions, before any graph capture
        self.lookahead = lookahead
        D = self.cfg.head_dim
        hkv = model.hkv
        bytes_per_block = 2 * self.cfg.num_layers * hkv * BLOCK * D * torch.finfo(model.dtype).bits // 8
        if num_blocks is None:
            if self.is_gpu:
                free, _ = torch.cuda.mem_get_info(self.device)
                num_blocks = int(free * kv_fraction) // bytes_per_block
            else:
                num_blocks = 256
            if self.tp.world > 1:  # every rank must hold the same block pool
                t = torch.tensor([num_blocks], device=self.device)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.tp.group)
                num_blocks = int(t.item())
        self.num_blocks = int(num_blocks)
        self.kv_caches = []
        for _ in range(self.cfg.num_layers):
            self.kv_caches.append(ops.new_kv_cache(self.num_blocks, hkv, D, self.device, model.dtype))
        self.allocator = lib().BlockAllocator(self.num_blocks)
        self.nsplit, self.bps = ops.decode_splits(self.max_blocks_per_seq)
        if prefix_cache is None:
            prefix_cache = os.environ.get("LS_PREFIX_CACHE", "1") != "0"
        self.prefix: Optional[PrefixCache] = (PrefixCache(self.allocator, BLOCK, max_copies=MAX_KV_COPIES)
                                              if prefix_cache else None)
        # ---- step arena + executor
        G = model.hq // model.hkv
        max_tokens = max_prefill_tokens + max_batch
        max_tiles = (max_prefill_tokens * G + ops.PREFILL_ROWS - 1) // ops.PREFILL_ROWS + max_batch + 1
        self.layout = ArenaLayout.build(max_tokens, max_batch, self.max_blocks_per_seq, max_tiles, MAX_DELTAS)
        if self.is_gpu:
            self.exec = NativeStepExecutor(model, self.kv_caches, self.layout, NSLOTS, self.nsplit, self.bps,
                                           self.use_graphs, self.device)
        else:
            self.exec = PyStepExecutor(model, self.kv_caches, self.layout, NSLOTS, self.nsplit, self.bps,
                                       self.device, self.tp.group, self.tp.world)
        self._slot = 0
        self._G = G
        self._ids = itertools.count(1)
        self._inbox: "queue.Queue[Request]" = queue.Queue()
        self.waiting: List[Request] = []
        self.running: List[Request] = []
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._wake = threading.Event()
        self._inflight: Optional[_InFlight] = None
        self._step_id = 0
        self.ttft_s: collections.deque = collections.deque(maxlen=4096)   # engine-side arrival -> first token
        self.stats = {"prefill_steps": 0, "decode_steps": 0, "mixed_steps": 0, "prefill_tokens": 0,
                      "decode_tokens": 0, "preemptions": 0, "requests": 0, "finished": 0, "graph_steps": 0,
                      "host_ms": 0.0, "wait_ms": 0.0, "launch_ms": 0.0, "retire_ms": 0.0, "prefix_hit_tokens": 0,
                      "prompt_tokens": 0}
        # prompt lengths of the most recent requests (decode attention cost follows the longest context)
        self.prompt_lens: collections.deque = collections.deque(maxlen=8192)
        # wall-clock (time.time) times at which requests reached the scheduler
        self.arrival_log: collections.deque = collections.deque(maxlen=8192)
        # token counts of the recent steps that carried prefill work
        self.prefill_step_tokens: collections.deque = collections.deque(maxlen=4096)
        self.buckets = sorted(set(graph_buckets or [b for b in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192,
                                                                 224, 256, 320, 384, 448, 512) if b <= max_batch]
                                  + [max_batch]))
        self._eos = set(self.cfg.eos_token_ids)
        if tokenizer is not None and getattr(tokenizer, "eos_ids", None):
            self._eos |= set(tokenizer.eos_ids)
        self._eos_list = sorted(self._eos)
        self._tok_bytes: Optional[List[bytes]] = None

    # ------------------------------------------------------------------ public api
    def submit(self, prompt_ids: List[int], params: Optional[SamplingParams] = None,
               callback: Optional[Callable[[TokenEvent], None]] = None) -> Request:
        params = params or SamplingParams()
        prompt_ids = list(prompt_ids)[-(self.max_model_len - 1):] or [self.cfg.bos_token_id]
        r = Request(next(self._ids), prompt_ids, params, callback)
        r.seed = params.seed if params.seed is not None else (r.request_id * 7919) & 0x7FFFFFFF
        self._inbox.put(r)
        self._wake.set()
        return r

    def generate(self, prompts: List[List[int]], params: Optional[SamplingParams] = None) -> List[Request]:
        """Synchronous helper: run all prompts to completion (drives the loop inline
        when no background thread is running)."""
        reqs = [self.submit(p, params) for p in prompts]
        if self._thread is None:
            while not all(r.finished for r in reqs):
                self.step()
            self._flush()
        else:
            for r in reqs:
                r.wait()
        return reqs

    def start(self) -> None:
        if self._thread is not None:
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._loop, name="llm-engine", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        self._wake.set()
        if self._thread is not None:
            self._thread.join(timeout=30)
            self._thread = None
        if self.tp.world > 1 and self.tp.rank == 0:
            self._flush()
            self.exec.shutdown()  # tell the workers to leave worker_loop()

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or not self._inbox.empty() or self._inflight is not None)

    def capture_graphs(self, sizes: Optional[Sequence[int]] = None) -> None:
        """Capture decode graphs up front (every TP rank captures in lock-step)."""
        if not self.use_graphs:
            return
        self._flush()
        for b in sizes or self.buckets:
            self.exec.capture(b)

    def worker_loop(self) -> None:
        """Non-zero TP ranks: mirror rank 0's steps until it stops."""
        assert self.tp.world > 1 and self.tp.rank != 0
        if self.is_gpu:
            torch.cuda.set_device(_device_index(self.device))
        self.exec.worker_loop()

    # ------------------------------------------------------------------ loop
    def _loop(self) -> None:
        import sys
        # the engine thread shares the GIL with agent threads: a short switch interval
        # bounds how long host bookkeeping elsewhere can delay the next GPU launch
        sys.setswitchinterval(min(sys.getswitchinterval(), 0.001))
        if self.is_gpu:
            torch.cuda.set_device(_device_index(self.device))
        self._loop_body()

    def _loop_body(self) -> None:
        from ..utils.profiling import ThreadProfiler
        prof = ThreadProfiler("llm-engine")
        while not self._stop.is_set():
            prof.tick()
            if not self.has_work():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                self.step()
            except Exception:  # noqa: BLE001
                log.exception("engine step failed; failing in-flight requests")
                self._inflight = None
                for r in list(self.running) + list(self.waiting):
                    self._finish(r, "error")
                self.running.clear()
                self.waiting.clear()

    def _drain_inbox(self) -> None:
        while True:
            try:
                r = self._inbox.get_nowait()
            except queue.Empty:
                break
            self.waiting.append(r)
            if self.prefix is not None:
                self.prefix.observe(r)
            self.stats["requests"] += 1
            self.stats["prompt_tokens"] += len(r.prompt_ids)
            self.prompt_lens.append(len(r.prompt_ids))
            self.arrival_log.append(time.time())

    def step(self) -> None:
        """Schedule + launch one step, then retire the previous in-flight step."""
        t0 = time.perf_counter()
        self._drain_inbox()
        # sequences needing host-exact history (penalties) force a synchronous step
        if self._inflight is not None and (not self.lookahead or any(r.params.needs_history for r in self.running)):
            self._flush()
        decode = self._schedule_decode()
        chunks = self._schedule_prefill(len(decode))
        if not decode and not chunks:
            self._flush()
            return
        if self.prefix is not None and self.prefix.pending:
            # a capture's block copies make this step an eager one (graphs carry no copies)
            self.prefix.collect_captures(self._step_id + 1, headroom=len(decode))
        launched = self._launch(decode, chunks)
        prev, self._inflight = self._inflight, launched
        self.stats["host_ms"] += (time.perf_counter() - t0) * 1000
        if prev is not None:
            t1 = time.perf_counter()
            self._retire(prev)
            self.stats["retire_ms"] += (time.perf_counter() - t1) * 1000
        if not self.lookahead:
            self._flush()

    def _flush(self) -> None:
        if self._inflight is not None:
            prev, self._inflight = self._inflight, None
            self._retire(prev)

    # ------------------------------------------------------------------ scheduling
    def _blocks_needed(self, r: Request, upto: int) -> int:
        return max(0, (upto + BLOCK - 1) // BLOCK - len(r.blocks))

    def _decode_candidates(self) -> List[Request]:
        return [r for r in self.running
                if not r.finished and r.num_launched < r.params.max_tokens and r.total_len < self.max_model_len]

    def _schedule_decode(self) -> List[Request]:
        """Every running sequence (prompt cached, not finished, not at max_tokens) gets
        one decode token; allocate a block when it crosses a boundary (retiring the
        in-flight step and preempting the newest sequences when the pool is short)."""
        cands = self._decode_candidates()[: self.max_batch]
        need = sum(self._blocks_needed(r, r.num_computed + 1) for r in cands)
        sid = self._step_id + 1
        if need > self.allocator.num_free() and self.prefix is not None:
            self.prefix.reclaim(need, sid)   # idle cached prefixes go before any sequence does
        if need > self.allocator.num_free():
            self._flush()  # exact host state before preempting
            cands = self._decode_candidates()[: self.max_batch]
            need = sum(self._blocks_needed(r, r.num_computed + 1) for r in cands)
            if self.prefix is not None:
                self.prefix.reclaim(need, sid)
            while need > self.allocator.num_free() and len(cands) > 1 and self._preempt_one():
                cands = self._decode_candidates()[: self.max_batch]
                need = sum(self._blocks_needed(r, r.num_computed + 1) for r in cands)
        out: List[Request] = []
        for r in cands:
            n = self._blocks_needed(r, r.num_computed + 1)
            if n:
                if not self.allocator.can_allocate(n) and self.prefix is not None:
                    self.prefix.reclaim(n, sid)
                if not self.allocator.can_allocate(n):
                    continue
                r.blocks += self.allocator.allocate(n)
            out.append(r)
        # rows by context length, longest first.  The decode-attention launch at large batch
        # is one wave per (row, kv-head), all resident at once, dealt to the CUs in row
        # order: sorted rows give every CU a mix of long and short contexts, where arrival
        # order can stack long ones on one CU and the launch ends with that CU (B = 256,
        # contexts 265..566 in scattered blocks: 80.2 us sorted vs 87.7 us unsorted,
        # profiles/attn_r3c/pair_vs_sorted_ab.log)
        out.sort(key=lambda r: -r.num_computed)
        return out

    def _schedule_prefill(self, n_decode: int):
        # a full step (decode rows + prefill tokens) is a multiple of 256 tokens: hipBLASLt
        # picked a ~70 % slower qkv kernel at M = 16384 + 204 than at 16384 (RAG bench)
        budget = self.max_prefill_tokens - (n_decode % 256 if self.max_prefill_tokens > 4096 else 0)
        chosen = []
        while self.waiting and budget > 0 and len(self.running) + len(chosen) < self.max_batch:
            r = self.waiting[0]
            if r.finished:
                self.waiting.pop(0)
                continue
            total = r.num_tokens
            # a fresh prompt whose prefix is cached starts after it (KV copied in this step)
            hit, entry = (self.prefix.hit(r, self._step_id + 1)
                          if self.prefix is not None and r.num_computed == 0 and not r.blocks else (0, None))
            base = r.num_computed + hit
            remaining = total - base
            n = min(remaining, budget)
            need = self._blocks_needed(r, base + n)
            headroom = n_decode  # let every decoding sequence grow by one more block
            # full blocks of the prefix are shared with the entry (read-only: this prompt
            # writes from position `hit` on), the partial one is copied
            nshared = hit // BLOCK
            if hit:
                need = (base + n + BLOCK - 1) // BLOCK - nshared
            if hit and not self.allocator.can_allocate(need + headroom):
                self.prefix.reclaim(need + headroom, self._step_id + 1, keep=entry)
            if hit and self.allocator.can_allocate(need + headroom):
                r.num_computed = base
                r.blocks = list(entry.blocks[:nshared]) + list(self.allocator.allocate(need))
                r.shared_blocks = nshared
                self.prefix.apply_hit(r, entry, self._step_id + 1)
                chosen.append((r, n))
                budget -= n
                if n < remaining:
                    break
                self.waiting.pop(0)
                continue
            if hit:   # no room with the hit: the plain path decides (it may trim or stop)
                remaining = total - r.num_computed
                n = min(remaining, budget)
                need = self._blocks_needed(r, r.num_computed + n)
            if not self.allocator.can_allocate(need + headroom) and self.prefix is not None:
                self.prefix.reclaim(need + headroom, self._step_id + 1)
            if not self.allocator.can_allocate(need + headroom):
                if not chosen and not self.running:
                    fit = (self.allocator.num_free() + len(r.blocks)) * BLOCK - r.num_computed
                    if fit <= 0:
                        self._finish(self.waiting.pop(0), "length")
                        continue
                    n = min(n, fit)
                    need = self._blocks_needed(r, r.num_computed + n)
                else:
                    break
            r.blocks += self.allocator.allocate(need)
            chosen.append((r, n))
            budget -= n
            if n < remaining:
                break
            self.waiting.pop(0)
        self._align_step(chosen, n_decode)
        return chosen

    def _align_step(self, chosen, n_decode: int) -> None:
        """Trim the step's last prefill chunk so the step's token count (decode rows +
        prefill tokens) is a multiple of 256 when prompt work is left over anyway: the
        prefill GEMMs then run whole 256-row tiles, and hipBLASLt keeps its large-tile
        kernels (an M of 16384 + decode rows picked kernels ~25 % slower in the RAG bench).
        The trimmed tokens go first in the next step; nothing is trimmed when this step
        would drain the queue (that would cost a step)."""
        if not chosen:
            return
        T = n_decode + sum(n for _, n in chosen)
        cut = T % 256
        r, n = chosen[-1]
        more = bool(self.waiting)
        if T < 4096 or cut == 0 or n <= cut or not more:
            return
        chosen[-1] = (r, n - cut)
        if not self.waiting or self.waiting[0] is not r:
            self.waiting.insert(0, r)   # its last chunk no longer completes the prompt

    def _preempt_one(self, exclude: Optional[Request] = None) -> bool:
        for victim in reversed(self.running):
            if victim is exclude or victim.finished:
                continue
            self.running.remove(victim)
            self._free_blocks(victim)
            victim.num_computed = 0
            victim.pending_row = -1
            victim.pending_step = -1
            self.waiting.insert(0, victim)
            self.stats["preemptions"] += 1
            return True
        return False

    # ------------------------------------------------------------------ launch
    def _bucket(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        return self.buckets[-1]

    def _launch(self, decode: List[Request], chunks) -> _InFlight:
        nd = len(decode)
        npf = sum(n for _, n in chunks)
        T = nd + npf
        sample_reqs = list(decode) + [r for r, n in chunks if r.num_computed + n >= r.num_tokens]
        nrows = len(sample_reqs)
        n_top = min(max((r.params.logprobs for r in sample_reqs), default=0), 20)
        B = 0
        copies = self.prefix is not None and bool(self.prefix.copies)
        if npf == 0 and self.use_graphs and nd <= self.buckets[-1] and n_top == 0 and not copies:
            B = self._bucket(nd)
            if not self.exec.has_graph(B):
                self._flush()  # capture reuses the token-feedback buffer
                self.exec.capture(B)
        prev = self._inflight
        # free: the previous exec.step() waited for this slot's last upload
        self._slot = slot = (self._slot + 1) % NSLOTS
        a = self.exec.inputs[slot]
        ids, pos, slots = a["ids"], a["pos"], a["slots"]
        # ---- decode rows: one token each, input = previous sample (host or on-device feedback)
        ng = 0
        gdst, gsrc = a["gdst"], a["gsrc"]
        dbt, dctx = a["dbt"], a["dctx"]
        for j, r in enumerate(decode):
            p = r.num_computed
            if r.pending_row >= 0:
                assert prev is not None and r.pending_step == prev.step_id, "lost in-flight token"
                gdst[ng] = j
                gsrc[ng] = r.pending_row
                ng += 1
                ids[j] = 0
            else:
                ids[j] = r.token_at(p)
            pos[j] = p
            blk = r.blocks
            slots[j] = blk[p // BLOCK] * BLOCK + p % BLOCK
            dbt[j, : len(blk)] = blk
            dctx[j] = p + 1
        if B > nd:  # graph padding rows: no KV write, empty context, greedy
            ids[nd:B] = 0
            pos[nd:B] = 0
            slots[nd:B] = -1
            dctx[nd:B] = 0
        # ---- prefill chunks
        t = nd
        last_rows = []
        q_len, prefix = [], []
        pbt = a["pbt"]
        for k, (r, n) in enumerate(chunks):
            s = r.num_computed
            ids[t: t + n] = r.tokens(s, s + n)
            pp = np.arange(s, s + n, dtype=np.int64)
            pos[t: t + n] = pp
            blk = np.asarray(r.blocks, dtype=np.int64)
            slots[t: t + n] = blk[pp // BLOCK] * BLOCK + pp % BLOCK
            pbt[k, : len(blk)] = blk
            a["q_start"][k] = t
            a["ctx_len"][k] = s + n
            q_len.append(n)
            prefix.append(s)
            t += n
            if s + n >= r.num_tokens:
                last_rows.append(t - 1)
        ntiles = 0
        if chunks:
            a["q_len"][: len(chunks)] = q_len
            ntiles = ops.prefill_tiles_np(q_len, self._G, prefix, out=a["tiles"])
        rows_all = nrows == T
        if not rows_all:
            a["rows"][:nd] = np.arange(nd)
            a["rows"][nd:nrows] = last_rows
        # ---- sampling parameters (+ graph padding rows) and logit deltas
        nsr = max(nrows, B)
        temp, top_p, top_k, seeds, steps = a["temp"], a["top_p"], a["top_k"], a["seeds"], a["steps"]
        for j, r in enumerate(sample_reqs):
            p = r.params
            temp[j] = p.temperature
            top_p[j] = p.top_p
            top_k[j] = p.top_k
            seeds[j] = r.seed
            steps[j] = r.num_launched  # index of the token being sampled
        if nsr > nrows:
            temp[nrows:nsr] = 0.0
            top_p[nrows:nsr] = 1.0
            top_k[nrows:nsr] = 0
            seeds[nrows:nsr] = 0
            steps[nrows:nsr] = 0
        ndelta = self._write_deltas(a["deltas"], sample_reqs)
        # ---- header
        h = a["hdr"]
        h[:] = 0
        h[H_KIND] = KIND_STEP
        h[H_T] = T
        h[H_ND] = nd
        h[H_NPS] = len(chunks)
        h[H_NTILES] = ntiles
        h[H_NROWS] = nrows
        h[H_NGATHER] = ng
        h[H_NDELTA] = ndelta
        h[H_NTOP] = n_top
        h[H_BUCKET] = B
        h[H_ROWS_ALL] = 1 if rows_all else 0
        if self.prefix is not None and self.prefix.copies:
            assert B == 0, "KV block copies ride with eager (prefill) steps"
            cp = self.prefix.take_copies()
            a["kvcopy"][: len(cp)] = cp
            h[H_NCOPY] = len(cp)
            self.stats["prefix_hit_tokens"] = self.prefix.stats["hit_tokens"]
        # ---- advance host state (KV of these tokens is being written by this step)
        for r in decode:
            r.num_computed += 1
        for r, n in chunks:
            r.num_computed += n
            if r.num_computed >= r.num_tokens and r not in self.running:
                self.running.append(r)
        self._step_id += 1
        for j, r in enumerate(sample_reqs):
            r.num_launched += 1
            r.pending_row = j
            r.pending_step = self._step_id
        # ---- run
        t0 = time.perf_counter()
        # one GIL-released call: launch this step, wait for the previous step's results,
        # and for the next arena slot to be reusable
        self.exec.step(slot, prev.slot if prev is not None else -1, (slot + 1) % NSLOTS)
        if prev is not None:
            prev.ready = True
        self.stats["launch_ms"] += (time.perf_counter() - t0) * 1000
        if B:
            self.stats["decode_steps"] += 1
            self.stats["graph_steps"] += 1
        else:
            self.stats["mixed_steps" if nd and npf else ("prefill_steps" if npf else "decode_steps")] += 1
        self.stats["prefill_tokens"] += npf
        if npf:
            self.prefill_step_tokens.append(nd + npf)
        self.stats["decode_tokens"] += nd
        return _InFlight(sample_reqs, slot, n_top, self._step_id)

    def _write_deltas(self, out: np.ndarray, reqs: List[Request]) -> int:
        """(row, token, delta) triples: presence/frequency penalties, logit bias, and
        EOS suppression until min_tokens."""
        n = 0
        cap = out.shape[0]
        fview = out.view(np.float32)
        for j, r in enumerate(reqs):
            p = r.params
            items = []
            if p.needs_history:
                counts: Dict[int, int] = {}
                for t in r.output_ids:
                    counts[t] = counts.get(t, 0) + 1
                items += [(t, -(p.presence_penalty + p.frequency_penalty * c)) for t, c in counts.items()]
            if p.logit_bias:
                items += [(int(t), float(b)) for t, b in p.logit_bias.items()]
            if r.num_launched < p.min_tokens and not p.ignore_eos:
                items += [(t, -1e9) for t in self._eos_list]
            for t, d in items:
                if n >= cap:
                    log.warning("logit delta capacity (%d) exceeded; dropping the rest", cap)
                    return n
                out[n, 0] = j
                out[n, 1] = t
                fview[n, 2] = d
                n += 1
        return n

    # ------------------------------------------------------------------ retire
    def _retire(self, st: _InFlight) -> None:
        if not st.ready:
            t0 = time.perf_counter()
            self.exec.wait_out(st.slot)
            self.stats["wait_ms"] += (time.perf_counter() - t0) * 1000
        n = len(st.reqs)
        if n == 0:
            return
        o = self.exec.outputs[st.slot]
        tok_h = o["tok"][:n].tolist()
        lp_h = o["lp"][:n].tolist()
        ti_h = tl_h = None
        if st.n_top:
            ti_h = o["ti"][: n * st.n_top].reshape(n, st.n_top).tolist()
            tl_h = o["tl"][: n * st.n_top].reshape(n, st.n_top).tolist()
        now = time.perf_counter()
        for j, r in enumerate(st.reqs):
            if r.pending_step == st.step_id:
                r.pending_row = -1  # its newest token is on the host now
            if r.finished:
                continue  # a token launched after the request finished (lookahead) -> discard
            t = tok_h[j]
            r.output_ids.append(t)
            r.output_logprobs.append(lp_h[j])
            if r.first_token_time is None:
                r.first_token_time = now
                self.ttft_s.append(now - r.arrival)
            p = r.params
            reason = None
            if not p.ignore_eos and t in self._eos and len(r.output_ids) > p.min_tokens:
                reason = "stop"
            elif t in p.stop_token_ids:
                reason = "stop"
            elif len(r.output_ids) >= p.max_tokens:
                reason = "length"
            elif r.num_tokens >= self.max_model_len:
                reason = "length"
            delta = self._detok(r, t, final=reason is not None) if (r.callback is not None or p.stop) else ""
            if p.stop and reason is None:
                for s in p.stop:
                    k = r._text.find(s)
                    if k >= 0:
                        cut = len(r._text) - k
                        delta = delta[: max(0, len(delta) - cut)]
                        r._text = r._text[:k]
                        reason = "stop"
                        break
            top = list(zip(ti_h[j][: p.logprobs], tl_h[j][: p.logprobs])) if (ti_h is not None and p.logprobs) \
                else None
            if reason is not None:
                r.finished = True
                r.finish_reason = reason
                if self.tok is not None and r.callback is None and not p.stop:
                    r._text = self.tok.decode(r.output_ids)
            if r.callback is not None:
                try:
                    r.callback(TokenEvent(r.request_id, t, lp_h[j], delta, len(r.output_ids) - 1,
                                          reason is not None, reason, top))
                except Exception:  # noqa: BLE001
                    log.exception("token callback failed")
            if reason is not None:
                self._release(r)

    def _detok(self, r: Request, t: int, final: bool) -> str:
        if self.tok is None:
            return ""
        if self._tok_bytes is None:
            self._tok_bytes = [self.tok.decode_bytes([i]) for i in range(self.tok.vocab_size)]
        if 0 <= t < len(self._tok_bytes):
            r._emitted += self._tok_bytes[t]
        buf = bytes(r._emitted)
        try:
            s = buf.decode("utf-8")
            r._emitted.clear()
        except UnicodeDecodeError as e:
            if final or len(buf) - e.start > 3:
                s = buf.decode("utf-8", errors="replace")
                r._emitted.clear()
            else:
                s = buf[: e.start].decode("utf-8")
                del r._emitted[: e.start]
        r._text += s
        return s

    def _free_blocks(self, r: Request) -> None:
        """Return a request's own blocks; shared prefix blocks stay with their entry."""
        own = r.blocks[r.shared_blocks:]
        if own:
            self.allocator.free(own)
        if self.prefix is not None:
            self.prefix.release(r)
        r.blocks = []
        r.shared_blocks = 0

    def _release(self, r: Request) -> None:
        if r in self.running:
            self.running.remove(r)
        self._free_blocks(r)
        r.finish_time = time.perf_counter()
        self.stats["finished"] += 1
        r._done_event.set()

    def _finish(self, r: Request, reason: str) -> None:
        r.finished = True
        r.finish_reason = reason
        if r.callback is not None:
            try:
                r.callback(TokenEvent(r.request_id, -1, 0.0, "", len(r.output_ids), True, reason))
            except Exception:  # noqa: BLE001
                log.exception("token callback failed")
        if r in self.waiting:
            self.waiting.remove(r)
        self._release(r)
