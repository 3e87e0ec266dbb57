"""Continuous-batching LLM serving engine on MI355X.

Replaces the remote completion services the reference calls from
``ai-chat-completions`` / ``ai-text-completions`` (SURVEY §2.10 K2/K3;
``OpenAICompletionService.java:122-404``, ``OllamaProvider.java:273-311``) with a local
engine:

* paged KV cache (64-token blocks, V stored transposed; blocks managed by the native
  ``BlockAllocator``), sized from the 288 GB HBM budget;
* unified steps: every step carries one decode token per running sequence plus, when
  prompts are waiting, chunked-prefill tokens (``max_prefill_tokens`` per step), so new
  requests never stall the sequences already decoding;
* pure-decode steps replay a HIP graph captured per batch-size bucket (one graph serves
  every context length: the split-KV grid is sized for ``max_model_len``); mixed steps
  run eagerly;
* one-step lookahead: the next step's input tokens are gathered ON DEVICE from the
  previous step's sampled tokens, so step N+1 is launched before step N's tokens are
  copied back -- host bookkeeping (detokenisation, streaming callbacks, scheduling)
  overlaps the GPU instead of idling it.  Finishing is detected one step late; that
  step's extra token is discarded;
* sampling on device (temperature / top-k / top-p / seed / penalties / logit-bias,
  log-probs of the sampled token + top-n alternatives for FLARE);
* recompute-preemption when KV blocks run out;
* tensor parallel: rank 0 schedules and broadcasts each step over RCCL, all ranks run
  the sharded forward (all-reduce inside), rank 0 samples.
"""
from __future__ import annotations

import itertools
import os
import logging
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .. import ops
from ..models.llama import AttnMeta, LlamaModel
from ..native import lib

log = logging.getLogger(__name__)
BLOCK = ops.KV_BLOCK


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
    tok: torch.Tensor            # device int32 [n]
    lp: torch.Tensor             # device f32 [n]
    top_ids: Optional[torch.Tensor]
    top_lps: Optional[torch.Tensor]
    host_tok: torch.Tensor       # pinned copies
    host_lp: torch.Tensor
    host_ti: Optional[torch.Tensor]
    host_tl: Optional[torch.Tensor]
    event: Optional[object]
    step_id: int = 0


class LLMEngine:
    def __init__(self, model: LlamaModel, tokenizer=None, *, num_blocks: Optional[int] = None,
                 kv_fraction: float = 0.55, max_model_len: int = 4096, max_batch: int = 256,
                 max_prefill_tokens: int = 8192, use_graphs: bool = True, graph_buckets: Sequence[int] = (),
                 lookahead: bool = True, device=None):
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
            kc = torch.zeros(self.num_blocks, hkv, BLOCK, D, device=self.device, dtype=model.dtype)
            vc = torch.zeros(self.num_blocks, hkv, D, BLOCK, device=self.device, dtype=model.dtype)
            self.kv_caches.append((kc, vc))
        self.allocator = lib().BlockAllocator(self.num_blocks)
        self.nsplit, self.bps = ops.decode_splits(self.max_blocks_per_seq)
        self._ids = itertools.count(1)
        self._inbox: "queue.Queue[Request]" = queue.Queue()
        self.waiting: List[Request] = []
        self.running: List[Request] = []
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._wake = threading.Event()
        self._inflight: Optional[_InFlight] = None
        self._step_id = 0
        self.stats = {"prefill_steps": 0, "decode_steps": 0, "mixed_steps": 0, "prefill_tokens": 0,
                      "decode_tokens": 0, "preemptions": 0, "requests": 0, "finished": 0, "graph_steps": 0,
                      "host_ms": 0.0, "wait_ms": 0.0}
        self.buckets = sorted(set(graph_buckets or [b for b in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192,
                                                                 224, 256, 320, 384, 448, 512) if b <= max_batch]
                                  + [max_batch]))
        self._graphs: Dict[int, dict] = {}
        self._eos = set(self.cfg.eos_token_ids)
        if tokenizer is not None and getattr(tokenizer, "eos_ids", None):
            self._eos |= set(tokenizer.eos_ids)
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
            self._tp_send_header(kind=3, n=0, t=0)  # tell workers to exit

    def has_work(self) -> bool:
        return bool(self.waiting or self.running or not self._inbox.empty() or self._inflight is not None)

    # ------------------------------------------------------------------ loop
    def _loop(self) -> None:
        import sys
        # the engine thread shares the GIL with agent threads: a short switch interval
        # bounds how long host bookkeeping elsewhere can delay the next GPU launch
        sys.setswitchinterval(min(sys.getswitchinterval(), 0.001))
        if self.is_gpu:
            torch.cuda.set_device(self.device)
        prof_path = os.environ.get("LANGSTREAM_PROFILE_ENGINE")
        if prof_path:
            import cProfile
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            try:
                self._loop_body()
            finally:
                pr.disable()
                with open(prof_path, "w") as f:
                    pstats.Stats(pr, stream=f).sort_stats("cumulative").print_stats(60)
            return
        self._loop_body()

    def _loop_body(self) -> None:
        while not self._stop.is_set():
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
            self.stats["requests"] += 1

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
        launched = self._launch(decode, chunks)
        prev, self._inflight = self._inflight, launched
        self.stats["host_ms"] += (time.perf_counter() - t0) * 1000
        if prev is not None:
            self._retire(prev)
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
        if need > self.allocator.num_free():
            self._flush()  # exact host state before preempting
            cands = self._decode_candidates()[: self.max_batch]
            need = sum(self._blocks_needed(r, r.num_computed + 1) for r in cands)
            while need > self.allocator.num_free() and len(cands) > 1 and self._preempt_one():
                cands = self._decode_candidates()[: self.max_batch]
                need = sum(self._blocks_needed(r, r.num_computed + 1) for r in cands)
        out: List[Request] = []
        for r in cands:
            n = self._blocks_needed(r, r.num_computed + 1)
            if n:
                if not self.allocator.can_allocate(n):
                    continue
                r.blocks += self.allocator.allocate(n)
            out.append(r)
        return out

    def _schedule_prefill(self, n_decode: int):
        budget = self.max_prefill_tokens
        chosen = []
        while self.waiting and budget > 0 and len(self.running) + len(chosen) < self.max_batch:
            r = self.waiting[0]
            if r.finished:
                self.waiting.pop(0)
                continue
            total = len(r.all_ids)
            remaining = total - r.num_computed
            n = min(remaining, budget)
            need = self._blocks_needed(r, r.num_computed + n)
            headroom = n_decode  # let every decoding sequence grow by one more block
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
        return chosen

    def _preempt_one(self, exclude: Optional[Request] = None) -> bool:
        for victim in reversed(self.running):
            if victim is exclude or victim.finished:
                continue
            self.running.remove(victim)
            self.allocator.free(victim.blocks)
            victim.blocks = []
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
        prev = self._inflight
        # ---- decode rows (host arrays)
        ids_np = np.zeros(nd + npf, dtype=np.int32)
        pos_np = np.zeros(nd + npf, dtype=np.int32)
        slot_np = np.full(nd + npf, -1, dtype=np.int64)
        gather_dst, gather_src = [], []
        for j, r in enumerate(decode):
            p = r.num_computed
            if r.pending_row >= 0:
                assert prev is not None and r.pending_step == prev.step_id, "lost in-flight token"
                gather_dst.append(j)
                gather_src.append(r.pending_row)
            else:
                ids_np[j] = r.all_ids[p]
            pos_np[j] = p
            slot_np[j] = r.blocks[p // BLOCK] * BLOCK + p % BLOCK
        # ---- prefill rows
        sample_reqs = list(decode)
        last_rows = []
        q_start, q_len, ctx_len, prefix = [], [], [], []
        t = nd
        for r, n in chunks:
            s = r.num_computed
            ids = r.all_ids[s: s + n]
            ids_np[t: t + n] = ids
            pos_np[t: t + n] = np.arange(s, s + n, dtype=np.int32)
            blk = np.asarray(r.blocks, dtype=np.int64)
            pp = np.arange(s, s + n)
            slot_np[t: t + n] = blk[pp // BLOCK] * BLOCK + pp % BLOCK
            q_start.append(t)
            q_len.append(n)
            ctx_len.append(s + n)
            prefix.append(s)
            t += n
            if s + n >= len(r.all_ids):
                last_rows.append(t - 1)
                sample_reqs.append(r)
        maxb = self.max_blocks_per_seq
        host = {"ids": ids_np, "pos": pos_np, "slots": slot_np}
        if nd:
            dbt = np.zeros((nd, maxb), dtype=np.int32)
            ctx = np.zeros(nd, dtype=np.int32)
            for j, r in enumerate(decode):
                dbt[j, : len(r.blocks)] = r.blocks
                ctx[j] = r.num_computed + 1
            host["dbt"], host["ctx"] = dbt, ctx
        if chunks:
            pbt = np.zeros((len(chunks), max(len(r.blocks) for r, _ in chunks)), dtype=np.int32)
            for j, (r, _) in enumerate(chunks):
                pbt[j, : len(r.blocks)] = r.blocks
            host.update(pbt=pbt, q_start=np.asarray(q_start, np.int32), q_len=np.asarray(q_len, np.int32),
                        ctx_len=np.asarray(ctx_len, np.int32),
                        tiles=ops.prefill_tiles(q_len, self.model.hq // self.model.hkv, prefix).numpy())
        # ---- advance host state (KV of these tokens is being written by this step)
        for r in decode:
            r.num_computed += 1
        for r, n in chunks:
            r.num_computed += n
            if r.num_computed >= len(r.all_ids) and r not in self.running:
                self.running.append(r)
        for r in sample_reqs:
            r.num_launched += 1
        gd = torch.tensor(gather_dst, dtype=torch.long) if gather_dst else None
        gs = torch.tensor(gather_src, dtype=torch.long) if gather_src else None
        # ---- run
        if npf == 0 and self.use_graphs and nd <= self.buckets[-1]:
            logits = self._decode_graph(nd, host, gd, gs, prev)
            self.stats["decode_steps"] += 1
            self.stats["graph_steps"] += 1
        else:
            logits = self._forward_eager(host, nd, npf, last_rows, gd, gs, prev)
            self.stats["mixed_steps" if nd else "prefill_steps"] += 1
        self.stats["prefill_tokens"] += npf
        self.stats["decode_tokens"] += nd
        self._step_id += 1
        if not sample_reqs:
            e = torch.empty(0, dtype=torch.int32)
            return _InFlight([], e, e, None, None, e, e, None, None, None, self._step_id)
        for j, r in enumerate(sample_reqs):
            r.pending_row = j
            r.pending_step = self._step_id
        st = self._sample(logits, sample_reqs)
        st.step_id = self._step_id
        return st

    def _ids_with_gather(self, ids_dev: torch.Tensor, gd, gs, prev) -> None:
        if gd is not None:
            ids_dev[gd.to(self.device, non_blocking=True)] = prev.tok[gs.to(self.device, non_blocking=True)]

    def _forward_eager(self, host, nd, npf, last_rows, gd, gs, prev) -> torch.Tensor:
        dev = self.device
        d = {k: torch.from_numpy(v).to(dev, non_blocking=True) for k, v in host.items()}
        self._ids_with_gather(d["ids"], gd, gs, prev)
        if self.tp.world > 1:
            self._tp_send_step(dict(host, last=np.asarray(last_rows, np.int64)), d["ids"])
        return self._eager_core(d, nd, npf, last_rows)

    def _eager_core(self, d, nd, npf, last_rows) -> torch.Tensor:
        D = self.cfg.head_dim
        ws = None
        if nd:
            ws = torch.empty(max(1, nd * self.model.hq * self.nsplit * (D + 2)), dtype=torch.float32,
                             device=self.device)
        meta = AttnMeta(positions=d["pos"], slots=d["slots"], num_decode=nd,
                        d_block_tables=d.get("dbt"), d_ctx_lens=d.get("ctx"), nsplit=self.nsplit,
                        blocks_per_split=self.bps, workspace=ws, num_prefill_tokens=npf,
                        p_block_tables=d.get("pbt"), q_start=d.get("q_start"), q_len=d.get("q_len"),
                        ctx_len=d.get("ctx_len"), tiles=d.get("tiles"))
        hidden = self.model.forward(d["ids"], meta, self.kv_caches)
        rows = list(range(nd)) + list(last_rows)
        if len(rows) == hidden.shape[0]:
            sel = hidden
        else:
            sel = hidden.index_select(0, torch.tensor(rows, dtype=torch.long).to(self.device, non_blocking=True))
        return self.model.logits(sel)

    # -- graphs
    def _alloc_decode_buffers(self, B: int) -> dict:
        dev = self.device
        D = self.cfg.head_dim
        return {
            "ids": torch.zeros(B, dtype=torch.int32, device=dev),
            "pos": torch.zeros(B, dtype=torch.int32, device=dev),
            "slots": torch.full((B,), -1, dtype=torch.int64, device=dev),
            "dbt": torch.zeros(B, self.max_blocks_per_seq, dtype=torch.int32, device=dev),
            "ctx": torch.zeros(B, dtype=torch.int32, device=dev),
            "ws": torch.empty(max(1, B * self.model.hq * self.nsplit * (D + 2)), dtype=torch.float32, device=dev),
        }

    def _decode_forward(self, buf: dict) -> torch.Tensor:
        meta = AttnMeta(positions=buf["pos"], slots=buf["slots"], num_decode=buf["ids"].shape[0],
                        d_block_tables=buf["dbt"], d_ctx_lens=buf["ctx"], nsplit=self.nsplit,
                        blocks_per_split=self.bps, workspace=buf["ws"])
        hidden = self.model.forward(buf["ids"], meta, self.kv_caches)
        return self.model.logits(hidden)

    def _get_graph(self, B: int) -> dict:
        g = self._graphs.get(B)
        if g is not None:
            return g
        buf = self._alloc_decode_buffers(B)
        g = {"buf": buf, "graph": None, "out": None}
        if self.use_graphs:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up (allocator, hipBLASLt heuristics)
                    self._decode_forward(buf)
            torch.cuda.current_stream(self.device).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, pool=self._graph_pool()):
                out = self._decode_forward(buf)
            g["graph"], g["out"] = graph, out
        self._graphs[B] = g
        return g

    def _graph_pool(self):
        if not hasattr(self, "_pool"):
            self._pool = torch.cuda.graph_pool_handle()
        return self._pool

    def capture_graphs(self, sizes: Optional[Sequence[int]] = None) -> None:
        for b in sizes or self.buckets:
            if self.tp.world > 1:
                self._tp_send_header(kind=4, n=b, t=0)  # every rank captures the same bucket together
            self._get_graph(b)

    def _decode_graph(self, nd: int, host, gd, gs, prev) -> torch.Tensor:
        B = self._bucket(nd)
        g = self._get_graph(B)
        buf = g["buf"]
        pad = B - nd
        ids = host["ids"]
        pos, slots, ctx, dbt = host["pos"], host["slots"], host["ctx"], host["dbt"]
        if pad:
            ids = np.concatenate([ids, np.zeros(pad, np.int32)])
            pos = np.concatenate([pos, np.zeros(pad, np.int32)])
            slots = np.concatenate([slots, np.full(pad, -1, np.int64)])
            ctx = np.concatenate([ctx, np.zeros(pad, np.int32)])
            dbt = np.concatenate([dbt, np.zeros((pad, dbt.shape[1]), np.int32)])
        buf["ids"].copy_(torch.from_numpy(ids), non_blocking=True)
        buf["pos"].copy_(torch.from_numpy(pos), non_blocking=True)
        buf["slots"].copy_(torch.from_numpy(slots), non_blocking=True)
        buf["ctx"].copy_(torch.from_numpy(ctx), non_blocking=True)
        buf["dbt"].copy_(torch.from_numpy(dbt), non_blocking=True)
        self._ids_with_gather(buf["ids"], gd, gs, prev)
        if self.tp.world > 1:
            self._tp_send_decode(B, buf)
        if g["graph"] is not None:
            g["graph"].replay()
            return g["out"][:nd]
        return self._decode_forward(buf)[:nd]

    # ------------------------------------------------------------------ sampling / retire
    def _sample(self, logits: torch.Tensor, reqs: List[Request]) -> _InFlight:
        n = len(reqs)
        dev = logits.device
        rows, toks, deltas = [], [], []
        for j, r in enumerate(reqs):
            p = r.params
            if p.needs_history:
                counts: Dict[int, int] = {}
                for t in r.output_ids:
                    counts[t] = counts.get(t, 0) + 1
                for t, c in counts.items():
                    rows.append(j)
                    toks.append(t)
                    deltas.append(-(p.presence_penalty + p.frequency_penalty * c))
            if p.logit_bias:
                for t, b in p.logit_bias.items():
                    rows.append(j)
                    toks.append(int(t))
                    deltas.append(float(b))
            if r.num_launched - 1 < p.min_tokens and not p.ignore_eos:
                for t in self._eos:
                    rows.append(j)
                    toks.append(t)
                    deltas.append(-1e9)
        if rows:
            logits = logits.clone()
            ops.apply_logit_deltas(logits, torch.tensor(rows, dtype=torch.int32).to(dev),
                                   torch.tensor(toks, dtype=torch.int32).to(dev),
                                   torch.tensor(deltas, dtype=torch.float32).to(dev))
        params = np.empty((n, 3), dtype=np.float32)
        ints = np.empty((n, 3), dtype=np.int64)
        for j, r in enumerate(reqs):
            p = r.params
            params[j] = (p.temperature, p.top_p, 0.0)
            ints[j] = (p.top_k, r.seed, r.num_launched - 1)
        pd = torch.from_numpy(params).to(dev, non_blocking=True)
        idv = torch.from_numpy(ints).to(dev, non_blocking=True)
        n_top = min(max(r.params.logprobs for r in reqs), 20)
        tok, lp, ti, tl = ops.sample(logits, pd[:, 0].contiguous(), idv[:, 0].to(torch.int32), pd[:, 1].contiguous(),
                                     idv[:, 1].contiguous(), idv[:, 2].contiguous(), n_top=n_top)
        if self.is_gpu:
            ht = torch.empty(n, dtype=torch.int32, pin_memory=True)
            hl = torch.empty(n, dtype=torch.float32, pin_memory=True)
            ht.copy_(tok, non_blocking=True)
            hl.copy_(lp, non_blocking=True)
            hti = htl = None
            if ti is not None:
                hti = torch.empty(ti.shape, dtype=torch.int32, pin_memory=True)
                htl = torch.empty(tl.shape, dtype=torch.float32, pin_memory=True)
                hti.copy_(ti, non_blocking=True)
                htl.copy_(tl, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            ht, hl, hti, htl, ev = tok, lp, ti, tl, None
        return _InFlight(reqs, tok, lp, ti, tl, ht, hl, hti, htl, ev)

    def _retire(self, st: _InFlight) -> None:
        t0 = time.perf_counter()
        if st.event is not None:
            st.event.synchronize()
        self.stats["wait_ms"] += (time.perf_counter() - t0) * 1000
        tok_h = st.host_tok.tolist()
        lp_h = st.host_lp.tolist()
        ti_h = st.host_ti.tolist() if st.host_ti is not None else None
        tl_h = st.host_tl.tolist() if st.host_tl is not None else None
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
            p = r.params
            reason = None
            if not p.ignore_eos and t in self._eos and len(r.output_ids) > p.min_tokens:
                reason = "stop"
            elif t in p.stop_token_ids:
                reason = "stop"
            elif len(r.output_ids) >= p.max_tokens:
                reason = "length"
            elif len(r.all_ids) >= self.max_model_len:
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

    def _release(self, r: Request) -> None:
        if r in self.running:
            self.running.remove(r)
        if r.blocks:
            self.allocator.free(r.blocks)
            r.blocks = []
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

    # ------------------------------------------------------------------ tensor parallel plumbing
    # Rank 0 broadcasts a fixed 4-int header then the step's tensors; workers mirror it.
    def _tp_send_header(self, kind: int, n: int, t: int, extra: int = 0) -> None:
        h = torch.tensor([kind, n, t, extra], dtype=torch.int64, device=self.device)
        dist.broadcast(h, src=self._tp_src(), group=self.tp.group)

    def _tp_src(self) -> int:
        return dist.get_global_rank(self.tp.group, 0) if self.tp.group is not None else 0

    def _bcast(self, t: torch.Tensor) -> None:
        dist.broadcast(t, src=self._tp_src(), group=self.tp.group)

    _STEP_KEYS = ("pos", "slots", "dbt", "ctx", "pbt", "q_start", "q_len", "ctx_len", "tiles", "last")

    def _tp_send_step(self, host: dict, ids_dev: torch.Tensor) -> None:
        nd = host["dbt"].shape[0] if "dbt" in host else 0
        T = host["ids"].shape[0]
        self._tp_send_header(1, nd, T)
        shapes = []
        for k in self._STEP_KEYS:
            a = host.get(k)
            shapes += list(a.shape) + [0] * (2 - a.ndim) if a is not None else [-1, -1]
        self._bcast(torch.tensor(shapes, dtype=torch.int64, device=self.device))
        self._bcast(ids_dev)
        for k in self._STEP_KEYS:
            if host.get(k) is not None:
                self._bcast(torch.from_numpy(np.ascontiguousarray(host[k])).to(self.device))

    def _tp_send_decode(self, B: int, buf: dict) -> None:
        self._tp_send_header(2, B, 0)
        for k in ("ids", "pos", "slots", "ctx", "dbt"):
            self._bcast(buf[k])

    def worker_loop(self) -> None:
        """Non-zero TP ranks: mirror rank 0's steps until told to stop."""
        assert self.tp.world > 1 and self.tp.rank != 0
        dev = self.device
        dtypes = {"pos": torch.int32, "slots": torch.int64, "dbt": torch.int32, "ctx": torch.int32,
                  "pbt": torch.int32, "q_start": torch.int32, "q_len": torch.int32, "ctx_len": torch.int32,
                  "tiles": torch.int32, "last": torch.int64}
        while True:
            h = torch.empty(4, dtype=torch.int64, device=dev)
            self._bcast(h)
            kind, n, t, _ = (int(x) for x in h.tolist())
            if kind == 3:
                return
            if kind == 4:
                self._get_graph(n)
                continue
            if kind == 1:
                shp = torch.empty(2 * len(self._STEP_KEYS), dtype=torch.int64, device=dev)
                self._bcast(shp)
                shp = shp.tolist()
                ids = torch.empty(t, dtype=torch.int32, device=dev)
                self._bcast(ids)
                d = {"ids": ids}
                for i, k in enumerate(self._STEP_KEYS):
                    a, b = shp[2 * i], shp[2 * i + 1]
                    if a < 0:
                        continue
                    x = torch.empty((a, b) if b else (a,), dtype=dtypes[k], device=dev)
                    self._bcast(x)
                    d[k] = x
                npf = t - n
                last_rows = d.pop("last").tolist() if "last" in d else []
                self._eager_core(d, n, npf, last_rows)
            elif kind == 2:
                g = self._get_graph(n)
                buf = g["buf"]
                for k in ("ids", "pos", "slots", "ctx", "dbt"):
                    self._bcast(buf[k])
                if g["graph"] is not None:
                    g["graph"].replay()
                else:
                    self._decode_forward(buf)
