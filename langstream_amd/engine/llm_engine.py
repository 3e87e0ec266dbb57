"""Continuous-batching LLM serving engine on MI355X.

Replaces the remote completion services the reference calls from
``ai-chat-completions`` / ``ai-text-completions`` (SURVEY §2.10 K2/K3;
``OpenAICompletionService.java:122-404``, ``OllamaProvider.java:273-311``) with a local
engine:

* paged KV cache (64-token blocks, V stored transposed; blocks managed by the native
  ``BlockAllocator``), sized from the 288 GB HBM budget;
* scheduler: FCFS admission, chunked prefill (``max_prefill_tokens`` per step) that
  packs many prompts into one varlen step, decode for every running sequence, and
  recompute-preemption when KV blocks run out;
* decode steps replayed from HIP graphs captured per batch-size bucket (one graph
  serves every context length: the split-KV grid is sized for ``max_model_len``);
* sampling on device (temperature / top-k / top-p / seed / penalties / logit-bias,
  log-probs of the sampled token + top-n alternatives for FLARE);
* streaming: a per-request callback receives every token, its log-prob and the text
  delta (the chunk coalescing of ``OpenAICompletionService.java:256-306`` is done by
  the agent on top of this);
* tensor parallel: rank 0 schedules and broadcasts each step's inputs over RCCL, all
  ranks run the sharded forward (all-reduce inside), rank 0 samples.
"""
from __future__ import annotations

import itertools
import logging
import math
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

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
    num_computed: int = 0        # tokens whose KV is in the cache
    finished: bool = False
    finish_reason: Optional[str] = None
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    _emitted_bytes: int = 0
    _text: str = ""
    _done_event: threading.Event = field(default_factory=threading.Event)
    seed: int = 0

    @property
    def all_ids(self) -> List[int]:
        return self.prompt_ids + self.output_ids

    @property
    def text(self) -> str:
        return self._text

    def wait(self, timeout: Optional[float] = None) -> bool:
        return self._done_event.wait(timeout)


class LLMEngine:
    def __init__(self, model: LlamaModel, tokenizer=None, *, num_blocks: Optional[int] = None,
                 kv_fraction: float = 0.55, max_model_len: int = 4096, max_batch: int = 256,
                 max_prefill_tokens: int = 8192, use_graphs: bool = True, graph_buckets: Sequence[int] = (),
                 device=None):
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
        D = self.cfg.head_dim
        hkv = model.hkv
        bytes_per_block = 2 * self.cfg.num_layers * hkv * BLOCK * D * 2
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
        self.num_blocks = num_blocks
        self.kv_caches = []
        for _ in range(self.cfg.num_layers):
            kc = torch.zeros(num_blocks, hkv, BLOCK, D, device=self.device, dtype=model.dtype)
            vc = torch.zeros(num_blocks, hkv, D, BLOCK, device=self.device, dtype=model.dtype)
            self.kv_caches.append((kc, vc))
        self.allocator = lib().BlockAllocator(num_blocks)
        self.nsplit, self.bps = ops.decode_splits(self.max_blocks_per_seq)
        self._ids = itertools.count(1)
        self._inbox: "queue.Queue[Request]" = queue.Queue()
        self.waiting: List[Request] = []
        self.running: List[Request] = []
        self._lock = threading.Lock()
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._wake = threading.Event()
        self.stats = {"prefill_steps": 0, "decode_steps": 0, "prefill_tokens": 0, "decode_tokens": 0,
                      "preemptions": 0, "requests": 0, "finished": 0}
        self.buckets = sorted(set(graph_buckets or [b for b in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192,
                                                                 224, 256, 320, 384, 448, 512) if b <= max_batch]
                                  + [max_batch]))
        self._graphs: Dict[int, dict] = {}
        self._eos = set(self.cfg.eos_token_ids)
        if tokenizer is not None and getattr(tokenizer, "eos_ids", None):
            self._eos |= set(tokenizer.eos_ids)

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
        return bool(self.waiting or self.running or not self._inbox.empty())

    # ------------------------------------------------------------------ loop
    def _loop(self) -> None:
        torch.cuda.set_device(self.device) if self.is_gpu else None
        while not self._stop.is_set():
            if not self.has_work():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                self.step()
            except Exception:  # noqa: BLE001
                log.exception("engine step failed; failing in-flight requests")
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
        self._drain_inbox()
        batch = self._schedule_prefill()
        if batch:
            self._run_prefill(batch)
            return
        if self.running:
            self._run_decode()

    # ------------------------------------------------------------------ scheduling
    def _blocks_needed(self, r: Request, upto: int) -> int:
        return max(0, (upto + BLOCK - 1) // BLOCK - len(r.blocks))

    def _schedule_prefill(self):
        """Pick (request, n_tokens) chunks to prefill this step.  Partially prefilled
        requests (chunked prefill) are continued first."""
        budget = self.max_prefill_tokens
        chosen = []
        # continue partially prefilled requests (kept at the head of `waiting`)
        while self.waiting and budget > 0 and len(self.running) + len(chosen) < self.max_batch:
            r = self.waiting[0]
            total = len(r.all_ids)
            remaining = total - r.num_computed
            n = min(remaining, budget)
            need = self._blocks_needed(r, r.num_computed + n)
            # keep headroom so running sequences can still grow by one block each
            headroom = len(self.running)
            if not self.allocator.can_allocate(need + headroom):
                if not chosen and not self.running:
                    # nothing else can make progress: shrink the chunk to what fits
                    fit = (self.allocator.num_free() + len(r.blocks)) * BLOCK - r.num_computed
                    if fit <= 0:
                        self._finish(self.waiting.pop(0), "length")  # prompt cannot fit at all
                        continue
                    n = min(n, fit)
                    need = self._blocks_needed(r, r.num_computed + n)
                else:
                    break
            r.blocks += self.allocator.allocate(need)
            chosen.append((r, n))
            budget -= n
            if n < remaining:
                break  # chunk boundary: this request continues next step
            self.waiting.pop(0)
        return chosen

    def _preempt_one(self) -> bool:
        if not self.running:
            return False
        victim = self.running.pop()  # most recently admitted
        self.allocator.free(victim.blocks)
        victim.blocks = []
        victim.num_computed = 0
        self.waiting.insert(0, victim)
        self.stats["preemptions"] += 1
        return True

    # ------------------------------------------------------------------ prefill
    def _run_prefill(self, batch) -> None:
        ids, pos, slots, q_start, q_len, ctx_len, last_idx, bt_rows = [], [], [], [], [], [], [], []
        prefix_lens = []
        t = 0
        for r, n in batch:
            all_ids = r.all_ids
            s = r.num_computed
            ids.extend(all_ids[s: s + n])
            pos.extend(range(s, s + n))
            for p in range(s, s + n):
                slots.append(r.blocks[p // BLOCK] * BLOCK + p % BLOCK)
            q_start.append(t)
            q_len.append(n)
            ctx_len.append(s + n)
            prefix_lens.append(s)
            t += n
            last_idx.append(t - 1)
            bt_rows.append(r.blocks)
        dev = self.device
        maxb = max(len(b) for b in bt_rows)
        bt = torch.zeros(len(batch), maxb, dtype=torch.int32)
        for i, b in enumerate(bt_rows):
            bt[i, : len(b)] = torch.tensor(b, dtype=torch.int32)
        G = self.model.hq // self.model.hkv
        host = {
            "ids": torch.tensor(ids, dtype=torch.int32), "pos": torch.tensor(pos, dtype=torch.int32),
            "slots": torch.tensor(slots, dtype=torch.int64), "bt": bt,
            "q_start": torch.tensor(q_start, dtype=torch.int32), "q_len": torch.tensor(q_len, dtype=torch.int32),
            "ctx_len": torch.tensor(ctx_len, dtype=torch.int32),
            "tiles": ops.prefill_tiles(q_len, G, prefix_lens),
            "last": torch.tensor(last_idx, dtype=torch.int64),
        }
        if self.tp.world > 1:
            self._tp_send_prefill(host)
        logits = self._prefill_forward(host)
        self.stats["prefill_steps"] += 1
        self.stats["prefill_tokens"] += t
        # advance state; sample for requests whose prompt is now fully cached
        done_rows, done_reqs = [], []
        for i, (r, n) in enumerate(batch):
            r.num_computed += n
            if r.num_computed >= len(r.all_ids):
                done_rows.append(i)
                done_reqs.append(r)
                if r not in self.running:
                    self.running.append(r)
        if done_rows:
            rows = torch.tensor(done_rows, device=logits.device, dtype=torch.long)
            self._sample_and_emit(logits.index_select(0, rows), done_reqs)

    def _prefill_forward(self, host: dict) -> torch.Tensor:
        dev = self.device
        d = {k: v.to(dev, non_blocking=True) for k, v in host.items()}
        meta = AttnMeta(is_prefill=True, positions=d["pos"], slots=d["slots"], block_tables=d["bt"],
                        q_start=d["q_start"], q_len=d["q_len"], ctx_len=d["ctx_len"], tiles=d["tiles"])
        hidden = self.model.forward(d["ids"], meta, self.kv_caches)
        return self.model.logits(hidden.index_select(0, d["last"]))

    # ------------------------------------------------------------------ decode
    def _bucket(self, n: int) -> int:
        if not self.use_graphs:
            return n
        for b in self.buckets:
            if b >= n:
                return b
        return self.buckets[-1]

    def _alloc_decode_buffers(self, B: int) -> dict:
        dev = self.device
        D = self.cfg.head_dim
        return {
            "ids": torch.zeros(B, dtype=torch.int32, device=dev),
            "pos": torch.zeros(B, dtype=torch.int32, device=dev),
            "slots": torch.full((B,), -1, dtype=torch.int64, device=dev),
            "bt": torch.zeros(B, self.max_blocks_per_seq, dtype=torch.int32, device=dev),
            "ctx": torch.zeros(B, dtype=torch.int32, device=dev),
            "ws": torch.empty(max(1, B * self.model.hq * self.nsplit * (D + 2)), dtype=torch.float32, device=dev),
        }

    def _decode_forward(self, buf: dict) -> torch.Tensor:
        meta = AttnMeta(is_prefill=False, positions=buf["pos"], slots=buf["slots"], block_tables=buf["bt"],
                        ctx_lens=buf["ctx"], nsplit=self.nsplit, blocks_per_split=self.bps, workspace=buf["ws"])
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
                # all ranks must capture the same bucket together
                self._tp_send_header(kind=4, n=b, t=0)
            self._get_graph(b)

    def _run_decode(self) -> None:
        # make sure every running sequence has room for one more token
        i = 0
        while i < len(self.running):
            r = self.running[i]
            need = self._blocks_needed(r, r.num_computed + 1)
            if need and not self.allocator.can_allocate(need):
                if not self._preempt_one():
                    break
                continue
            if need:
                r.blocks += self.allocator.allocate(need)
            i += 1
        reqs = self.running[: self.max_batch]
        if not reqs:
            return
        n = len(reqs)
        B = self._bucket(n)
        ids = torch.zeros(B, dtype=torch.int32)
        pos = torch.zeros(B, dtype=torch.int32)
        slots = torch.full((B,), -1, dtype=torch.int64)
        ctx = torch.zeros(B, dtype=torch.int32)
        bt = torch.zeros(B, self.max_blocks_per_seq, dtype=torch.int32)
        for j, r in enumerate(reqs):
            p = r.num_computed
            ids[j] = r.all_ids[p]
            pos[j] = p
            slots[j] = r.blocks[p // BLOCK] * BLOCK + p % BLOCK
            ctx[j] = p + 1
            bt[j, : len(r.blocks)] = torch.tensor(r.blocks, dtype=torch.int32)
        host = {"ids": ids, "pos": pos, "slots": slots, "ctx": ctx, "bt": bt}
        if self.tp.world > 1:
            self._tp_send_decode(B, host)
        logits = self._decode_run(B, host)
        for r in reqs:
            r.num_computed += 1
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += n
        self._sample_and_emit(logits[:n], reqs)

    def _decode_run(self, B: int, host: dict) -> torch.Tensor:
        g = self._get_graph(B)
        buf = g["buf"]
        for k in ("ids", "pos", "slots", "ctx", "bt"):
            buf[k].copy_(host[k], non_blocking=True)
        if g["graph"] is not None:
            g["graph"].replay()
            return g["out"]
        return self._decode_forward(buf)

    # ------------------------------------------------------------------ sampling
    def _sample_and_emit(self, logits: torch.Tensor, reqs: List[Request]) -> None:
        n = len(reqs)
        dev = logits.device
        ps = [r.params for r in reqs]
        # penalties / logit bias (sparse, only for rows that ask for them)
        rows, toks, deltas = [], [], []
        for j, r in enumerate(reqs):
            p = r.params
            if p.presence_penalty or p.frequency_penalty:
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
            if len(r.output_ids) < p.min_tokens and not p.ignore_eos:
                for t in self._eos:
                    rows.append(j)
                    toks.append(t)
                    deltas.append(-1e9)
        if rows:
            logits = logits.clone()
            ops.apply_logit_deltas(logits, torch.tensor(rows, dtype=torch.int32, device=dev),
                                   torch.tensor(toks, dtype=torch.int32, device=dev),
                                   torch.tensor(deltas, dtype=torch.float32, device=dev))
        temp = torch.tensor([p.temperature for p in ps], dtype=torch.float32)
        topk = torch.tensor([p.top_k for p in ps], dtype=torch.int32)
        topp = torch.tensor([p.top_p for p in ps], dtype=torch.float32)
        seeds = torch.tensor([r.seed for r in reqs], dtype=torch.int64)
        steps = torch.tensor([len(r.output_ids) for r in reqs], dtype=torch.int64)
        n_top = max(p.logprobs for p in ps)
        tok, lp, ti, tl = ops.sample(logits, temp.to(dev), topk.to(dev), topp.to(dev), seeds.to(dev),
                                     steps.to(dev), n_top=min(n_top, 20))
        tok_h = tok.cpu().tolist()
        lp_h = lp.cpu().tolist()
        ti_h = ti.cpu().tolist() if ti is not None else None
        tl_h = tl.cpu().tolist() if tl is not None else None
        now = time.perf_counter()
        for j, r in enumerate(reqs):
            t = tok_h[j]
            r.output_ids.append(t)
            r.output_logprobs.append(lp_h[j])
            if r.first_token_time is None:
                r.first_token_time = now
            reason = None
            p = r.params
            if not p.ignore_eos and t in self._eos and len(r.output_ids) > p.min_tokens:
                reason = "stop"
            elif t in p.stop_token_ids:
                reason = "stop"
            elif len(r.output_ids) >= p.max_tokens:
                reason = "length"
            elif len(r.all_ids) >= self.max_model_len:
                reason = "length"
            delta = self._detok(r, final=reason is not None)
            if p.stop and reason is None:
                for s in p.stop:
                    k = r._text.find(s)
                    if k >= 0:
                        cut = len(r._text) - k
                        delta = delta[: max(0, len(delta) - cut)]
                        r._text = r._text[:k]
                        reason = "stop"
                        break
            top = None
            if ti_h is not None and p.logprobs:
                top = list(zip(ti_h[j][: p.logprobs], tl_h[j][: p.logprobs]))
            if reason is not None:
                r.finished = True
                r.finish_reason = reason
            if r.callback is not None:
                try:
                    r.callback(TokenEvent(r.request_id, t, lp_h[j], delta, len(r.output_ids) - 1,
                                          reason is not None, reason, top))
                except Exception:  # noqa: BLE001
                    log.exception("token callback failed")
            if reason is not None:
                self._release(r)

    def _detok(self, r: Request, final: bool) -> str:
        if self.tok is None:
            return ""
        b = self.tok.decode_bytes(r.output_ids)
        new = b[r._emitted_bytes:]
        try:
            s = new.decode("utf-8")
        except UnicodeDecodeError:
            if not final:
                # hold back an incomplete multi-byte sequence
                for cut in range(1, 4):
                    try:
                        s = new[:-cut].decode("utf-8")
                        new = new[:-cut]
                        break
                    except UnicodeDecodeError:
                        continue
                else:
                    return ""
            else:
                s = new.decode("utf-8", errors="replace")
        r._emitted_bytes += len(new)
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
    # Rank 0 broadcasts a fixed 4-int header then the step's tensors; workers replay.
    def _tp_send_header(self, kind: int, n: int, t: int) -> None:
        h = torch.tensor([kind, n, t, 0], dtype=torch.int64, device=self.device)
        dist.broadcast(h, src=self._tp_src(), group=self.tp.group)

    def _tp_src(self) -> int:
        return dist.get_global_rank(self.tp.group, 0) if self.tp.group is not None else 0

    def _bcast(self, t: torch.Tensor) -> torch.Tensor:
        t = t.to(self.device)
        dist.broadcast(t, src=self._tp_src(), group=self.tp.group)
        return t

    def _tp_send_prefill(self, host: dict) -> None:
        T = host["ids"].numel()
        self._tp_send_header(1, host["q_len"].numel(), T)
        shape = torch.tensor([host["bt"].shape[1], host["tiles"].shape[0]], dtype=torch.int64)
        self._bcast(shape)
        for k in ("ids", "pos", "slots", "bt", "q_start", "q_len", "ctx_len", "tiles", "last"):
            self._bcast(host[k])

    def _tp_send_decode(self, B: int, host: dict) -> None:
        self._tp_send_header(2, B, 0)
        for k in ("ids", "pos", "slots", "ctx", "bt"):
            self._bcast(host[k])

    def worker_loop(self) -> None:
        """Non-zero TP ranks: mirror rank 0's steps until told to stop."""
        assert self.tp.world > 1 and self.tp.rank != 0
        dev = self.device
        while True:
            h = torch.empty(4, dtype=torch.int64, device=dev)
            dist.broadcast(h, src=self._tp_src(), group=self.tp.group)
            kind, n, t = (int(x) for x in h[:3].tolist())
            if kind == 3:
                return
            if kind == 4:
                self._get_graph(n)
                continue
            if kind == 1:
                shape = torch.empty(2, dtype=torch.int64, device=dev)
                dist.broadcast(shape, src=self._tp_src(), group=self.tp.group)
                maxb, ntiles = (int(x) for x in shape.tolist())
                spec = {"ids": (t, torch.int32), "pos": (t, torch.int32), "slots": (t, torch.int64),
                        "bt": ((n, maxb), torch.int32), "q_start": (n, torch.int32), "q_len": (n, torch.int32),
                        "ctx_len": (n, torch.int32), "tiles": ((ntiles, 2), torch.int32), "last": (n, torch.int64)}
                host = {}
                for k, (shp, dt) in spec.items():
                    x = torch.empty(shp, dtype=dt, device=dev)
                    dist.broadcast(x, src=self._tp_src(), group=self.tp.group)
                    host[k] = x
                self._prefill_forward(host)
            elif kind == 2:
                B = n
                spec = {"ids": (B, torch.int32), "pos": (B, torch.int32), "slots": (B, torch.int64),
                        "ctx": (B, torch.int32), "bt": ((B, self.max_blocks_per_seq), torch.int32)}
                host = {}
                for k, (shp, dt) in spec.items():
                    x = torch.empty(shp, dtype=dt, device=dev)
                    dist.broadcast(x, src=self._tp_src(), group=self.tp.group)
                    host[k] = x
                self._decode_run(B, host)
