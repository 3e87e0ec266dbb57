"""Llama-family decoder (Llama-3 8B / 70B and small test configs) on the HIP kernels.

This is the local replacement for the reference's remote chat/text completion
services (``ChatCompletionsStep.java:132-155`` ->
``OpenAICompletionService.java:122-311``).  Design, MI355X-first:

* weights packed for the GEMM shapes hipBLASLt likes: fused ``qkv`` [(Hq+2Hkv)*D, H],
  fused ``gate_up`` [2F, H]; bf16; sized per TP rank (column-parallel qkv/gate_up,
  row-parallel o/down, vocab-parallel embedding and LM head).
* one fused HIP kernel per elementwise stage: fused_add_rmsnorm (residual add + norm),
  rope_and_cache (RoPE + paged-KV write, V stored transposed), silu_and_mul.
* attention: MFMA paged prefill (varlen, causal, chunked-prefix) and paged decode
  (split-KV) kernels reading the engine's KV cache directly.
* TP: one process per GPU, RCCL all-reduce after o_proj and down_proj (2 per layer) and
  an all-gather of the vocab-sharded logits.  The all-reduce is on the torch.distributed
  process group so decode steps stay capturable in a HIP graph.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .. import ops
from ..ops import reference as ref


@dataclass
class LlamaConfig:
    name: str = "llama"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128009)

    @property
    def num_params(self) -> int:
        H, Fi, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        qkv = H * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
        o = self.num_heads * self.head_dim * H
        mlp = 3 * H * Fi
        return L * (qkv + o + mlp + 2 * H) + V * H * (1 if self.tie_embeddings else 2) + H

    def flops_per_token(self, ctx: int = 0) -> float:
        """Forward FLOPs per token (2 * matmul params + attention)."""
        H, Fi, L = self.hidden_size, self.intermediate_size, self.num_layers
        lin = 2 * L * (H * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
                       + self.num_heads * self.head_dim * H + 3 * H * Fi) + 2 * self.vocab_size * H
        attn = 4 * L * self.num_heads * self.head_dim * ctx
        return float(lin + attn)


PRESETS = {
    "llama-3-8b": LlamaConfig(name="llama-3-8b"),
    "llama-3.1-8b": LlamaConfig(name="llama-3.1-8b", max_position=131072,
                                rope_scaling={"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                                              "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}),
    "llama-3-70b": LlamaConfig(name="llama-3-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
                               num_heads=64, num_kv_heads=8),
    # small configs for tests / CPU plumbing (same code path, tiny shapes)
    "llama-tiny": LlamaConfig(name="llama-tiny", vocab_size=512, hidden_size=256, intermediate_size=512,
                              num_layers=2, num_heads=4, num_kv_heads=2, head_dim=64, max_position=2048,
                              bos_token_id=1, eos_token_ids=(2,)),
    "llama-small": LlamaConfig(name="llama-small", vocab_size=32000, hidden_size=1024, intermediate_size=2816,
                               num_layers=4, num_heads=8, num_kv_heads=2, head_dim=128, max_position=4096,
                               bos_token_id=1, eos_token_ids=(2,)),
}


@dataclass
class TPInfo:
    rank: int = 0
    world: int = 1
    group: Optional[object] = None
    force_pg: bool = False   # run the native TP path (collectives, vocab-parallel sampling) even at world 1

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather_last(self, t: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return t
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim=-1)


@dataclass
class AttnMeta:
    """Per-step attention metadata (device tensors).

    A step packs ``num_decode`` decode tokens (rows [0, num_decode), one per running
    sequence) followed by prefill chunks (rows [num_decode, T)); either part may be
    empty.  Decode rows use the paged decode kernel, prefill rows the paged prefill
    kernel (``q_start`` is the ABSOLUTE first row of each prefill sequence)."""
    positions: torch.Tensor                      # [T] int32
    slots: torch.Tensor                          # [T] int64
    num_decode: int = 0
    # decode part
    d_block_tables: Optional[torch.Tensor] = None  # [nd, max_blocks] int32
    d_ctx_lens: Optional[torch.Tensor] = None      # [nd] int32
    nsplit: int = 1
    blocks_per_split: int = 1 << 30
    workspace: Optional[torch.Tensor] = None
    # prefill part
    num_prefill_tokens: int = 0
    p_block_tables: Optional[torch.Tensor] = None  # [np, max_blocks] int32
    q_start: Optional[torch.Tensor] = None         # [np] int32 (absolute rows)
    q_len: Optional[torch.Tensor] = None           # [np] int32
    ctx_len: Optional[torch.Tensor] = None         # [np] int32
    tiles: Optional[torch.Tensor] = None           # [ntiles, 2] int32


_PGEMM = {"0": 0, "all": 2}.get(os.environ.get("LS_PGEMM", "1"), 1)
_PGEMM_MIN_T = int(os.environ.get("LS_PGEMM_MIN_T", "8192"))   # below: hipBLASLt + silu_and_mul is faster


def _pgemm(x: torch.Tensor, w: torch.Tensor, silu: bool) -> bool:
    """Prefill-sized rows on the GPU go to the 256x256-tile MFMA GEMM (same rule as
    runner.hip's pgemm())."""
    return (_PGEMM > (0 if silu else 1) and x.is_cuda and x.shape[0] >= _PGEMM_MIN_T and x.dtype == torch.bfloat16
            and x.stride(-1) == 1 and ops.hip().gemm_prefill_supported(w, silu))


def _linear(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    return ops.gemm_prefill(x, w) if _pgemm(x, w, False) else F.linear(x, w)


def tp_kv_heads(num_kv_heads: int, world: int) -> int:
    """KV heads per TP rank.  With more ranks than KV heads every KV head is REPLICATED on
    world / num_kv_heads consecutive ranks (each rank keeps the one KV head its query
    heads attend to), so e.g. an 8-KV-head model still shards over TP=16."""
    if num_kv_heads % world == 0:
        return num_kv_heads // world
    if world % num_kv_heads == 0:
        return 1
    raise ValueError(f"TP degree {world} must divide or be a multiple of the {num_kv_heads} KV heads")


class LlamaLayer:
    def __init__(self, cfg: LlamaConfig, tp: TPInfo, device, dtype):
        H, D = cfg.hidden_size, cfg.head_dim
        assert cfg.num_heads % tp.world == 0, "TP must divide the query heads"
        assert cfg.intermediate_size % tp.world == 0
        self.hq = cfg.num_heads // tp.world
        self.hkv = tp_kv_heads(cfg.num_kv_heads, tp.world)
        self.f = cfg.intermediate_size // tp.world
        std = 0.02
        mk = lambda *s: (torch.randn(*s, device=device, dtype=torch.float32) * std).to(dtype)  # noqa: E731
        self.qkv_w = mk((self.hq + 2 * self.hkv) * D, H)
        self.o_w = mk(H, self.hq * D) / math.sqrt(2 * cfg.num_layers)
        self.gate_up_w = mk(2 * self.f, H)
        self.down_w = mk(H, self.f) / math.sqrt(2 * cfg.num_layers)
        self.in_norm = torch.ones(H, device=device, dtype=dtype)
        self.post_norm = torch.ones(H, device=device, dtype=dtype)

    def tensors(self):
        return [self.qkv_w, self.o_w, self.gate_up_w, self.down_w, self.in_norm, self.post_norm]


class LlamaModel:
    """Random-init (or state-dict-loaded) Llama weights + forward over the paged KV cache."""

    def __init__(self, cfg: LlamaConfig, device="cuda", dtype=torch.bfloat16, tp: Optional[TPInfo] = None,
                 seed: int = 0):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPInfo()
        g = torch.random.fork_rng(devices=[self.device] if self.device.type == "cuda" else [])
        with g:
            torch.manual_seed(seed + 1000 * self.tp.rank)
            H = cfg.hidden_size
            assert cfg.vocab_size % self.tp.world == 0 or True
            self.vocab_per_rank = (cfg.vocab_size + self.tp.world - 1) // self.tp.world
            self.vocab_start = self.tp.rank * self.vocab_per_rank
            self.embed = (torch.randn(self.vocab_per_rank, H, device=self.device) * 0.02).to(dtype)
            self.layers = [LlamaLayer(cfg, self.tp, self.device, dtype) for _ in range(cfg.num_layers)]
            self.final_norm = torch.ones(H, device=self.device, dtype=dtype)
            self.lm_head = self.embed if cfg.tie_embeddings else (
                torch.randn(self.vocab_per_rank, H, device=self.device) * 0.02).to(dtype)
        self.hq = cfg.num_heads // self.tp.world
        self.hkv = tp_kv_heads(cfg.num_kv_heads, self.tp.world)
        self.cos_sin = ref.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, cfg.rope_scaling,
                                        device=self.device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)

    # ------------------------------------------------------------------ weights io
    def state_dict(self) -> dict:
        sd = {"embed": self.embed, "final_norm": self.final_norm, "lm_head": self.lm_head}
        for i, l in enumerate(self.layers):
            for n in ("qkv_w", "o_w", "gate_up_w", "down_w", "in_norm", "post_norm"):
                sd[f"layers.{i}.{n}"] = getattr(l, n)
        return sd

    def load_state_dict(self, sd: dict) -> None:
        """Load packed weights (our layout).  HF checkpoints are converted by
        ``models.loader.convert_hf_llama``."""
        self.embed.copy_(sd["embed"])
        self.final_norm.copy_(sd["final_norm"])
        if not self.cfg.tie_embeddings:
            self.lm_head.copy_(sd["lm_head"])
        for i, l in enumerate(self.layers):
            for n in ("qkv_w", "o_w", "gate_up_w", "down_w", "in_norm", "post_norm"):
                getattr(l, n).copy_(sd[f"layers.{i}.{n}"])

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        if self.tp.world == 1:
            return F.embedding(ids.long(), self.embed)
        local = ids.long() - self.vocab_start
        mask = (local < 0) | (local >= self.vocab_per_rank)
        h = F.embedding(local.clamp(0, self.vocab_per_rank - 1), self.embed)
        h = h.masked_fill(mask[:, None], 0)
        return self.tp.all_reduce(h)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv_caches: list) -> torch.Tensor:
        """Returns hidden states [T, H] after the final norm (all rows)."""
        cfg = self.cfg
        eps = cfg.rms_eps
        h = self.embed_tokens(ids)
        residual = h
        x = ops.rmsnorm(h, self.layers[0].in_norm, eps)
        D = cfg.head_dim
        for li, layer in enumerate(self.layers):
            kc, vc = kv_caches[li]
            qkv = _linear(x, layer.qkv_w)
            ops.rope_and_cache(qkv, meta.positions, self.cos_sin, meta.slots, kc, vc, self.hq, self.hkv)
            q = qkv[:, : self.hq * D]
            nd = meta.num_decode
            if meta.num_prefill_tokens == 0:
                attn = ops.paged_decode_attention(q, kc, vc, meta.d_block_tables, meta.d_ctx_lens, self.scale,
                                                  nsplit=meta.nsplit, blocks_per_split=meta.blocks_per_split,
                                                  workspace=meta.workspace)
            else:
                attn = torch.empty(q.shape[0], self.hq * D, dtype=q.dtype, device=q.device)
                if nd:
                    ops.paged_decode_attention(q[:nd], kc, vc, meta.d_block_tables, meta.d_ctx_lens, self.scale,
                                               out=attn[:nd], nsplit=meta.nsplit,
                                               blocks_per_split=meta.blocks_per_split, workspace=meta.workspace)
                ops.paged_prefill_attention(q, kc, vc, meta.p_block_tables, meta.q_start, meta.q_len, meta.ctx_len,
                                            meta.tiles, self.hq, self.scale, out=attn)
            o = _linear(attn, layer.o_w)
            self.tp.all_reduce(o)
            ops.fused_add_rmsnorm(o, residual, layer.post_norm, eps)
            if _pgemm(o, layer.gate_up_w, True):
                a = ops.gemm_prefill(o, layer.gate_up_w, silu=True)
            else:
                a = ops.silu_and_mul(F.linear(o, layer.gate_up_w))
            d = _linear(a, layer.down_w)
            self.tp.all_reduce(d)
            nxt = self.layers[li + 1].in_norm if li + 1 < len(self.layers) else self.final_norm
            ops.fused_add_rmsnorm(d, residual, nxt, eps)
            x = d
        return x

    def _native_runner(self, kv_caches: list):
        """The C++ step executor (``ops/csrc/runner.hip``), built once per KV-cache set.
        It issues the whole forward with the GIL released: a Python-driven forward
        re-acquires the GIL after every op and stalls behind busy agent threads."""
        key = id(kv_caches)
        r = getattr(self, "_runner", None)
        if r is not None and r[0] == key:
            return r[1]
        L = self.layers
        pg = None
        if self.tp.world > 1 or self.tp.force_pg:
            pg = self.tp.group if self.tp.group is not None else dist.group.WORLD
        runner = ops.hip().LlamaRunner(
            self.embed, [l.qkv_w for l in L], [l.o_w for l in L], [l.gate_up_w for l in L],
            [l.down_w for l in L], [l.in_norm for l in L], [l.post_norm for l in L], self.final_norm,
            self.lm_head, [kv[0] for kv in kv_caches], [kv[1] for kv in kv_caches], self.cos_sin, self.hq,
            self.hkv, self.cfg.head_dim, self.cfg.rms_eps, self.scale, self.cfg.vocab_size, self.vocab_start, pg)
        self._runner = (key, runner, kv_caches)
        return runner

    def forward_logits(self, ids: torch.Tensor, meta: AttnMeta, kv_caches: list,
                       rows: Optional[torch.Tensor] = None, local: bool = False) -> torch.Tensor:
        """Forward + LM head for ``rows`` (all rows if None) -> f32 [N, V].  On the GPU
        the native executor runs it; elsewhere the Python path (same math).  local: see
        ``logits`` (the Python path only; the native executor samples vocab-parallel itself)."""
        if self.device.type == "cuda" and ops.hip_available():
            ws = meta.workspace
            bps = meta.blocks_per_split
            if meta.num_decode:
                bps = min(bps, meta.d_block_tables.shape[1])
                if meta.nsplit > 1:
                    need = meta.num_decode * self.hq * meta.nsplit * (self.cfg.head_dim + 2)
                    assert ws is not None and ws.numel() >= need, "decode workspace too small"
            return self._native_runner(kv_caches).forward(
                ids, meta.positions, meta.slots, meta.num_decode, meta.d_block_tables, meta.d_ctx_lens,
                meta.nsplit, bps, ws, meta.num_prefill_tokens, meta.p_block_tables, meta.q_start, meta.q_len,
                meta.ctx_len, meta.tiles, rows)
        hidden = self.forward(ids, meta, kv_caches)
        if rows is not None:
            hidden = hidden.index_select(0, rows)
        return self.logits(hidden, local=local)

    def local_vocab(self) -> int:
        """Valid vocabulary entries of this rank's LM-head slice."""
        return max(0, min(self.vocab_per_rank, self.cfg.vocab_size - self.vocab_start))

    def logits(self, hidden: torch.Tensor, local: bool = False) -> torch.Tensor:
        """[N, H] -> f32 [N, V] (vocab-parallel matmul + all-gather under TP).  local=True
        under TP: this rank's [N, local_vocab()] slice (ops.sample_vocab_parallel)."""
        if hidden.is_cuda and hidden.dtype != torch.float32:
            # f32 output from the GEMM itself (same as the native runner's LM head)
            lg = torch.mm(hidden, self.lm_head.t(), out_dtype=torch.float32)
        else:
            lg = F.linear(hidden, self.lm_head).float()
        if self.tp.world > 1:
            if local:
                return lg[:, : self.local_vocab()]
            lg = self.tp.all_gather_last(lg)
        return lg[:, : self.cfg.vocab_size]
