"""BERT-family sentence encoder (bge-small-en / multilingual-e5-small / MiniLM shapes).

Local replacement for the reference's DJL + libtorch-CPU embedding path
(``AbstractHuggingFaceEmbeddingService.java:42-224``, which predicts one text at a
time -- comment at :192-193) and for the remote embedding services.

Padding-free: a batch is packed into one [T, H] token matrix with per-sequence
start/len; attention is the varlen MFMA encoder kernel, so no FLOPs are spent on pad
tokens.

Fused path (default; ops/csrc/gemm_fused.hip): per layer FOUR hand-written MFMA GEMMs +
the attention kernel and nothing else -- every bias, the erf-GELU, both residual adds
and both LayerNorms live in GEMM epilogues.  A GEMM that feeds a LayerNorm stores the
un-normalised row and per-row partial statistics; the next GEMM applies the LayerNorm
algebraically (input side: LN(x).W^T = r (x.W'^T) - r mu c1 + c2 with W' = W*gamma,
c1 = rowsum(W'), c2 = W.beta precomputed here; residual side: elementwise).  Only the
last layer's LayerNorm runs as a kernel, before CLS/mean pooling + L2 normalise.
Unfused path (LS_BERT_FUSED=0 or unsupported widths): library GEMMs + the bias/GELU and
bias+residual+LayerNorm kernels.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.nn.functional as F

from .. import ops


@dataclass
class BertConfig:
    name: str = "bge-small-en"
    vocab_size: int = 30522
    hidden_size: int = 384
    num_layers: int = 12
    num_heads: int = 12
    intermediate_size: int = 1536
    max_position: int = 512
    type_vocab_size: int = 2
    ln_eps: float = 1e-12
    pooling: str = "cls"          # "cls" (bge) | "mean" (e5, sentence-transformers)
    normalize: bool = True

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads


PRESETS = {
    "bge-small-en": BertConfig(),
    "bge-small-en-v1.5": BertConfig(name="bge-small-en-v1.5"),
    "multilingual-e5-small": BertConfig(name="multilingual-e5-small", vocab_size=250037, pooling="mean"),
    "all-MiniLM-L6-v2": BertConfig(name="all-MiniLM-L6-v2", num_layers=6, pooling="mean"),
    "bge-base-en": BertConfig(name="bge-base-en", hidden_size=768, num_heads=12, intermediate_size=3072),
    "bert-tiny": BertConfig(name="bert-tiny", vocab_size=30522, hidden_size=128, num_layers=2, num_heads=4,
                            intermediate_size=512),
}


class BertLayer:
    def __init__(self, cfg: BertConfig, device, dtype):
        H, Fi = cfg.hidden_size, cfg.intermediate_size
        mk = lambda *s: (torch.randn(*s, device=device) * 0.02).to(dtype)  # noqa: E731
        z = lambda n: torch.zeros(n, device=device, dtype=dtype)  # noqa: E731
        o = lambda n: torch.ones(n, device=device, dtype=dtype)  # noqa: E731
        self.qkv_w, self.qkv_b = mk(3 * H, H), z(3 * H)
        self.o_w, self.o_b = mk(H, H), z(H)
        self.ln1_g, self.ln1_b = o(H), z(H)
        self.ff1_w, self.ff1_b = mk(Fi, H), z(Fi)
        self.ff2_w, self.ff2_b = mk(H, Fi), z(H)
        self.ln2_g, self.ln2_b = o(H), z(H)

    NAMES = ("qkv_w", "qkv_b", "o_w", "o_b", "ln1_g", "ln1_b", "ff1_w", "ff1_b", "ff2_w", "ff2_b", "ln2_g", "ln2_b")


class BertEncoder:
    def __init__(self, cfg: BertConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        with torch.random.fork_rng(devices=[self.device] if self.device.type == "cuda" else []):
            torch.manual_seed(seed)
            H = cfg.hidden_size
            mk = lambda *s: (torch.randn(*s, device=self.device) * 0.02).to(dtype)  # noqa: E731
            self.wte = mk(cfg.vocab_size, H)
            self.wpe = mk(cfg.max_position, H)
            self.wtt = mk(cfg.type_vocab_size, H)
            self.emb_g = torch.ones(H, device=self.device, dtype=dtype)
            self.emb_b = torch.zeros(H, device=self.device, dtype=dtype)
            self.layers = [BertLayer(cfg, self.device, dtype) for _ in range(cfg.num_layers)]
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        if self.device.type == "cuda":  # weights are read from the auxiliary stream
            torch.cuda.current_stream(self.device).synchronize()

    def state_dict(self) -> dict:
        sd = {"wte": self.wte, "wpe": self.wpe, "wtt": self.wtt, "emb_g": self.emb_g, "emb_b": self.emb_b}
        for i, l in enumerate(self.layers):
            for n in BertLayer.NAMES:
                sd[f"layers.{i}.{n}"] = getattr(l, n)
        return sd

    def load_state_dict(self, sd: dict) -> None:
        for k in ("wte", "wpe", "wtt", "emb_g", "emb_b"):
            getattr(self, k).copy_(sd[k])
        for i, l in enumerate(self.layers):
            for n in BertLayer.NAMES:
                getattr(l, n).copy_(sd[f"layers.{i}.{n}"])

    # ------------------------------------------------------------------ fused layout
    def fused_supported(self) -> bool:
        c = self.cfg
        return (os.environ.get("LS_BERT_FUSED", "1") != "0" and c.hidden_size % 128 == 0
                and c.intermediate_size % 128 == 0)

    def fused_params(self):
        """Per layer: (qkv W' or W, c1, c2), (ff1 W', c1, c2) -- the LayerNorm of the
        previous sub-block folded into the weights (cached)."""
        if getattr(self, "_fused", None) is None:
            out = []
            prev_g = prev_b = None
            for l in self.layers:
                if prev_g is None:
                    qkv = (l.qkv_w, None, None)
                else:
                    qkv = self._fold(l.qkv_w, prev_g, prev_b)
                out.append((qkv, self._fold(l.ff1_w, l.ln1_g, l.ln1_b)))
                prev_g, prev_b = l.ln2_g, l.ln2_b
            self._fused = out
        return self._fused

    @staticmethod
    def _fold(w, g, b):
        wp = (w.float() * g.float()[None]).to(w.dtype)
        return wp, wp.float().sum(1).contiguous(), (w.float() @ b.float()).contiguous()

    def forward_fused(self, ids, pos, starts, lens, tiles, out_dtype=torch.float32):
        """The fused layer sequence through ops.gemm_fused (GPU kernels or fp32 reference)."""
        cfg = self.cfg
        H, nh, eps = cfg.hidden_size, cfg.num_heads, cfg.ln_eps
        T = ids.shape[0]
        x = ops.embed_layernorm(ids, pos, None, self.wte, self.wpe, self.wtt, self.emb_g, self.emb_b, eps)
        xp2 = st2 = None
        prev_g = prev_b = None
        for l, ((wq, qc1, qc2), (w1, fc1, fc2)) in zip(self.layers, self.fused_params()):
            if xp2 is None:
                qkv = ops.gemm_fused(x, wq, bias=l.qkv_b)
            else:
                qkv = ops.gemm_fused(xp2, wq, bias=l.qkv_b, ln_stats_in=st2, ln_width=H, c1=qc1, c2=qc2, eps=eps)
            a = ops.varlen_encoder_attention(qkv, starts, lens, tiles, nh, nh, self.scale)
            st1 = torch.empty(T, H // 64, 2, dtype=torch.float32, device=x.device)
            if xp2 is None:
                xp1 = ops.gemm_fused(a, l.o_w, bias=l.o_b, residual=x, stats_out=st1)
            else:
                xp1 = ops.gemm_fused(a, l.o_w, bias=l.o_b, residual=xp2, ln_stats_in=st2, ln_width=H,
                                     res_g=prev_g, res_b=prev_b, eps=eps, stats_out=st1)
            h = ops.gemm_fused(xp1, w1, bias=l.ff1_b, gelu=True, ln_stats_in=st1, ln_width=H, c1=fc1, c2=fc2,
                               eps=eps)
            st2 = torch.empty(T, H // 64, 2, dtype=torch.float32, device=x.device)
            xp2 = ops.gemm_fused(h, l.ff2_w, bias=l.ff2_b, residual=xp1, ln_stats_in=st1, ln_width=H,
                                 res_g=l.ln1_g, res_b=l.ln1_b, eps=eps, stats_out=st2)
            prev_g, prev_b = l.ln2_g, l.ln2_b
        x = ops.layernorm(xp2, prev_g, prev_b, eps)
        mode = 0 if cfg.pooling == "cls" else 1
        return ops.pool_embeddings(x, starts, lens, mode, cfg.normalize, out_dtype=out_dtype)

    @torch.inference_mode()
    def forward_packed(self, ids: torch.Tensor, pos: torch.Tensor, starts: torch.Tensor, lens: torch.Tensor,
                       tiles: torch.Tensor, out_dtype=torch.float32) -> torch.Tensor:
        """ids/pos: [T] int32 (packed), starts/lens: [B] int32 -> pooled [B, H]."""
        cfg = self.cfg
        nh = cfg.num_heads
        mode = 0 if cfg.pooling == "cls" else 1
        if self.device.type == "cuda" and ops.hip_available() and out_dtype in (torch.float32, self.dtype):
            # native executor (ops/csrc/runner.hip): whole encoder with the GIL released
            if getattr(self, "_runner", None) is None:
                fused = []
                if self.fused_supported():   # 6 extra tensors per layer select the fused path
                    for (wq, qc1, qc2), (w1, fc1, fc2) in self.fused_params():
                        z = torch.zeros(0, device=self.device)
                        fused.append([wq, qc1 if qc1 is not None else z, qc2 if qc2 is not None else z, w1, fc1, fc2])
                self._runner = ops.hip().BertRunner(
                    self.wte, self.wpe, self.wtt, self.emb_g, self.emb_b,
                    [[getattr(l, n) for n in BertLayer.NAMES] for l in self.layers], nh, cfg.ln_eps, self.scale,
                    mode, cfg.normalize, fused)
            return self._runner.forward(ids, pos, starts, lens, tiles, out_dtype == torch.float32)
        if self.fused_supported():
            return self.forward_fused(ids, pos, starts, lens, tiles, out_dtype)
        x = ops.embed_layernorm(ids, pos, None, self.wte, self.wpe, self.wtt, self.emb_g, self.emb_b, cfg.ln_eps)
        for l in self.layers:
            qkv = F.linear(x, l.qkv_w, l.qkv_b)
            a = ops.varlen_encoder_attention(qkv, starts, lens, tiles, nh, nh, self.scale)
            o = F.linear(a, l.o_w)
            x = ops.layernorm(o, l.ln1_g, l.ln1_b, cfg.ln_eps, bias=l.o_b, residual=x)
            h = F.linear(x, l.ff1_w)
            ops.bias_gelu_(h, l.ff1_b)
            o2 = F.linear(h, l.ff2_w)
            x = ops.layernorm(o2, l.ln2_g, l.ln2_b, cfg.ln_eps, bias=l.ff2_b, residual=x)
        return ops.pool_embeddings(x, starts, lens, mode, cfg.normalize, out_dtype=out_dtype)

    def pack(self, token_lists: List[List[int]]):
        """Host-side packing of a batch: ids, positions, starts, lens, tiles (CPU tensors)."""
        lens = [min(len(t), self.cfg.max_position) for t in token_lists]
        flat, pos, starts = [], [], []
        s = 0
        for t, n in zip(token_lists, lens):
            starts.append(s)
            flat.extend(t[:n])
            pos.extend(range(n))
            s += n
        return (torch.tensor(flat, dtype=torch.int32), torch.tensor(pos, dtype=torch.int32),
                torch.tensor(starts, dtype=torch.int32), torch.tensor(lens, dtype=torch.int32),
                ops.prefill_tiles(lens, 1))

    def pack_arrays(self, ids, lens):
        """``pack`` for already-packed numpy token ids / lengths (tokenizer
        ``encode_batch_packed``): positions and starts built vectorised."""
        import numpy as np
        lens0 = np.asarray(lens, dtype=np.int64)
        lens = np.minimum(lens0, self.cfg.max_position)
        starts = np.cumsum(lens) - lens
        if (lens != lens0).any():   # rows longer than max_position: keep each row's prefix
            src = np.cumsum(lens0) - lens0
            keep = np.repeat(src, lens) + (np.arange(int(lens.sum())) - np.repeat(starts, lens))
            ids = np.asarray(ids)[keep]
        pos = np.arange(int(lens.sum()), dtype=np.int64) - np.repeat(starts, lens)
        return (torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int32)),
                torch.from_numpy(pos.astype(np.int32)), torch.from_numpy(starts.astype(np.int32)),
                torch.from_numpy(lens.astype(np.int32)),
                torch.from_numpy(ops.prefill_tiles_np(lens, 1, np.zeros(len(lens), np.int64))))

    def encode_arrays(self, ids, lens, out_dtype=torch.float32) -> torch.Tensor:
        if len(lens) == 0:
            return torch.zeros(0, self.cfg.hidden_size, dtype=out_dtype, device=self.device)
        d_ids, pos, st, ln, tiles = (t.to(self.device, non_blocking=True) for t in self.pack_arrays(ids, lens))
        return self.forward_packed(d_ids, pos, st, ln, tiles, out_dtype)

    def encode_tokens(self, token_lists: List[List[int]], out_dtype=torch.float32) -> torch.Tensor:
        if not token_lists:
            return torch.zeros(0, self.cfg.hidden_size, dtype=out_dtype, device=self.device)
        ids, pos, st, ln, tiles = (t.to(self.device, non_blocking=True) for t in self.pack(token_lists))
        return self.forward_packed(ids, pos, st, ln, tiles, out_dtype)
