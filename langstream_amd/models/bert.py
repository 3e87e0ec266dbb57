"""BERT-family sentence encoder (bge-small-en / multilingual-e5-small / MiniLM shapes).

Local replacement for the reference's DJL + libtorch-CPU embedding path
(``AbstractHuggingFaceEmbeddingService.java:42-224``, which predicts one text at a
time -- comment at :192-193) and for the remote embedding services.

Padding-free: a batch is packed into one [T, H] token matrix with per-sequence
start/len; attention is the varlen MFMA encoder kernel, so no FLOPs are spent on pad
tokens.  Per layer: QKV GEMM (+bias, hipBLASLt) -> varlen attention (HIP) -> O GEMM ->
fused bias+residual+LayerNorm (HIP) -> FFN1 GEMM -> fused bias+GELU (HIP) -> FFN2 GEMM
-> fused bias+residual+LayerNorm (HIP); then CLS/mean pooling + L2 normalise (HIP).
"""
from __future__ import annotations

import math
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
                self._runner = ops.hip().BertRunner(
                    self.wte, self.wpe, self.wtt, self.emb_g, self.emb_b,
                    [[getattr(l, n) for n in BertLayer.NAMES] for l in self.layers], nh, cfg.ln_eps, self.scale,
                    mode, cfg.normalize)
            return self._runner.forward(ids, pos, starts, lens, tiles, out_dtype == torch.float32)
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

    def encode_tokens(self, token_lists: List[List[int]], out_dtype=torch.float32) -> torch.Tensor:
        if not token_lists:
            return torch.zeros(0, self.cfg.hidden_size, dtype=out_dtype, device=self.device)
        ids, pos, st, ln, tiles = (t.to(self.device, non_blocking=True) for t in self.pack(token_lists))
        return self.forward_packed(ids, pos, st, ln, tiles, out_dtype)
