"""Checkpoint loading: HuggingFace -> packed layouts, tensor-parallel sharding, safetensors IO.

The reference loads models inside the remote providers or through DJL
(``AbstractHuggingFaceEmbeddingService.java:42-224``); here weights are packed once into
the GEMM-friendly layouts of ``models/llama.py`` / ``models/bert.py`` and each TP rank
keeps only its shard (a 70B model at TP=8 is ~17.5 GB per MI355X, leaving >250 GB of
HBM for the KV cache).

Only non-executing loaders are used: safetensors, or ``torch.load(weights_only=True)``.
Loading is streamed tensor by tensor (``safe_open``) so host memory stays bounded.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Iterable, Optional, Tuple

import torch

from .llama import LlamaConfig

# ---------------------------------------------------------------- safetensors IO


def iter_checkpoint(path: str) -> Iterable[Tuple[str, torch.Tensor]]:
    """Yield (name, tensor) from a file or a directory of ``*.safetensors`` (or
    ``*.bin``/``*.pt`` via ``torch.load(weights_only=True)``)."""
    files = [path] if os.path.isfile(path) else sorted(
        glob.glob(os.path.join(path, "*.safetensors")) or glob.glob(os.path.join(path, "*.bin"))
        or glob.glob(os.path.join(path, "*.pt")))
    if not files:
        raise FileNotFoundError(f"no checkpoint files under {path}")
    for f in files:
        if f.endswith(".safetensors"):
            from safetensors import safe_open
            with safe_open(f, framework="pt", device="cpu") as fh:
                for k in fh.keys():
                    yield k, fh.get_tensor(k)
        else:
            sd = torch.load(f, map_location="cpu", weights_only=True)
            yield from sd.items()


def save_packed(sd: Dict[str, torch.Tensor], path: str, metadata: Optional[dict] = None) -> None:
    from safetensors.torch import save_file
    save_file({k: v.detach().contiguous().cpu() for k, v in sd.items()}, path,
              metadata={k: json.dumps(v) for k, v in (metadata or {}).items()})


def load_packed(path: str, device="cpu") -> Dict[str, torch.Tensor]:
    """Load a packed state dict (our names); converts HF checkpoints on the fly."""
    sd = dict(iter_checkpoint(path))
    if any(k.startswith("model.layers.") or k == "model.embed_tokens.weight" for k in sd):
        cfg = llama_config_from_hf(path) if os.path.isdir(path) else None
        sd = convert_hf_llama(sd, cfg)
    elif any(k.startswith(("bert.", "encoder.layer.", "embeddings.")) for k in sd):
        sd = convert_hf_bert(sd)
    return {k: v.to(device) for k, v in sd.items()}


# ---------------------------------------------------------------- Llama


def llama_config_from_hf(model_dir: str) -> LlamaConfig:
    with open(os.path.join(model_dir, "config.json")) as f:
        c = json.load(f)
    eos = c.get("eos_token_id", 2)
    return LlamaConfig(
        name=c.get("_name_or_path", "llama"), vocab_size=c["vocab_size"], hidden_size=c["hidden_size"],
        intermediate_size=c["intermediate_size"], num_layers=c["num_hidden_layers"],
        num_heads=c["num_attention_heads"], num_kv_heads=c.get("num_key_value_heads", c["num_attention_heads"]),
        head_dim=c.get("head_dim", c["hidden_size"] // c["num_attention_heads"]),
        rope_theta=c.get("rope_theta", 10000.0), rope_scaling=c.get("rope_scaling"),
        rms_eps=c.get("rms_norm_eps", 1e-5), max_position=c.get("max_position_embeddings", 8192),
        tie_embeddings=c.get("tie_word_embeddings", False), bos_token_id=c.get("bos_token_id", 1),
        eos_token_ids=tuple(eos) if isinstance(eos, list) else (eos,))


def convert_hf_llama(hf: Dict[str, torch.Tensor], cfg: Optional[LlamaConfig] = None) -> Dict[str, torch.Tensor]:
    """HF ``LlamaForCausalLM`` names -> packed names (fused qkv / gate_up)."""
    out = {"embed": hf["model.embed_tokens.weight"], "final_norm": hf["model.norm.weight"]}
    out["lm_head"] = hf.get("lm_head.weight", hf["model.embed_tokens.weight"])
    i = 0
    while f"model.layers.{i}.self_attn.q_proj.weight" in hf:
        p = f"model.layers.{i}."
        out[f"layers.{i}.qkv_w"] = torch.cat([hf[p + "self_attn.q_proj.weight"], hf[p + "self_attn.k_proj.weight"],
                                              hf[p + "self_attn.v_proj.weight"]], 0)
        out[f"layers.{i}.o_w"] = hf[p + "self_attn.o_proj.weight"]
        out[f"layers.{i}.gate_up_w"] = torch.cat([hf[p + "mlp.gate_proj.weight"], hf[p + "mlp.up_proj.weight"]], 0)
        out[f"layers.{i}.down_w"] = hf[p + "mlp.down_proj.weight"]
        out[f"layers.{i}.in_norm"] = hf[p + "input_layernorm.weight"]
        out[f"layers.{i}.post_norm"] = hf[p + "post_attention_layernorm.weight"]
        i += 1
    if cfg is not None:
        assert i == cfg.num_layers, f"checkpoint has {i} layers, config {cfg.num_layers}"
    return out


def shard_llama(sd: Dict[str, torch.Tensor], cfg: LlamaConfig, rank: int, world: int) -> Dict[str, torch.Tensor]:
    """Full packed state dict -> this TP rank's shard: column-parallel qkv / gate_up
    (by heads / by FFN columns), row-parallel o / down, vocab-parallel embed / lm_head
    (padded to a multiple of ``world``), replicated norms."""
    if world == 1:
        return dict(sd)
    from .llama import tp_kv_heads
    D = cfg.head_dim
    hq, hkv, f = cfg.num_heads // world, tp_kv_heads(cfg.num_kv_heads, world), cfg.intermediate_size // world
    # first KV head of this rank (replicated heads when world > num_kv_heads)
    kv0 = rank * hkv if cfg.num_kv_heads >= world else rank // (world // cfg.num_kv_heads)
    Hq, Hkv, F = cfg.num_heads * D, cfg.num_kv_heads * D, cfg.intermediate_size
    vpr = (cfg.vocab_size + world - 1) // world
    out = {}
    for k, v in sd.items():
        if k.endswith(".qkv_w"):
            q, kk, vv = v[:Hq], v[Hq: Hq + Hkv], v[Hq + Hkv:]
            out[k] = torch.cat([q[rank * hq * D:(rank + 1) * hq * D], kk[kv0 * D:(kv0 + hkv) * D],
                                vv[kv0 * D:(kv0 + hkv) * D]], 0)
        elif k.endswith(".o_w"):
            out[k] = v[:, rank * hq * D:(rank + 1) * hq * D]
        elif k.endswith(".gate_up_w"):
            g, u = v[:F], v[F:]
            out[k] = torch.cat([g[rank * f:(rank + 1) * f], u[rank * f:(rank + 1) * f]], 0)
        elif k.endswith(".down_w"):
            out[k] = v[:, rank * f:(rank + 1) * f]
        elif k in ("embed", "lm_head"):
            part = v[rank * vpr:(rank + 1) * vpr]
            if part.shape[0] < vpr:
                part = torch.cat([part, part.new_zeros(vpr - part.shape[0], v.shape[1])], 0)
            out[k] = part
        else:
            out[k] = v
    return {k: v.contiguous() for k, v in out.items()}


# ---------------------------------------------------------------- BERT


def convert_hf_bert(hf: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """HF ``BertModel`` names (with or without the ``bert.`` prefix) -> packed names."""
    def g(name):
        for p in ("", "bert.", "model."):
            if p + name in hf:
                return hf[p + name]
        raise KeyError(name)

    out = {"wte": g("embeddings.word_embeddings.weight"), "wpe": g("embeddings.position_embeddings.weight"),
           "wtt": g("embeddings.token_type_embeddings.weight"), "emb_g": g("embeddings.LayerNorm.weight"),
           "emb_b": g("embeddings.LayerNorm.bias")}
    i = 0
    while True:
        p = f"encoder.layer.{i}."
        try:
            q = g(p + "attention.self.query.weight")
        except KeyError:
            break
        out[f"layers.{i}.qkv_w"] = torch.cat([q, g(p + "attention.self.key.weight"),
                                              g(p + "attention.self.value.weight")], 0)
        out[f"layers.{i}.qkv_b"] = torch.cat([g(p + "attention.self.query.bias"), g(p + "attention.self.key.bias"),
                                              g(p + "attention.self.value.bias")], 0)
        out[f"layers.{i}.o_w"] = g(p + "attention.output.dense.weight")
        out[f"layers.{i}.o_b"] = g(p + "attention.output.dense.bias")
        out[f"layers.{i}.ln1_g"] = g(p + "attention.output.LayerNorm.weight")
        out[f"layers.{i}.ln1_b"] = g(p + "attention.output.LayerNorm.bias")
        out[f"layers.{i}.ff1_w"] = g(p + "intermediate.dense.weight")
        out[f"layers.{i}.ff1_b"] = g(p + "intermediate.dense.bias")
        out[f"layers.{i}.ff2_w"] = g(p + "output.dense.weight")
        out[f"layers.{i}.ff2_b"] = g(p + "output.dense.bias")
        out[f"layers.{i}.ln2_g"] = g(p + "output.LayerNorm.weight")
        out[f"layers.{i}.ln2_b"] = g(p + "output.LayerNorm.bias")
        i += 1
    return out
