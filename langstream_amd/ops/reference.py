"""Plain-PyTorch (fp32) reference implementations of every HIP kernel.

Used (a) as the numerics oracle in the GPU tests and (b) as the CPU execution path
(CPU-only unit tests, the CPU plumbing benchmark).  On a GPU tensor the HIP kernels
are ALWAYS used; see ``langstream_amd.ops``.
"""
from __future__ import annotations

import math

import torch

KV_BLOCK = 64


def rmsnorm(x, w, eps):
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(x.dtype)


def fused_add_rmsnorm(x, residual, w, eps):
    r = (x.float() + residual.float()).to(x.dtype)
    residual.copy_(r)
    x.copy_(rmsnorm(r, w, eps))


def layernorm(x, bias, residual, g, b, eps):
    v = x.float()
    if bias is not None:
        v = v + bias.float()
    if residual is not None:
        v = v + residual.float()
    return torch.nn.functional.layer_norm(v, (v.shape[-1],), g.float(), b.float(), eps).to(x.dtype)


def embed_layernorm(ids, pos_ids, type_ids, wte, wpe, wtt, g, b, eps):
    v = wte[ids.long()].float() + wpe[pos_ids.long()].float()
    v = v + (wtt[type_ids.long()].float() if type_ids is not None else wtt[0].float())
    return torch.nn.functional.layer_norm(v, (v.shape[-1],), g.float(), b.float(), eps).to(wte.dtype)


def silu_and_mul(x):
    F = x.shape[-1] // 2
    g, u = x[..., :F].float(), x[..., F:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def bias_gelu(x, bias):
    v = x.float() + (bias.float() if bias is not None else 0.0)
    return torch.nn.functional.gelu(v).to(x.dtype)


def ln_row_stats(st, width, eps):
    """(mean, rstd) per row from partial (sum, sumsq) statistics [M, T, 2]."""
    s = st[..., 0].sum(-1)
    ss = st[..., 1].sum(-1)
    mu = s / width
    var = (ss / width - mu * mu).clamp_min(0.0)
    return mu, torch.rsqrt(var + eps)


def gemm_fused(x, w, bias=None, gelu=False, residual=None, ln_stats_in=None, ln_width=0, c1=None, c2=None,
               res_g=None, res_b=None, eps=1e-12, stats_out=None):
    """fp32 reference of ops/csrc/gemm_fused.hip (epilogue order documented there)."""
    v = x.float() @ w.float().t()
    mu = rs = None
    if ln_stats_in is not None:
        mu, rs = ln_row_stats(ln_stats_in.float(), ln_width, eps)
        mu, rs = mu[:, None], rs[:, None]
        if res_g is None:
            v = rs * (v - mu * c1.float()[None]) + c2.float()[None]
    if bias is not None:
        v = v + bias.float()
    if gelu:
        v = torch.nn.functional.gelu(v)
    if residual is not None:
        r = residual.float()
        if ln_stats_in is not None and res_g is not None:
            r = (r - mu) * rs * res_g.float() + res_b.float()
        v = v + r
    out = v.to(x.dtype)
    if stats_out is not None:
        o = out.float().view(out.shape[0], -1, 64)
        stats_out.copy_(torch.stack([o.sum(-1), (o * o).sum(-1)], -1))
    return out


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, scaling: dict | None = None,
                 device=None) -> torch.Tensor:
    """[max_pos, D] f32: cols [0, D/2) = cos, [D/2, D) = sin.  Supports the Llama-3.1
    "llama3" frequency scaling (factor / low_freq_factor / high_freq_factor)."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2 / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lf, hf = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        low_wl, high_wl = old / lf, old / hf
        wl = 2 * math.pi / inv
        smooth = (old / wl - lf) / (hf - lf)
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        mid = (wl <= low_wl) & (wl >= high_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([t.cos(), t.sin()], dim=-1).float().to(device)


def apply_rope(x, pos, cos_sin):
    """x: [T, H, D]; HF rotate_half convention."""
    D = x.shape[-1]
    half = D // 2
    cs = cos_sin[pos.long()]
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    x1, x2 = x[..., :half].float(), x[..., half:].float()
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def rope_and_cache(qkv, pos, cos_sin, slots, k_cache, v_cache, Hq, Hkv, apply_rope_flag=True):
    T = qkv.shape[0]
    D = k_cache.shape[3]
    BS = k_cache.shape[2]
    v = qkv.view(T, Hq + 2 * Hkv, D)
    if apply_rope_flag:
        v[:, : Hq + Hkv] = apply_rope(v[:, : Hq + Hkv], pos, cos_sin)
    for t in range(T):
        s = int(slots[t])
        if s < 0:
            continue
        blk, off = divmod(s, BS)
        k_cache[blk, :, off, :] = v[t, Hq: Hq + Hkv]
        v_cache[blk, :, off // 8, :, off % 8] = v[t, Hq + Hkv:]    # [NB, Hkv, BS/8, D, 8]


def gather_kv(k_cache, v_cache, block_table, n):
    """Contiguous K [n, Hkv, D] and V [n, Hkv, D] of one sequence from the paged cache."""
    BS = k_cache.shape[2]
    nb = (n + BS - 1) // BS
    ks = [k_cache[int(block_table[i])] for i in range(nb)]           # [Hkv, BS, D]
    # V blocks [Hkv, BS/8, D, 8] -> [Hkv, BS, D]
    vs = [v_cache[int(block_table[i])].permute(0, 1, 3, 2).reshape(v_cache.shape[1], BS, -1) for i in range(nb)]
    K = torch.cat(ks, dim=1)[:, :n].transpose(0, 1)
    V = torch.cat(vs, dim=1)[:, :n].transpose(0, 1)
    return K, V


def attention(q, k, v, scale, causal_offset: int | None):
    """q [Tq, Hq, D], k/v [Tk, Hkv, D] -> [Tq, Hq, D]; causal if offset given
    (query i sits at absolute position offset + i)."""
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    kf = k.float().repeat_interleave(G, dim=1)
    vf = v.float().repeat_interleave(G, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal_offset is not None:
        qi = torch.arange(q.shape[0], device=q.device)[:, None] + causal_offset
        ki = torch.arange(k.shape[0], device=q.device)[None, :]
        s = s.masked_fill((ki > qi)[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, vf).to(q.dtype)


def paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale):
    B = q.shape[0]
    D = k_cache.shape[3]
    qv = q.reshape(B, -1, D)
    outs = []
    for b in range(B):
        n = int(ctx_lens[b])
        if n == 0:
            outs.append(torch.zeros_like(qv[b: b + 1]))
            continue
        K, V = gather_kv(k_cache, v_cache, block_tables[b], n)
        outs.append(attention(qv[b: b + 1], K, V, scale, causal_offset=None))
    return torch.cat(outs, 0)


def paged_prefill_attention(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, Hq, scale):
    D = k_cache.shape[3]
    T = q.shape[0]
    out = torch.empty(T, Hq, D, dtype=q.dtype, device=q.device)
    for s in range(len(q_start)):
        qs, ql, cl = int(q_start[s]), int(q_len[s]), int(ctx_len[s])
        K, V = gather_kv(k_cache, v_cache, block_tables[s], cl)
        qq = q[qs: qs + ql, : Hq * D].reshape(ql, Hq, D)
        out[qs: qs + ql] = attention(qq, K, V, scale, causal_offset=cl - ql)
    return out.reshape(T, Hq * D)


def varlen_encoder_attention(qkv, q_start, q_len, Hq, Hkv, scale):
    T = qkv.shape[0]
    D = qkv.shape[1] // (Hq + 2 * Hkv)
    v = qkv.view(T, Hq + 2 * Hkv, D)
    out = torch.empty(T, Hq, D, dtype=qkv.dtype, device=qkv.device)
    for s in range(len(q_start)):
        a, n = int(q_start[s]), int(q_len[s])
        out[a: a + n] = attention(v[a: a + n, :Hq], v[a: a + n, Hq: Hq + Hkv], v[a: a + n, Hq + Hkv:], scale, None)
    return out.reshape(T, Hq * D)


def pool_embeddings(x, start, length, mode, normalize):
    outs = []
    for s, n in zip(start.tolist(), length.tolist()):
        n = max(n, 1)
        seg = x[s: s + n].float()
        v = seg[0] if mode == 0 else seg.mean(0)
        outs.append(v)
    o = torch.stack(outs) if outs else x.new_zeros((0, x.shape[1]), dtype=torch.float32)
    if normalize:
        o = torch.nn.functional.normalize(o, dim=-1, eps=1e-12)
    return o


def knn_topk(X, Q, k):
    s = Q.float() @ X.float().t()
    kk = min(k, X.shape[0])
    v, i = torch.topk(s, kk, dim=-1)
    if kk < k:
        pad = k - kk
        v = torch.cat([v, v.new_full((v.shape[0], pad), float("-inf"))], -1)
        i = torch.cat([i, i.new_full((i.shape[0], pad), -1)], -1)
    return v, i.int()


def sample(logits, temperature, top_k, top_p, generators=None):
    """Reference sampler.  Returns (tokens int32 [B], logprobs f32 [B])."""
    lf = logits.float()
    logp = torch.log_softmax(lf, dim=-1)
    toks = []
    for r in range(lf.shape[0]):
        T = float(temperature[r])
        if T <= 0:
            toks.append(int(torch.argmax(lf[r])))
            continue
        z = lf[r] / T
        probs = torch.softmax(z, -1)
        k = int(top_k[r])
        p = float(top_p[r])
        if k > 0 and k < probs.numel():
            kth = torch.topk(probs, k).values[-1]
            probs = torch.where(probs >= kth, probs, torch.zeros_like(probs))
        if 0 < p < 1:
            sp, si = torch.sort(probs, descending=True)
            c = torch.cumsum(sp, 0)
            keep = c - sp < p * c[-1]
            mask = torch.zeros_like(probs, dtype=torch.bool)
            mask[si[keep]] = True
            probs = torch.where(mask, probs, torch.zeros_like(probs))
        g = generators[r] if generators else None
        toks.append(int(torch.multinomial(probs / probs.sum(), 1, generator=g)))
    t = torch.tensor(toks, dtype=torch.int32, device=logits.device)
    return t, logp.gather(1, t.long()[:, None])[:, 0]
