"""langstream_amd.ops -- the compute path.

Every function dispatches on the device of its inputs:

* GPU tensors -> the hand-written gfx950 HIP kernels in ``ops/csrc`` (module
  ``_hip_ops``, built in-tree by ``langstream_amd._build``).  If the extension is
  missing on a GPU we raise -- there is NO silent eager fallback on the GPU.
* CPU tensors -> ``ops.reference`` (plain fp32 PyTorch), used by the CPU test
  suite and the CPU plumbing pipeline.

Plain dense GEMMs are not here: they go to hipBLASLt through ``torch.matmul`` /
``torch.nn.functional.linear`` (allowed for library GEMMs); everything fused or
attention-shaped is ours.
"""
from __future__ import annotations

import importlib.machinery
import importlib.util
import os
import sys
from typing import Optional, Sequence

import torch

from . import reference as ref

KV_BLOCK = 64


def new_kv_cache(num_blocks: int, hkv: int, head_dim: int, device, dtype, zeros: bool = True):
    """(K, V) paged caches of one layer: K [NB, Hkv, 64, D]; V^T in 8-key groups
    [NB, Hkv, 8, D, 8] (element (d, key) of a block at [key // 8, d, key % 8]; see
    ops/csrc/common.h vt_off)."""
    mk = torch.zeros if zeros else torch.empty
    return (mk(num_blocks, hkv, KV_BLOCK, head_dim, device=device, dtype=dtype),
            mk(num_blocks, hkv, KV_BLOCK // 8, head_dim, 8, device=device, dtype=dtype))


PREFILL_ROWS = 128  # query rows per prefill-attention workgroup (see attention_prefill.hip)

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_hip_ops.so")
_ext = None
_ext_err: Optional[BaseException] = None


def _load():
    global _ext, _ext_err
    if _ext is not None or _ext_err is not None:
        return _ext
    try:
        if not os.path.exists(_SO):
            raise ImportError(f"{_SO} not built (run python -m langstream_amd._build)")
        loader = importlib.machinery.ExtensionFileLoader("_hip_ops", _SO)
        spec = importlib.util.spec_from_file_location("_hip_ops", _SO, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        sys.modules["langstream_amd.ops._hip_ops"] = mod
        _ext = mod
        _load_pgemm_route(mod)
    except BaseException as e:  # noqa: BLE001 - remember and re-raise on GPU use
        _ext_err = e
    return _ext


def _load_pgemm_route(mod, path: Optional[str] = None) -> int:
    """Load ops/pgemm_route_gfx950.csv (tools/pgemm_route_tune.py: N,K,M,lib_us,pp_us per
    256-row M bucket) into the runner's prefill routing table: the plain projections run on
    gemm_prefill where it measured >= 3 % faster than hipBLASLt.  LS_PGEMM_ROUTE=0: off."""
    path = path or os.path.join(_HERE, "pgemm_route_gfx950.csv")
    if os.environ.get("LS_PGEMM_ROUTE", "1") == "0" or not os.path.exists(path):
        return 0
    import csv
    rows = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            key = (int(r["N"]), int(r["K"]))
            rows.setdefault(key, {})[int(r["M"]) // 256] = float(r["pp_us"]) < 0.97 * float(r["lib_us"])
    for (n, k), d in rows.items():
        mod.set_pgemm_route(n, k, [int(d.get(b, False)) for b in range(max(d) + 1)])
    return len(rows)


_TUNED = None


def enable_decode_gemm_tuning(path: Optional[str] = None) -> bool:
    """Load the cold-timed hipBLASLt/rocBLAS solution picks for the decode-step projection
    GEMMs (``tools/gemm_cold_select.py``) into PyTorch TunableOp with tuning disabled: the
    listed (M, N, K) use the picked solution, every other GEMM keeps the default heuristic.
    Opt out with ``LS_GEMM_TUNING=0``."""
    global _TUNED
    if _TUNED is not None:
        return _TUNED
    path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_decode_gfx950.csv")
    _TUNED = False
    if os.environ.get("LS_GEMM_TUNING", "1") == "0" or not os.path.exists(path) or not torch.cuda.is_available():
        return False
    import tempfile
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(False)
    tun.set_filename(os.path.join(tempfile.gettempdir(), f"ls_tunableop_{os.getpid()}.csv"),
                     insert_device_ordinal=False)
    _TUNED = bool(tun.read_file(path))
    return _TUNED


def hip_available() -> bool:
    return _load() is not None


def hip() :
    """The native module; raises loudly when it cannot be loaded."""
    m = _load()
    if m is None:
        raise RuntimeError(f"langstream_amd HIP kernels unavailable: {_ext_err!r}")
    return m


def _gpu(*ts) -> bool:
    return any(isinstance(t, torch.Tensor) and t.is_cuda for t in ts)


# ---------------------------------------------------------------- norms
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _gpu(x):
        out = torch.empty_like(x) if out is None else out
        hip().rmsnorm(out, x, w, eps)
        return out
    r = ref.rmsnorm(x, w, eps)
    if out is not None:
        out.copy_(r)
        return out
    return r


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float) -> None:
    """In place: residual += x ; x = rmsnorm(residual) * w."""
    if _gpu(x):
        hip().fused_add_rmsnorm(x, residual, w, eps)
    else:
        ref.fused_add_rmsnorm(x, residual, w, eps)


def layernorm(x, g, b, eps, bias=None, residual=None, out=None):
    if _gpu(x):
        out = torch.empty_like(x) if out is None else out
        hip().layernorm(out, x, bias, residual, g, b, eps)
        return out
    r = ref.layernorm(x, bias, residual, g, b, eps)
    if out is not None:
        out.copy_(r)
        return out
    return r


def embed_layernorm(ids, pos_ids, type_ids, wte, wpe, wtt, g, b, eps):
    if _gpu(wte):
        out = torch.empty(ids.numel(), wte.shape[1], dtype=wte.dtype, device=wte.device)
        hip().embed_layernorm(out, ids, pos_ids, type_ids, wte, wpe, wtt, g, b, eps)
        return out
    return ref.embed_layernorm(ids, pos_ids, type_ids, wte, wpe, wtt, g, b, eps)


# ---------------------------------------------------------------- GEMM with fused epilogues
def gemm_fused(x, w, bias=None, gelu=False, residual=None, ln_stats_in=None, ln_width=0, c1=None, c2=None,
               res_g=None, res_b=None, eps=1e-12, stats_out=None, out=None):
    """out = epilogue(x . w^T) on MFMA (ops/csrc/gemm_fused.hip): bias, erf-GELU, residual,
    and LayerNorm folded in from the neighbours (``ln_stats_in`` partial row statistics of
    the LayerNorm input + ``c1``/``c2`` for an un-normalised input, or + ``res_g``/``res_b``
    to normalise the residual); ``stats_out`` [M, N/64, 2] receives the output rows'
    partial (sum, sumsq)."""
    if _gpu(x):
        out = torch.empty(x.shape[0], w.shape[0], dtype=x.dtype, device=x.device) if out is None else out
        hip().gemm_fused(out, x, w, bias, gelu, residual, ln_stats_in, ln_width, c1, c2, res_g, res_b, eps,
                         stats_out)
        return out
    r = ref.gemm_fused(x, w, bias, gelu, residual, ln_stats_in, ln_width, c1, c2, res_g, res_b, eps, stats_out)
    if out is not None:
        out.copy_(r)
        return out
    return r


def gemm_prefill(x, w, silu=False, out=None, variant=-1):
    """Prefill-sized MFMA GEMM (ops/csrc/gemm_prefill.hip, 256 x 256 tiles): x . w^T, or with
    ``silu`` the Llama SwiGLU of the fused gate_up weight [2F, K]: silu(x.g^T) * (x.u^T).
    ``variant``: -1 the configured kernel (LS_PGEMM_KERNEL), 0 the 32-deep ring kernel,
    1 the ping-pong kernel (K % 128 == 0)."""
    if _gpu(x):
        n = w.shape[0] // 2 if silu else w.shape[0]
        out = torch.empty(x.shape[0], n, dtype=x.dtype, device=x.device) if out is None else out
        hip().gemm_prefill(out, x, w, silu, variant)
        return out
    y = x.float() @ w.float().t()
    r = (ref.silu_and_mul(y) if silu else y).to(x.dtype)
    if out is not None:
        out.copy_(r)
        return out
    return r


def gemm(x, w, bias=None, act=None, residual=None):
    """Hand-written MFMA linear: act in (None, "gelu", "swiglu"); swiglu takes the fused
    gate_up weight [2F, K] and returns silu(x.g^T) * (x.u^T)."""
    if act == "swiglu":
        F = w.shape[0] // 2
        if _gpu(x):
            out = torch.empty(x.shape[0], F, dtype=x.dtype, device=x.device)
            hip().skinny_gemm_silu(out, x, w)
            return out
        return ref.silu_and_mul(x.float() @ w.float().t()).to(x.dtype)
    return gemm_fused(x, w, bias=bias, gelu=act == "gelu", residual=residual)


# ---------------------------------------------------------------- activations
def silu_and_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _gpu(x):
        F = x.shape[-1] // 2
        out = torch.empty(*x.shape[:-1], F, dtype=x.dtype, device=x.device) if out is None else out
        hip().silu_and_mul(out, x)
        return out
    return ref.silu_and_mul(x)


def bias_gelu_(x: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    if _gpu(x):
        hip().bias_gelu(x, bias)
        return x
    x.copy_(ref.bias_gelu(x, bias))
    return x


# ---------------------------------------------------------------- rope / kv cache
def rope_and_cache(qkv, pos, cos_sin, slots, k_cache, v_cache, Hq: int, Hkv: int, apply_rope: bool = True):
    if _gpu(qkv):
        hip().rope_and_cache(qkv, pos, cos_sin, slots, k_cache, v_cache, Hq, Hkv, apply_rope)
    else:
        ref.rope_and_cache(qkv, pos, cos_sin, slots, k_cache, v_cache, Hq, Hkv, apply_rope)


# ---------------------------------------------------------------- attention
def decode_splits(max_blocks: int, min_blocks_per_split: int = 0) -> tuple[int, int]:
    """Split-KV plan for decode: (nsplit_max, min_blocks_per_split).  The kernel picks
    the split count per launch from the batch (no split once B*Hkv workgroups fill the
    chip; see attention_decode.hip), and each sequence spreads its own context evenly
    over the splits (at least `min_blocks_per_split` blocks each, one per wave), so one
    captured graph serves every context length.  The workspace is sized for nsplit_max."""
    if min_blocks_per_split <= 0:
        min_blocks_per_split = int(os.environ.get("LS_ATTN_MIN_BPS", "4"))
    bps = max(1, min_blocks_per_split)
    nsplit = max(1, (max_blocks + bps - 1) // bps)
    return nsplit, bps


def paged_decode_attention(q, k_cache, v_cache, block_tables, ctx_lens, scale, out=None,
                           nsplit: int = 1, blocks_per_split: int = 1 << 30, workspace=None):
    """q: [B, Hq*D] (may be a strided view into the QKV buffer); returns [B, Hq*D]."""
    B = ctx_lens.shape[0]
    D = k_cache.shape[3]
    Hq = q.shape[-1] // D if q.dim() == 2 else q.shape[1]
    if _gpu(q):
        out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device) if out is None else out
        if nsplit > 1:
            assert workspace is not None and workspace.numel() >= B * Hq * nsplit * (D + 2)
        ws = workspace if workspace is not None else out.new_empty(0, dtype=torch.float32)
        hip().paged_decode_attention(out, q, k_cache, v_cache, block_tables, ctx_lens, scale, nsplit,
                                     min(blocks_per_split, block_tables.shape[1]), ws)
        return out
    r = ref.paged_decode_attention(q.reshape(B, Hq, D), k_cache, v_cache, block_tables, ctx_lens, scale)
    r = r.reshape(B, Hq * D)
    if out is not None:
        out.copy_(r)
        return out
    return r


def paged_decode_attention_rope(qkv, pos, cos_sin, slots, k_cache, v_cache, block_tables, ctx_lens, scale,
                                Hq: int, out=None, nsplit: int = 1, blocks_per_split: int = 1 << 30,
                                workspace=None):
    """Decode-only step with RoPE + the KV-cache write fused into attention.  qkv:
    [B, (Hq + 2 Hkv) D] un-rotated projection rows (left unmodified); the new token of
    each row (ctx_lens count it) is written to the cache at ``slots`` and attended from
    registers.  Returns [B, Hq*D]; numerically rope_and_cache + paged_decode_attention."""
    B = ctx_lens.shape[0]
    D = k_cache.shape[3]
    Hkv = k_cache.shape[1]
    if _gpu(qkv):
        out = torch.empty(B, Hq * D, dtype=qkv.dtype, device=qkv.device) if out is None else out
        if nsplit > 1:
            assert workspace is not None and workspace.numel() >= B * Hq * nsplit * (D + 2)
        ws = workspace if workspace is not None else out.new_empty(0, dtype=torch.float32)
        hip().paged_decode_attention_rope(out, qkv, pos, cos_sin, slots, k_cache, v_cache, block_tables, ctx_lens,
                                          scale, nsplit, min(blocks_per_split, block_tables.shape[1]), ws)
        return out
    work = qkv.clone()
    ref.rope_and_cache(work, pos, cos_sin, slots, k_cache, v_cache, Hq, Hkv, True)
    return paged_decode_attention(work[:, : Hq * D], k_cache, v_cache, block_tables, ctx_lens, scale, out=out)


def prefill_tiles(q_lens: Sequence[int], G: int, prefix_lens: Sequence[int] | None = None) -> torch.Tensor:
    """Work list for the prefill kernel: (seq, first row), rows = token*G + g, heaviest first."""
    tiles = []
    for s, ql in enumerate(q_lens):
        rows = ql * G
        pre = prefix_lens[s] if prefix_lens is not None else 0
        for r0 in range(0, rows, PREFILL_ROWS):
            last = min(r0 + PREFILL_ROWS, rows) - 1
            tiles.append((pre + last // G, s, r0))
    tiles.sort(key=lambda t: -t[0])
    t = torch.tensor([(s, r0) for _, s, r0 in tiles], dtype=torch.int32)
    return t.reshape(-1, 2)


def prefill_tiles_np(q_lens, G: int, prefix_lens, out=None):
    """numpy twin of :func:`prefill_tiles` (no torch calls: used by the engine's
    scheduler, which must not hand the GIL around).  Writes into ``out`` when given
    and returns the number of tiles."""
    import numpy as np
    q_lens = np.asarray(q_lens, dtype=np.int64)
    prefix = np.asarray(prefix_lens, dtype=np.int64)
    rows = q_lens * G
    n_per = (rows + PREFILL_ROWS - 1) // PREFILL_ROWS
    seq = np.repeat(np.arange(len(q_lens)), n_per)
    # index of each tile within its sequence, vectorised
    base = np.repeat(np.cumsum(n_per) - n_per, n_per)
    first = (np.arange(len(seq)) - base) * PREFILL_ROWS
    last = np.minimum(first + PREFILL_ROWS, rows[seq]) - 1
    work = prefix[seq] + last // G
    order = np.argsort(-work, kind="stable")
    tiles = np.stack([seq[order], first[order]], axis=1).astype(np.int32)
    if out is None:
        return tiles
    out[: len(tiles)] = tiles
    return len(tiles)


def paged_prefill_attention(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, tiles, Hq, scale,
                            out=None):
    T = q.shape[0]
    D = k_cache.shape[3]
    if _gpu(q):
        out = torch.empty(T, Hq * D, dtype=q.dtype, device=q.device) if out is None else out
        hip().paged_prefill_attention(out, q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, tiles,
                                      Hq, scale)
        return out
    r = ref.paged_prefill_attention(q, k_cache, v_cache, block_tables, q_start, q_len, ctx_len, Hq, scale)
    if out is None:
        return r
    for s, n in zip(q_start.tolist(), q_len.tolist()):
        out[s: s + n] = r[s: s + n]
    return out


def varlen_encoder_attention(qkv, q_start, q_len, tiles, Hq, Hkv, scale, out=None):
    T = qkv.shape[0]
    D = qkv.shape[1] // (Hq + 2 * Hkv)
    if _gpu(qkv):
        out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device) if out is None else out
        hip().varlen_encoder_attention(out, qkv, q_start, q_len, tiles, Hq, Hkv, scale)
        return out
    return ref.varlen_encoder_attention(qkv, q_start, q_len, Hq, Hkv, scale)


# ---------------------------------------------------------------- sampling
def sample(logits, temperature, top_k, top_p, seeds, steps, n_top: int = 0):
    """Returns (tokens int32 [B], logprobs f32 [B], top_ids [B,n]|None, top_lps [B,n]|None)."""
    B = logits.shape[0]
    if _gpu(logits):
        dev = logits.device
        tok = torch.empty(B, dtype=torch.int32, device=dev)
        lp = torch.empty(B, dtype=torch.float32, device=dev)
        ti = torch.empty(B * max(n_top, 1), dtype=torch.int32, device=dev)
        tl = torch.empty(B * max(n_top, 1), dtype=torch.float32, device=dev)
        hip().sample_tokens(logits, temperature, top_k, top_p, seeds, steps, tok, lp, ti, tl, n_top)
        if n_top:
            return tok, lp, ti.view(B, n_top), tl.view(B, n_top)
        return tok, lp, None, None
    gens = []
    for r in range(B):
        g = torch.Generator()
        g.manual_seed(int(seeds[r]) * 1_000_003 + int(steps[r]))
        gens.append(g)
    tok, lp = ref.sample(logits, temperature, top_k, top_p, gens)
    if n_top:
        logp = torch.log_softmax(logits.float(), -1)
        v, i = torch.topk(logp, n_top, dim=-1)
        return tok, lp, i.int(), v
    return tok, lp, None, None


def sample_vocab_parallel(local, vstart: int, vocab: int, temperature, top_k, top_p, seeds, steps, n_top: int = 0,
                          group=None, world: int = 1):
    """``sample`` over vocab-sharded logits (tensor parallelism): ``local`` is this rank's
    f32 [R, Vl] slice starting at global token ``vstart``.  Exchanges per-row statistics,
    top-k/top-p histograms and candidates instead of the logit rows (sampling.hip), and
    returns the same (tokens, logprobs, top_ids, top_lps) on every rank."""
    import torch.distributed as dist
    R = local.shape[0]
    if _gpu(local):
        dev = local.device
        h = hip()
        local = local.float().contiguous()
        stats = torch.empty(R * 4, dtype=torch.float32, device=dev)
        h.tp_sample_stats(local, vstart, stats)
        stats_all = torch.empty(world * R * 4, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(stats_all, stats, group=group)
        hist = torch.empty(R * 2 * 1024, dtype=torch.int64, device=dev)
        h.tp_sample_hist(local, vocab, temperature, top_k, top_p, stats_all, world, hist)
        dist.all_reduce(hist, group=group)
        cw = 3 + 2 * n_top
        cand = torch.empty(R * cw, dtype=torch.float32, device=dev)
        h.tp_sample_pick(local, vstart, vocab, temperature, top_k, top_p, seeds, steps, stats_all, world, hist,
                         n_top, cand)
        cand_all = torch.empty(world * R * cw, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(cand_all, cand, group=group)
        tok = torch.empty(R, dtype=torch.int32, device=dev)
        lp = torch.empty(R, dtype=torch.float32, device=dev)
        ti = torch.empty(R * max(n_top, 1), dtype=torch.int32, device=dev)
        tl = torch.empty(R * max(n_top, 1), dtype=torch.float32, device=dev)
        h.tp_sample_final(stats_all, cand_all, world, R, temperature, n_top, tok, lp, ti, tl)
        if n_top:
            return tok, lp, ti.view(R, n_top), tl.view(R, n_top)
        return tok, lp, None, None
    # CPU (gloo): exact greedy tokens, log-probs and top-n from exchanged row statistics;
    # rows that sample gather their full logit rows and use the reference sampler.
    lf = local.float()
    mx, am = lf.max(dim=-1)
    lse = torch.logsumexp(lf, dim=-1)
    st = torch.stack([mx, (am + vstart).double().float(), lse], -1).contiguous()
    parts = [torch.empty_like(st) for _ in range(world)]
    dist.all_gather(parts, st, group=group)
    allst = torch.stack(parts)                                  # [W, R, 3]
    logZ = torch.logsumexp(allst[..., 2], dim=0)
    w_best = allst[..., 0].argmax(dim=0)                        # first rank wins ties = lower index
    rr = torch.arange(R)
    tok = allst[w_best, rr, 1].round().long()
    lp = allst[w_best, rr, 0] - logZ
    sampled = (temperature.float() > 0).cpu()
    if bool(sampled.any()):
        idx = sampled.nonzero()[:, 0]
        rows = lf.index_select(0, idx).contiguous()
        rparts = [torch.empty_like(rows) for _ in range(world)]
        dist.all_gather(rparts, rows, group=group)
        full = torch.cat(rparts, -1)[:, :vocab]
        t2, l2, _, _ = sample(full, temperature[idx], top_k[idx], top_p[idx], seeds[idx], steps[idx])
        tok[idx] = t2.long()
        lp[idx] = l2.float()
    ti = tl = None
    if n_top:
        v, i = torch.topk(lf, min(n_top, lf.shape[1]), dim=-1)
        c = torch.cat([v, (i + vstart).float()], -1).contiguous()
        cparts = [torch.empty_like(c) for _ in range(world)]
        dist.all_gather(cparts, c, group=group)
        k = v.shape[1]
        vs = torch.cat([p[:, :k] for p in cparts], -1)
        ids = torch.cat([p[:, k:] for p in cparts], -1)
        tv, pos = torch.topk(vs, n_top, dim=-1)
        ti = ids.gather(1, pos).round().int()
        tl = tv - logZ[:, None]
    return tok.int(), lp, ti, tl


def apply_logit_deltas(logits, rows, toks, delta):
    if _gpu(logits):
        hip().apply_logit_deltas(logits, rows, toks, delta)
    else:
        for r, t, d in zip(rows.tolist(), toks.tolist(), delta.tolist()):
            if 0 <= t < logits.shape[1]:
                logits[r, t] += d


# ---------------------------------------------------------------- embeddings / vectors
def pool_embeddings(x, start, length, mode: int, normalize: bool, out_dtype=torch.float32):
    if _gpu(x):
        out = torch.empty(start.numel(), x.shape[1], dtype=out_dtype, device=x.device)
        hip().pool_embeddings(out, x, start, length, mode, normalize)
        return out
    return ref.pool_embeddings(x, start, length, mode, normalize).to(out_dtype)


def l2_normalize_rows(x):
    if _gpu(x):
        out = torch.empty_like(x)
        hip().l2_normalize_rows(out, x)
        return out
    return torch.nn.functional.normalize(x.float(), dim=-1, eps=1e-12).to(x.dtype)


def knn_topk(X, Q, k: int, sample_chunks: Optional[int] = None, _ablate: int = 0):
    """Top-k rows of X by dot product with each query row.  Returns (scores f32 [Q,k], idx int32 [Q,k]).
    GPU: the first ``sample_chunks`` x 1024 rows are searched exactly and set a per-query
    threshold for the rest (0 = search every chunk exactly); ties go to the lower row."""
    if _gpu(X):
        Qn, N = Q.shape[0], X.shape[0]
        nchunks = (N + 1023) // 1024
        dev = X.device
        out_s = torch.empty(Qn, k, dtype=torch.float32, device=dev)
        out_i = torch.empty(Qn, k, dtype=torch.int32, device=dev)
        if sample_chunks is None:
            # large batches: a 16-chunk sample (the exact pass costs ~0.2 ms at Q = 1024 with
            # 32); the weaker threshold adds candidates the per-wave buffers absorb
            sample_chunks = 16 if Qn >= 1024 else 32
        ws_s = torch.empty(max(1, Qn * nchunks * k), dtype=torch.float32, device=dev)
        ws_i = torch.empty(Qn * nchunks * k + 3 * Qn, dtype=torch.int32, device=dev)
        if _ablate:   # tools/engine_bench.py --knn-ablate only: timing ablations, wrong results
            hip().knn_topk_ablate(X, Q, k, out_s, out_i, ws_s, ws_i, sample_chunks, _ablate)
            return out_s, out_i
        hip().knn_topk(X, Q, k, out_s, out_i, ws_s, ws_i, sample_chunks)
        if sample_chunks > 0 and nchunks > sample_chunks and bool(ws_i[-Qn:].any()):
            # a candidate list overflowed (many rows above the sample's K-th best): exact rerun
            hip().knn_topk(X, Q, k, out_s, out_i, ws_s, ws_i, 0)
        return out_s, out_i
    return ref.knn_topk(X, Q, k)
