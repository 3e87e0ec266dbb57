"""Numerics of every HIP kernel against the plain-PyTorch fp32 reference (ops.reference).

All tests here need a real gfx950 GPU and the in-tree ``_hip_ops.so``; the ops layer
raises (never falls back) when the extension is missing, so a pass here means the
native kernels ran.
"""
import math

import pytest
import torch

from langstream_amd import ops
from langstream_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = err > tol
    assert not bad.any(), f"{msg} max err {err.max().item():.4g} at {bad.nonzero()[:5].tolist()}"


def test_extension_loaded():
    assert ops.hip_available(), "native _hip_ops.so must load on the GPU box"


@pytest.mark.parametrize("H", [384, 4096, 8192])
def test_rmsnorm(H):
    torch.manual_seed(0)
    x = torch.randn(37, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    _close(ops.rmsnorm(x, w, 1e-5), ref.rmsnorm(x.cpu(), w.cpu(), 1e-5), 0.05, 0.02)


def test_fused_add_rmsnorm():
    torch.manual_seed(1)
    x = torch.randn(19, 4096, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(19, 4096, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(4096, device=DEV, dtype=torch.bfloat16)
    xc, rc = x.cpu().clone(), r.cpu().clone()
    ops.fused_add_rmsnorm(x, r, w, 1e-5)
    ref.fused_add_rmsnorm(xc, rc, w.cpu(), 1e-5)
    _close(r, rc, 0.02, 0.01, "residual")
    _close(x, xc, 0.05, 0.02, "normed")


def test_layernorm_bias_residual():
    torch.manual_seed(2)
    x = torch.randn(50, 384, device=DEV, dtype=torch.bfloat16)
    res = torch.randn_like(x)
    bias, g, b = (torch.randn(384, device=DEV, dtype=torch.bfloat16) for _ in range(3))
    got = ops.layernorm(x, g, b, 1e-12, bias=bias, residual=res)
    exp = ref.layernorm(x.cpu(), bias.cpu(), res.cpu(), g.cpu(), b.cpu(), 1e-12)
    _close(got, exp, 0.05, 0.02)


def test_embed_layernorm():
    torch.manual_seed(3)
    V, P, H = 1000, 512, 384
    wte = torch.randn(V, H, device=DEV, dtype=torch.bfloat16)
    wpe = torch.randn(P, H, device=DEV, dtype=torch.bfloat16)
    wtt = torch.randn(2, H, device=DEV, dtype=torch.bfloat16)
    g, b = torch.randn(H, device=DEV, dtype=torch.bfloat16), torch.randn(H, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, V, (77,), device=DEV, dtype=torch.int32)
    pos = torch.randint(0, P, (77,), device=DEV, dtype=torch.int32)
    tt = torch.randint(0, 2, (77,), device=DEV, dtype=torch.int32)
    got = ops.embed_layernorm(ids, pos, tt, wte, wpe, wtt, g, b, 1e-12)
    exp = ref.embed_layernorm(ids.cpu(), pos.cpu(), tt.cpu(), wte.cpu(), wpe.cpu(), wtt.cpu(), g.cpu(), b.cpu(), 1e-12)
    _close(got, exp, 0.05, 0.02)


def test_silu_mul_and_gelu():
    torch.manual_seed(4)
    x = torch.randn(33, 2 * 1536, device=DEV, dtype=torch.bfloat16)
    _close(ops.silu_and_mul(x), ref.silu_and_mul(x.cpu()), 0.02, 0.02)
    y = torch.randn(33, 1536, device=DEV, dtype=torch.bfloat16)
    bias = torch.randn(1536, device=DEV, dtype=torch.bfloat16)
    exp = ref.bias_gelu(y.cpu(), bias.cpu())
    _close(ops.bias_gelu_(y, bias), exp, 0.02, 0.02)


def _alloc_cache(nb, Hkv, D, dev):
    return ops.new_kv_cache(nb, Hkv, D, dev, torch.bfloat16)


@pytest.mark.parametrize("T,D", [(150, 128), (2600, 128), (37, 64)])
def test_rope_and_cache(T, D):
    # T <= 2048 takes the decode-sized 2-token tiles, larger T the 16-token tiles
    torch.manual_seed(5)
    Hq, Hkv = 8, 2
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.arange(T, device=DEV, dtype=torch.int32) + 7
    cs = ref.rope_cos_sin(4096, D, 500000.0, device=DEV)
    nb = (T + ops.KV_BLOCK - 1) // ops.KV_BLOCK + 4
    perm = torch.randperm(nb * ops.KV_BLOCK)[:T]
    slots = perm.to(DEV, torch.int64)
    slots[3] = -1
    kc, vc = _alloc_cache(nb, Hkv, D, DEV)
    kr, vr = _alloc_cache(nb, Hkv, D, "cpu")
    qkv_c = qkv.cpu().clone()
    ops.rope_and_cache(qkv, pos, cs, slots, kc, vc, Hq, Hkv)
    ref.rope_and_cache(qkv_c, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq, Hkv)
    _close(qkv, qkv_c, 0.03, 0.01, "qkv")
    _close(kc, kr, 0.03, 0.01, "k cache")
    _close(vc, vr, 0.0, 0.0, "v cache")


def _random_paged(B, ctx, Hkv, D, dev, seed=0):
    torch.manual_seed(seed)
    nblk = [(c + ops.KV_BLOCK - 1) // ops.KV_BLOCK for c in ctx]
    NB = sum(nblk) + 3
    kc = torch.randn(NB, Hkv, ops.KV_BLOCK, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(NB, Hkv, ops.KV_BLOCK // 8, D, 8, device=dev, dtype=torch.bfloat16)
    perm = torch.randperm(NB)
    maxb = max(nblk)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    k = 0
    for b in range(B):
        for i in range(nblk[b]):
            bt[b, i] = perm[k]
            k += 1
    return kc, vc, bt.to(dev)


@pytest.mark.parametrize("G", [4, 8])
@pytest.mark.parametrize("nsplit,min_bps", [(1, 4), (3, 4), (3, 1), (16, 1)])
def test_paged_decode_attention(G, nsplit, min_bps):
    Hkv, D = 2, 128
    Hq = Hkv * G
    ctx = [1, 63, 64, 65, 300, 777]
    B = len(ctx)
    kc, vc, bt = _random_paged(B, ctx, Hkv, D, DEV, seed=G)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    q = qkv[:, : Hq * D]
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    ws = torch.empty(B * Hq * nsplit * (D + 2), device=DEV, dtype=torch.float32)
    got = ops.paged_decode_attention(q, kc, vc, bt, cl, scale, nsplit=nsplit, blocks_per_split=min_bps, workspace=ws)
    exp = ref.paged_decode_attention(q.cpu().reshape(B, Hq, D), kc.cpu(), vc.cpu(), bt.cpu(), cl.cpu(), scale)
    _close(got, exp.reshape(B, Hq * D), 0.03, 0.03)


@pytest.mark.parametrize("B,sort", [(256, False), (257, True)])
def test_paged_decode_attention_wave_per_pair(B, sort):
    """B*Hkv >= 2048 takes the one-wave-per-(seq, kv-head) kernel; ragged contexts
    exercise the masked tail-block loads (rows in arrival order, and sorted longest
    first as the engine schedules them, at an odd batch)."""
    Hkv, G, D = 8, 4, 128
    Hq = Hkv * G
    gen = torch.Generator().manual_seed(7)
    ctx = torch.randint(1, 300, (B,), generator=gen).tolist()
    if sort:
        ctx.sort(reverse=True)
    B = len(ctx)
    kc, vc, bt = _random_paged(B, ctx, Hkv, D, DEV, seed=3)
    q = torch.randn(B, Hq * D, device=DEV, dtype=torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    got = ops.paged_decode_attention(q, kc, vc, bt, cl, scale, nsplit=1)
    exp = ref.paged_decode_attention(q.cpu().reshape(B, Hq, D), kc.cpu(), vc.cpu(), bt.cpu(), cl.cpu(), scale)
    _close(got, exp.reshape(B, Hq * D), 0.03, 0.03)


def _rope_decode_case(ctx, Hkv, G, D, seed):
    Hq = Hkv * G
    B = len(ctx)
    kc, vc, bt = _random_paged(B, ctx, Hkv, D, DEV, seed=seed)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    pos = (cl - 1).clamp(min=0)
    btc = bt.cpu()
    slots = torch.tensor([int(btc[b, (c - 1) // ops.KV_BLOCK]) * ops.KV_BLOCK + (c - 1) % ops.KV_BLOCK if c > 0 else -1
                          for b, c in enumerate(ctx)], dtype=torch.int64, device=DEV)
    cs = ref.rope_cos_sin(4096, D, 500000.0, device=DEV)
    return Hq, kc, vc, bt, qkv, cl, pos, slots, cs


@pytest.mark.parametrize("ctx,Hkv,G,nsplit,min_bps", [
    ([1, 2, 63, 64, 65, 66, 129, 300, 777], 2, 4, 1, 4),
    ([1, 2, 63, 64, 65, 66, 129, 300, 777], 2, 4, 3, 1),
    ([1, 65, 129, 777], 2, 8, 16, 1),
    ("ragged256", 8, 4, 1, 4),
])
def test_paged_decode_attention_rope(ctx, Hkv, G, nsplit, min_bps):
    """Fused RoPE + KV write + decode attention == rope_and_cache, then attention over
    the cache (fp32 reference); the new token's K / V^T land in the cache."""
    D = 128
    if ctx == "ragged256":   # B*Hkv >= 2048: one wave per (seq, kv-head)
        ctx = torch.randint(1, 300, (256,), generator=torch.Generator().manual_seed(11)).tolist()
    Hq, kc, vc, bt, qkv, cl, pos, slots, cs = _rope_decode_case(ctx, Hkv, G, D, seed=G + nsplit)
    B = len(ctx)
    kr, vr = kc.cpu().clone(), vc.cpu().clone()
    qkv_c = qkv.cpu().clone()
    ref.rope_and_cache(qkv_c, pos.cpu(), cs.cpu(), slots.cpu(), kr, vr, Hq, Hkv)
    exp = ref.paged_decode_attention(qkv_c[:, : Hq * D].reshape(B, Hq, D), kr, vr, bt.cpu(), cl.cpu(),
                                     1 / math.sqrt(D))
    qkv_before = qkv.clone()
    ws = torch.empty(B * Hq * nsplit * (D + 2), device=DEV, dtype=torch.float32)
    got = ops.paged_decode_attention_rope(qkv, pos, cs, slots, kc, vc, bt, cl, 1 / math.sqrt(D), Hq,
                                          nsplit=nsplit, blocks_per_split=min_bps, workspace=ws)
    _close(got, exp.reshape(B, Hq * D), 0.03, 0.03, "attention")
    _close(kc, kr, 0.03, 0.01, "k cache")
    _close(vc, vr, 0.0, 0.0, "v cache")
    assert torch.equal(qkv, qkv_before), "the fused kernel must not modify the projection rows"


@pytest.mark.parametrize("G", [1, 4, 8])
def test_paged_prefill_attention(G):
    Hkv, D = 2, 128
    Hq = Hkv * G
    q_lens = [1, 17, 64, 130, 200]
    prefix = [0, 5, 64, 0, 300]
    ctx = [a + b for a, b in zip(q_lens, prefix)]
    B = len(q_lens)
    kc, vc, bt = _random_paged(B, ctx, Hkv, D, DEV, seed=10 + G)
    T = sum(q_lens)
    q = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    starts = [0]
    for n in q_lens[:-1]:
        starts.append(starts[-1] + n)
    qs = torch.tensor(starts, dtype=torch.int32, device=DEV)
    ql = torch.tensor(q_lens, dtype=torch.int32, device=DEV)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    tiles = ops.prefill_tiles(q_lens, G, prefix).to(DEV)
    scale = 1 / math.sqrt(D)
    got = ops.paged_prefill_attention(q, kc, vc, bt, qs, ql, cl, tiles, Hq, scale)
    exp = ref.paged_prefill_attention(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), qs.cpu(), ql.cpu(), cl.cpu(), Hq, scale)
    _close(got, exp, 0.03, 0.03)


@pytest.mark.parametrize("D,H", [(32, 12), (64, 4)])
def test_encoder_attention(D, H):
    torch.manual_seed(20)
    lens = [3, 64, 65, 200, 512]
    T = sum(lens)
    qkv = torch.randn(T, 3 * H * D, device=DEV, dtype=torch.bfloat16)
    starts = [0]
    for n in lens[:-1]:
        starts.append(starts[-1] + n)
    qs = torch.tensor(starts, dtype=torch.int32, device=DEV)
    ql = torch.tensor(lens, dtype=torch.int32, device=DEV)
    tiles = ops.prefill_tiles(lens, 1).to(DEV)
    scale = 1 / math.sqrt(D)
    got = ops.varlen_encoder_attention(qkv, qs, ql, tiles, H, H, scale)
    exp = ref.varlen_encoder_attention(qkv.cpu(), qs.cpu(), ql.cpu(), H, H, scale)
    _close(got, exp, 0.03, 0.03)


def test_sampling_greedy_and_logprobs():
    torch.manual_seed(30)
    B, V = 7, 128256
    logits = torch.randn(B, V, device=DEV) * 3
    temp = torch.zeros(B, device=DEV)
    topk = torch.zeros(B, dtype=torch.int32, device=DEV)
    topp = torch.ones(B, device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.int64)
    steps = torch.zeros(B, device=DEV, dtype=torch.int64)
    tok, lp, ti, tl = ops.sample(logits, temp, topk, topp, seeds, steps, n_top=3)
    assert torch.equal(tok.cpu().long(), logits.argmax(-1).cpu())
    exp_lp = torch.log_softmax(logits.float(), -1).gather(1, tok.long()[:, None])[:, 0]
    _close(lp, exp_lp, 1e-3, 1e-4)
    v, i = torch.topk(torch.log_softmax(logits.float(), -1), 3, -1)
    assert torch.equal(ti.cpu().long(), i.cpu())
    _close(tl, v, 1e-3, 1e-4)


def test_sampling_distribution_topk():
    # temperature sampling restricted to top-k: samples must stay inside the top-k set and
    # roughly follow the renormalised softmax
    torch.manual_seed(31)
    B, V = 4096, 1000
    base = torch.randn(V) * 2
    logits = base.to(DEV).repeat(B, 1)
    temp = torch.full((B,), 0.8, device=DEV)
    topk = torch.full((B,), 5, dtype=torch.int32, device=DEV)
    topp = torch.ones(B, device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.int64)
    steps = torch.zeros(B, device=DEV, dtype=torch.int64)
    tok, _, _, _ = ops.sample(logits, temp, topk, topp, seeds, steps)
    allowed = set(torch.topk(base, 5).indices.tolist())
    got = tok.cpu().tolist()
    assert set(got) <= allowed
    p = torch.softmax(base[list(sorted(allowed))] / 0.8, 0)
    freq = torch.tensor([got.count(t) for t in sorted(allowed)], dtype=torch.float32) / B
    assert (freq - p).abs().max() < 0.05


def test_sampling_top_p():
    torch.manual_seed(32)
    B, V = 2048, 500
    base = torch.randn(V) * 3
    logits = base.to(DEV).repeat(B, 1)
    temp = torch.ones(B, device=DEV)
    topk = torch.zeros(B, dtype=torch.int32, device=DEV)
    topp = torch.full((B,), 0.5, device=DEV)
    seeds = torch.arange(B, device=DEV, dtype=torch.int64) + 99
    steps = torch.ones(B, device=DEV, dtype=torch.int64)
    tok, _, _, _ = ops.sample(logits, temp, topk, topp, seeds, steps)
    probs = torch.softmax(base, 0)
    sp, si = torch.sort(probs, descending=True)
    keep = set(si[: int(((torch.cumsum(sp, 0) - sp) < 0.5).sum()) + 1].tolist())
    assert set(tok.cpu().tolist()) <= keep


def test_penalties():
    logits = torch.zeros(2, 10, device=DEV)
    rows = torch.tensor([0, 1, 1], dtype=torch.int32, device=DEV)
    toks = torch.tensor([3, 4, 9], dtype=torch.int32, device=DEV)
    d = torch.tensor([-1.0, 2.0, 0.5], device=DEV)
    ops.apply_logit_deltas(logits, rows, toks, d)
    assert logits[0, 3].item() == -1.0 and logits[1, 4].item() == 2.0 and logits[1, 9].item() == 0.5


@pytest.mark.parametrize("mode", [0, 1])
def test_pooling(mode):
    torch.manual_seed(40)
    lens = [1, 7, 100]
    x = torch.randn(sum(lens), 384, device=DEV, dtype=torch.bfloat16)
    st = torch.tensor([0, 1, 8], dtype=torch.int32, device=DEV)
    ln = torch.tensor(lens, dtype=torch.int32, device=DEV)
    got = ops.pool_embeddings(x, st, ln, mode, True)
    exp = ref.pool_embeddings(x.cpu(), st.cpu(), ln.cpu(), mode, True)
    _close(got, exp, 2e-3, 1e-2)


@pytest.mark.parametrize("N,Qn,k,dup", [(5000, 3, 20, 0), (1024, 20, 5, 0), (10, 2, 20, 0), (70000, 40, 64, 0),
                                         (100000, 17, 20, 0), (4096, 5, 20, 7), (3000, 4, 64, 50),
                                         (200000, 256, 20, 0), (50000, 64, 64, 3)])
def test_knn_topk(N, Qn, k, dup):
    """dup > 0 stores only `dup` distinct rows (massive score ties): exercises the
    K-round fallback behind the threshold + wave-sort fast path."""
    torch.manual_seed(50)
    X = torch.nn.functional.normalize(torch.randn(N, 384), dim=-1)
    if dup:
        X = X[torch.arange(N) % dup]
    X = X.to(DEV, torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(Qn, 384), dim=-1).to(DEV, torch.bfloat16)
    s, i = ops.knn_topk(X, Q, k)
    es, ei = ref.knn_topk(X.cpu(), Q.cpu(), k)
    # scores must match the reference ranking (ties between near-equal scores may reorder)
    valid = es > -1e30
    _close(torch.where(valid, s.cpu(), torch.zeros_like(s.cpu())), torch.where(valid, es, torch.zeros_like(es)), 2e-3)
    # every returned index must have the score we report
    for q in range(Qn):
        for j in range(k):
            if i[q, j] >= 0:
                sc = (X[i[q, j].long()].float() @ Q[q].float()).item()
                assert abs(sc - s[q, j].item()) < 2e-3
            else:
                assert not valid[q, j]


@pytest.mark.parametrize("N,Qn,D,k,dup", [(300000, 1024, 384, 20, 0), (300000, 2048, 384, 20, 0),
                                           (100000, 2048, 512, 10, 0), (50000, 1500, 256, 64, 0),
                                           (100000, 700, 128, 20, 0), (60000, 300, 384, 20, 5)])
def test_knn_topk_large_q(N, Qn, D, k, dup):
    """The large-batch main pass (knn_filter_q256_kernel: 256 queries per workgroup, rows
    through an LDS-DMA ring, per-wave LDS candidate buffers) against an fp32 top-k of the
    same bf16 operands on the GPU; dup > 0 (massive ties) overflows the per-wave buffers
    and the candidate lists and takes the exact rerun."""
    torch.manual_seed(N + Qn + D)
    X = torch.nn.functional.normalize(torch.randn(N, D, device=DEV), dim=-1)
    if dup:
        X = X[torch.arange(N, device=DEV) % dup]
    X = X.to(torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(Qn, D, device=DEV), dim=-1).to(torch.bfloat16)
    s, i = ops.knn_topk(X, Q, k)
    full = Q.float() @ X.float().t()
    es, _ = full.topk(k, dim=1)
    assert (s - es).abs().max().item() < 2e-3
    assert (i >= 0).all()
    got = full.gather(1, i.long())
    assert (got - s).abs().max().item() < 2e-3
    # no row twice in one answer
    srt = i.sort(dim=1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()
    del full


@pytest.mark.parametrize("N,Qn,dup", [(140_000, 300, 0), (140_000, 2048, 70_000), (200_000, 1024, 0)])
def test_knn_group_max_threshold_path_equals_exact(N, Qn, dup, monkeypatch):
    """Q >= 128 over >= 64k rows: thresholds from the group-max sample pass
    (knn_filter_q256_kernel MODE 2 + knn_group_thr_kernel) and a non-strict filter over
    the whole store give the same answers, ties included (dup: every row twice), as the
    exact-sample path and the all-exact search."""
    torch.manual_seed(N + Qn)
    X = torch.nn.functional.normalize(torch.randn(N, 384, device=DEV), dim=-1)
    if dup:
        X = X[torch.arange(N, device=DEV) % dup]
    X = X.to(torch.bfloat16)
    Q = torch.nn.functional.normalize(torch.randn(Qn, 384, device=DEV), dim=-1).to(torch.bfloat16)
    s, i = ops.knn_topk(X, Q, 20)
    s0, i0 = ops.knn_topk(X, Q, 20, sample_chunks=0)
    assert torch.equal(s, s0) and torch.equal(i, i0)
    monkeypatch.setenv("LS_KNN_EXACT_SAMPLE", "1")
    s1, i1 = ops.knn_topk(X, Q, 20)
    assert torch.equal(s1, s0) and torch.equal(i1, i0)


def test_knn_topk_threshold_overflow_and_exact():
    """Rows get MORE similar to the queries further into the store, so the sample's
    K-th best is a weak threshold: candidate lists overflow and the search reruns
    exactly.  Also: the sampled and the all-exact searches return identical answers."""
    torch.manual_seed(51)
    N, D, k = 120_000, 384, 20
    q = torch.nn.functional.normalize(torch.randn(3, D), dim=-1)
    alpha = torch.linspace(0, 1, N).unsqueeze(1)
    X = torch.nn.functional.normalize(alpha * q[torch.arange(N) % 3] + 0.5 * torch.randn(N, D), dim=-1)
    X = X.to(DEV, torch.bfloat16)
    Q = q.to(DEV, torch.bfloat16)
    s, i = ops.knn_topk(X, Q, k)
    es, ei = ref.knn_topk(X.cpu(), Q.cpu(), k)
    _close(s.cpu(), es, 2e-3)
    Q2 = torch.nn.functional.normalize(torch.randn(100, D), dim=-1).to(DEV, torch.bfloat16)
    s1, i1 = ops.knn_topk(X, Q2, k)
    s0, i0 = ops.knn_topk(X, Q2, k, sample_chunks=0)
    assert torch.equal(s1, s0) and torch.equal(i1, i0)


@pytest.mark.parametrize("M", [1, 37, 64, 256])
@pytest.mark.parametrize("N,K", [(384, 512), (1024, 4096), (256, 8192)])  # (256, 8192): split-K 16
def test_skinny_gemm(M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.hip().skinny_gemm(out, x, w)
    exp = x.float().cpu() @ w.float().cpu().t()
    _close(out, exp, 0.03, 0.03)


@pytest.mark.parametrize("M", [3, 64, 200])
def test_skinny_gemm_silu(M):
    K, F = 512, 320
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    ops.hip().skinny_gemm_silu(out, x, w)
    gu = x.float().cpu() @ w.float().cpu().t()
    exp = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    _close(out, exp, 0.03, 0.03)


@pytest.mark.parametrize("M", [1, 300, 2048, 3000])
@pytest.mark.parametrize("N,K", [(256, 64), (768, 1024), (512, 2080)])
def test_gemm_prefill(M, N, K):
    """256x256-tile prefill GEMM (gemm_prefill.hip) vs fp32: M tails, K not a multiple of
    the ring depth, several N tiles per group."""
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    assert ops.hip().gemm_prefill_supported(w, False)
    out = ops.gemm_prefill(x, w)
    _close(out, x.float().cpu() @ w.float().cpu().t(), 0.02, 0.02)


@pytest.mark.parametrize("M,F,K", [(77, 128, 256), (1000, 384, 1024), (4096, 256, 512)])
def test_gemm_prefill_silu(M, F, K):
    """gate_up GEMM with the SwiGLU in the epilogue vs fp32 silu(x.g^T) * (x.u^T)."""
    torch.manual_seed(M + F)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    assert ops.hip().gemm_prefill_supported(w, True)
    out = ops.gemm_prefill(x, w, silu=True)
    gu = x.float().cpu() @ w.float().cpu().t()
    _close(out, torch.nn.functional.silu(gu[:, :F]) * gu[:, F:], 0.02, 0.02)


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("M", [1, 300, 2048, 3000, 70000])
@pytest.mark.parametrize("N,K", [(256, 128), (768, 1024), (512, 2048)])
def test_gemm_prefill_pingpong(M, N, K, variant):
    """The ping-pong prefill GEMM (gemm_pp_kernel, variant 1) vs fp32: M tails, several
    N tiles per group, the shortest K (one iteration of two K tiles)."""
    torch.manual_seed(M + N + K + 1)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = ops.gemm_prefill(x, w, variant=variant)
    _close(out, x.float() @ w.float().t(), 0.02, 0.02)


@pytest.mark.parametrize("M,N,K", [(300, 256, 8192), (1024, 256, 8320), (1024, 4096, 14336),
                                   (2048, 4096, 14336), (3000, 512, 8192)])
def test_gemm_prefill_pingpong_splitk(M, N, K):
    """Split-K on the ping-pong kernel (under-filled tile grids with K >= 8192: the
    Llama down projection at 1024-4095 tokens): S K-ranges of whole tile pairs, f32
    partial slabs, then the reduction -- vs fp32, M tails included."""
    torch.manual_seed(M + N + K + 7)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = ops.gemm_prefill(x, w, variant=1)
    _close(out, x.float() @ w.float().t(), 0.02, 0.02)


@pytest.mark.parametrize("M,N,K", [(1, 512, 256), (129, 2048, 1024), (200, 768, 4096), (256, 128256, 4096),
                                   (300, 1024, 512)])
def test_gemm_prefill_f32_output(M, N, K):
    """The ping-pong kernel's f32-output form (the LM head of 129..256-row decode batches)
    vs fp32, M tails included; N = 128256 is the Llama-3 vocabulary."""
    torch.manual_seed(M + N + K + 11)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.hip().gemm_prefill_f32(out, x, w)
    torch.cuda.synchronize()
    ref = x.float() @ w.float().t()
    assert torch.allclose(out, ref, atol=2e-3, rtol=2e-3), float((out - ref).abs().max())


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("M,F,K", [(77, 128, 256), (1000, 384, 1024), (4096, 256, 512), (40000, 640, 256)])
def test_gemm_prefill_pingpong_silu(M, F, K, variant):
    torch.manual_seed(M + F + 1)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = ops.gemm_prefill(x, w, silu=True, variant=variant)
    gu = x.float().cpu() @ w.float().cpu().t()
    _close(out, torch.nn.functional.silu(gu[:, :F]) * gu[:, F:], 0.02, 0.02)


@pytest.mark.parametrize("name,N,K,silu", [("qkv", 6144, 4096, False), ("o", 4096, 4096, False),
                                            ("gate_up", 28672, 4096, True), ("down", 4096, 14336, False)])
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_gemm_prefill_llama_shapes(name, N, K, silu, variant):
    """Llama-3-8B projection shapes at a ragged M = 16384 - 77 (edge M tile), against a
    fp32 GEMM of the same bf16 operands on the GPU (torch.matmul in fp32)."""
    M = 16384 - 77
    torch.manual_seed(N + K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = ops.gemm_prefill(x, w, silu=silu, variant=variant)
    ref = x.float() @ w.float().t()
    if silu:
        ref = torch.nn.functional.silu(ref[:, : N // 2]) * ref[:, N // 2:]
    err = (out.float() - ref).abs().max().item()
    assert err <= 0.03 * ref.abs().max().item() + 0.03, (name, err)
    del ref, out


@pytest.mark.parametrize("M,K,N", [(5, 1024, 512), (128, 1024, 512), (256, 4096, 4096), (256, 8192, 256)])
def test_skinny_gemm_add_rmsnorm(M, K, N):
    # split-K 2 / 2 / 8 (decode o_proj shape) / 16 (past the reduction's unrolled 8)
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    res_exp = res.float().cpu() + x.float().cpu() @ w.float().cpu().t()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.hip().skinny_gemm_add_rmsnorm(out, x, w, res, g, 1e-5)
    _close(res, res_exp, 0.03, 0.03)
    exp = res_exp * torch.rsqrt(res_exp.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float().cpu()
    _close(out, exp, 0.05, 0.05)


@pytest.mark.parametrize("T,N,K", [(1, 6144, 4096), (2, 4096, 4096), (3, 512, 1536), (4, 4096, 14336),
                                   (1, 4096, 14336), (2, 1024, 3584)])
def test_gemv(T, N, K):
    torch.manual_seed(T * 7 + K)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    out = torch.empty(T, N, device=DEV, dtype=torch.bfloat16)
    ops.hip().gemv(out, x, w)
    exp = x.float().cpu() @ w.float().cpu().t()
    _close(out, exp, 0.03, 0.03)


@pytest.mark.parametrize("T,F,K", [(1, 14336, 4096), (3, 1024, 2048), (4, 512, 14336)])
def test_gemv_silu(T, F, K):
    torch.manual_seed(T + F)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) * 0.05).to(torch.bfloat16)
    out = torch.empty(T, F, device=DEV, dtype=torch.bfloat16)
    ops.hip().gemv_silu(out, x, w)
    gu = (x.float().cpu() @ w.float().cpu().t()).to(torch.bfloat16).float()
    exp = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    _close(out, exp, 0.03, 0.03)


@pytest.mark.parametrize("T,N,K", [(1, 4096, 4096), (2, 4096, 14336), (4, 1024, 2048)])
def test_gemv_add_rmsnorm(T, N, K):
    torch.manual_seed(T + N + K)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    res = torch.randn(T, N, device=DEV).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    ticket = torch.zeros(1, dtype=torch.int32, device=DEV)
    for rep in range(3):   # the ticket word must come back to 0 after every launch
        r = res.clone()
        out = torch.empty(T, N, device=DEV, dtype=torch.bfloat16)
        ops.hip().gemv_add_rmsnorm(out, x, w, r, nw, 1e-5, ticket)
        o = (x.float().cpu() @ w.float().cpu().t()).to(torch.bfloat16).float()
        er = (o + res.float().cpu()).to(torch.bfloat16).float()
        eo = er * torch.rsqrt(er.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float().cpu()
        _close(r, er, 0.03, 0.02)
        _close(out, eo, 0.03, 0.03)
        assert int(ticket.item()) == 0


@pytest.mark.parametrize("silu", [False, True])
@pytest.mark.parametrize("T,N,K", [(1, 6144, 4096), (3, 1024, 2048), (4, 512, 14336)])
def test_gemv_prologue_norm(silu, T, N, K):
    torch.manual_seed(T + N + K + silu)
    o = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    res = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    nw = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    res_out = torch.empty_like(res)
    out = torch.empty(T, N // 2 if silu else N, device=DEV, dtype=torch.bfloat16)
    (ops.hip().gemv_silu_norm if silu else ops.hip().gemv_norm)(out, o, res, res_out, nw, 1e-5, w)
    er = (o.float().cpu() + res.float().cpu()).to(torch.bfloat16).float()
    x = (er * torch.rsqrt(er.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float().cpu()).to(torch.bfloat16).float()
    y = x @ w.float().cpu().t()
    if silu:
        y = y.to(torch.bfloat16).float()
        y = torch.nn.functional.silu(y[:, : N // 2]) * y[:, N // 2:]
    _close(res_out, er, 0.02, 0.01)
    _close(out, y, 0.05, 0.03)


@pytest.mark.parametrize("T,K,prologue", [(1, 4096, False), (3, 2048, True), (2, 14336, False)])
def test_gemv_qkv_rope_cache(T, K, prologue):
    # qkv GEMV with RoPE + paged K / V^T cache writes in the epilogue vs a PyTorch fp32 chain
    torch.manual_seed(T * 5 + K)
    Hq, Hkv, D, BS, NB = 4, 2, 128, 64, 6
    N = (Hq + 2 * Hkv) * D
    w = (torch.randn(N, K, device=DEV) * 0.05).to(torch.bfloat16)
    x = torch.randn(T, K, device=DEV).to(torch.bfloat16)
    pos = torch.tensor([5, 77, 300, 9][:T], dtype=torch.int32, device=DEV)
    slots = torch.tensor([3, 64 + 10, -1, 200][:T], dtype=torch.int64, device=DEV)
    inv = 1.0 / (500000.0 ** (torch.arange(0, D, 2).float() / D))
    ang = torch.arange(512).float()[:, None] * inv[None]
    cos_sin = torch.cat([ang.cos(), ang.sin()], 1).to(DEV)
    kc = torch.zeros(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, BS // 8, D, 8, device=DEV, dtype=torch.bfloat16)
    out = torch.empty(T, N, device=DEV, dtype=torch.bfloat16)
    if prologue:
        o, res = x, torch.randn(T, K, device=DEV).to(torch.bfloat16)
        nw = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
        res_out = torch.empty_like(res)
        ops.hip().gemv_qkv(out, x, w, pos, cos_sin, slots, kc, vc, Hq, Hkv, True, o, res, res_out, nw, 1e-5)
        er = (o.float().cpu() + res.float().cpu()).to(torch.bfloat16).float()
        xin = (er * torch.rsqrt(er.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float().cpu()).to(torch.bfloat16).float()
        _close(res_out, er, 0.02, 0.01)
    else:
        ops.hip().gemv_qkv(out, x, w, pos, cos_sin, slots, kc, vc, Hq, Hkv, True, None, None, None, None, 1e-5)
        xin = x.float().cpu()
    y = (xin @ w.float().cpu().t()).to(torch.bfloat16).float().view(T, Hq + 2 * Hkv, D)
    cs = cos_sin.cpu()[pos.long().cpu()]
    c, s = cs[:, None, : D // 2], cs[:, None, D // 2:]
    qk = y[:, : Hq + Hkv]
    a, b = qk[..., : D // 2], qk[..., D // 2:]
    rot = torch.cat([a * c - b * s, b * c + a * s], -1)
    exp = torch.cat([rot, y[:, Hq + Hkv:]], 1)
    _close(out.view(T, -1, D), exp, 0.05, 0.02)
    kcc, vcc = kc.float().cpu(), vc.float().cpu()
    for t in range(T):
        sl = int(slots[t])
        if sl < 0:
            continue
        blk, off = divmod(sl, BS)
        _close(kcc[blk, :, off], exp[t, Hq: Hq + Hkv], 0.05, 0.02)
        _close(vcc[blk, :, off // 8, :, off % 8], exp[t, Hq + Hkv:], 0.05, 0.02)


def _ln_stats(x):
    """Partial (sum, sumsq) per 64-column sub-tile of bf16 rows, as gemm_fused writes them."""
    o = x.float().view(x.shape[0], -1, 64)
    return torch.stack([o.sum(-1), (o * o).sum(-1)], -1).contiguous()


@pytest.mark.parametrize("M", [1, 37, 300, 2049])
@pytest.mark.parametrize("N,K", [(1152, 384), (384, 384), (1536, 384), (384, 1536), (128, 128)])
@pytest.mark.parametrize("mode", ["bias", "bias_gelu", "res_stats", "lnin_gelu", "resln_stats", "plain"])
def test_gemm_fused(M, N, K, mode):
    """Hand-written MFMA GEMM (gemm_fused.hip) with each epilogue vs the fp32 reference."""
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    kw = {}
    if mode != "plain":
        kw["bias"] = (0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    if mode == "bias_gelu":
        kw["gelu"] = True
    if mode in ("res_stats", "resln_stats"):
        kw["residual"] = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        kw["stats_out"] = torch.empty(M, N // 64, 2, device=DEV)
    if mode == "resln_stats":
        kw["ln_stats_in"] = _ln_stats(kw["residual"])
        kw["ln_width"] = N
        kw["res_g"] = (1 + 0.3 * torch.randn(N, device=DEV)).to(torch.bfloat16)
        kw["res_b"] = (0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
        kw["eps"] = 1e-12
    if mode == "lnin_gelu":
        g = 1 + 0.3 * torch.randn(K, device=DEV)
        b = 0.1 * torch.randn(K, device=DEV)
        x = (3.0 + 2.0 * torch.randn(M, K, device=DEV)).to(torch.bfloat16)   # un-normalised input
        wp = (w.float() * g[None]).to(torch.bfloat16)
        kw.update(ln_stats_in=_ln_stats(x), ln_width=K, c1=wp.float().sum(1).contiguous(),
                  c2=(w.float() @ b).contiguous(), gelu=True, eps=1e-12)
        # the fused result must equal LN(x) . W^T + bias (GELU'd) computed the plain way
        xn = torch.nn.functional.layer_norm(x.float(), (K,), g, b, 1e-12)
        exp = torch.nn.functional.gelu(xn @ w.float().t() + kw["bias"].float())
        got = ops.gemm_fused(x, wp, **kw)
        _close(got, exp, 0.03, 0.03, mode)
        return
    cpu = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in kw.items()}
    if "stats_out" in cpu:
        cpu["stats_out"] = torch.empty_like(cpu["stats_out"])
    exp = ref.gemm_fused(x.cpu(), w.cpu(), **cpu)
    got = ops.gemm_fused(x, w, **kw)
    _close(got, exp, 0.02, 0.02, mode)
    if "stats_out" in kw:
        _close(kw["stats_out"], cpu["stats_out"], 0.05, 0.01, "stats")


def test_bert_fused_layers_match_plain_fp32():
    """The fused encoder (4 GEMMs + attention per layer, LayerNorms folded) on the GPU
    vs the plain fp32 layer sequence on the CPU, with non-trivial LayerNorm params."""
    import os
    from langstream_amd.models.bert import BertEncoder, PRESETS
    cfg = PRESETS["bge-small-en"]
    gpu = BertEncoder(cfg, device=DEV, seed=4)
    with torch.no_grad():
        for l in gpu.layers:
            for n in ("ln1_g", "ln2_g"):
                getattr(l, n).copy_((1 + 0.2 * torch.randn(cfg.hidden_size, device=DEV)).to(torch.bfloat16))
            for n in ("ln1_b", "ln2_b", "o_b", "ff2_b"):
                getattr(l, n).copy_((0.05 * torch.randn(cfg.hidden_size, device=DEV)).to(torch.bfloat16))
    cpu = BertEncoder(cfg, device="cpu", dtype=torch.float32)
    cpu.load_state_dict({k: v.float().cpu() for k, v in gpu.state_dict().items()})
    toks = [[101] + list(range(2000, 2000 + n)) + [102] for n in (3, 60, 250, 17)]
    assert gpu.fused_supported()
    eg = gpu.encode_tokens(toks)
    os.environ["LS_BERT_FUSED"] = "0"
    try:
        ec = cpu.encode_tokens(toks)
    finally:
        os.environ.pop("LS_BERT_FUSED", None)
    cos = torch.nn.functional.cosine_similarity(eg.cpu(), ec, dim=-1)
    assert cos.min() > 0.995, cos


# Llama-3-70B at TP=8: the per-rank shard shapes the TP decode path runs:
# qkv 8192 -> 1280, o 1024 -> 8192, gate_up 8192 -> 2x3584, down 3584 -> 8192.
TP8_SHAPES = [("qkv", 1280, 8192), ("o", 8192, 1024), ("down", 8192, 3584)]


@pytest.mark.parametrize("M", [1, 4, 64, 256])
@pytest.mark.parametrize("name,N,K", TP8_SHAPES)
def test_tp8_shard_shapes_skinny_and_gemv(M, name, N, K):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    exp = x.float().cpu() @ w.float().cpu().t()
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    ops.hip().skinny_gemm(out, x, w)
    _close(out, exp, 0.03, 0.03, f"skinny {name}")
    if M <= 4 and ops.hip().gemv_supported(w, False):
        out2 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        ops.hip().gemv(out2, x, w)
        _close(out2, exp, 0.03, 0.03, f"gemv {name}")


@pytest.mark.parametrize("M", [1, 3, 64, 256])
def test_tp8_gate_up_shard_silu(M):
    F, K = 3584, 8192
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    gu = (x.float().cpu() @ w.float().cpu().t()).to(torch.bfloat16).float()
    exp = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    out = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
    ops.hip().skinny_gemm_silu(out, x, w)
    _close(out, exp, 0.03, 0.03, "skinny silu")
    if M <= 4 and ops.hip().gemv_supported(w, True):
        out2 = torch.empty(M, F, device=DEV, dtype=torch.bfloat16)
        ops.hip().gemv_silu(out2, x, w)
        _close(out2, exp, 0.03, 0.03, "gemv silu")


@pytest.mark.parametrize("W", [2, 3, 8])
def test_vocab_parallel_sampling_matches_single_gpu_sampler(W):
    """The four tp_sample_* phases (sampling.hip), run per vocabulary slice with the
    exchanges done in torch (all-gather = concatenation, all-reduce = sum), reproduce the
    single-GPU sampler on the full rows: greedy and seeded top-k / top-p tokens, token
    log-probs and the top-n alternatives."""
    torch.manual_seed(60 + W)
    R, V, n_top = 37, 32005, 5
    h = ops.hip()
    logits = (torch.randn(R, V) * 3).to(DEV)
    temp = torch.tensor([0.0, 0.7, 1.0, 1.3] * 10, dtype=torch.float32)[:R].to(DEV)
    top_k = torch.tensor([0, 40, 0, 1, 7] * 8, dtype=torch.int32)[:R].to(DEV)
    top_p = torch.tensor([1.0, 0.9, 0.5] * 13, dtype=torch.float32)[:R].to(DEV)
    seeds = torch.randint(0, 1 << 30, (R,), dtype=torch.int64).to(DEV)
    steps = torch.randint(0, 100, (R,), dtype=torch.int64).to(DEV)
    tok, lp, ti, tl = ops.sample(logits, temp, top_k, top_p, seeds, steps, n_top=n_top)
    per = (V + W - 1) // W
    sl = [(w * per, min(V, (w + 1) * per)) for w in range(W)]
    parts = [logits[:, a:b].contiguous() for a, b in sl]
    stats = []
    for (a, _), p in zip(sl, parts):
        st = torch.empty(R * 4, device=DEV)
        h.tp_sample_stats(p, a, st)
        stats.append(st)
    stats_all = torch.cat(stats)
    hist = torch.zeros(R * 2 * 1024, dtype=torch.int64, device=DEV)
    for p in parts:
        hh = torch.empty_like(hist)
        h.tp_sample_hist(p, V, temp, top_k, top_p, stats_all, W, hh)
        hist += hh
    cands = []
    for (a, _), p in zip(sl, parts):
        c = torch.empty(R * (3 + 2 * n_top), device=DEV)
        h.tp_sample_pick(p, a, V, temp, top_k, top_p, seeds, steps, stats_all, W, hist, n_top, c)
        cands.append(c)
    tok2 = torch.empty(R, dtype=torch.int32, device=DEV)
    lp2 = torch.empty(R, device=DEV)
    ti2 = torch.empty(R * n_top, dtype=torch.int32, device=DEV)
    tl2 = torch.empty(R * n_top, device=DEV)
    h.tp_sample_final(stats_all, torch.cat(cands), W, R, temp, n_top, tok2, lp2, ti2, tl2)
    assert torch.equal(tok.cpu(), tok2.cpu())
    assert (lp.cpu() - lp2.cpu()).abs().max() < 1e-4
    assert torch.equal(ti.cpu(), ti2.view(R, n_top).cpu())
    assert (tl.cpu() - tl2.view(R, n_top).cpu()).abs().max() < 1e-4


# ------------------------------------------------------------------ gemm_decode.hip
# Exact Llama-3-8B decode shapes (M = batch rows) and the Llama-3-70B TP=8 shard shapes,
# every tile width / split count the dispatcher can pick, against fp32.
_DG_SHAPES = [("qkv8b", 6144, 4096), ("o8b", 4096, 4096), ("down8b", 4096, 14336),
              ("qkv70b_tp8", 1280, 8192), ("o70b_tp8", 8192, 1024), ("down70b_tp8", 8192, 3584)]


def _dg_ws(M, N):
    return torch.empty(64 * M * N + 4 * 256 * 256, device=DEV, dtype=torch.float32)


# Every decode-GEMM test also proves which kernel variant ran: the dispatcher keeps a
# host-side launch census per (BN, epilogue, tile rows, K splits).  _dg_* mirror the
# dispatcher's routing rules (gemm_decode.hip pick_split / dgemm_launch / decode_gemm).
_DG_SMALL_M = [5, 17, 64, 100, 128]
_DG_ALL_M = _DG_SMALL_M + [129, 200, 256]


def _dg_split(tiles, K, min_steps=4):
    best = 1
    for s in range(1, 65):
        if tiles * s > 264 or (K // 64) // s < min_steps:
            break
        best = s
    return best


def _dg_bm(M, bn, epi):
    if bn == 128 and epi in ("store", "partial", "silu"):
        return 64 if M <= 64 else 128 if M <= 128 else 256
    return 256


def _dg_key(M, bn, epi, s):
    return f"bn{bn}_{epi}_bm{_dg_bm(M, bn, epi)}_s{min(s, 16)}"   # the census caps splits at 16


def _dg_census_reset():
    ops.hip().decode_gemm_launch_counts(True)


def _dg_census_check(*keys):
    got = dict(ops.hip().decode_gemm_launch_counts(True))
    assert got == {k: 1 for k in keys}, (got, keys)


@pytest.mark.parametrize("M", _DG_ALL_M)
@pytest.mark.parametrize("name,N,K", _DG_SHAPES)
@pytest.mark.parametrize("bn,splits", [(0, 0), (128, 1), (128, 5), (256, 3), (64, 0), (64, 3)])
def test_decode_gemm(M, name, N, K, bn, splits):
    if bn == 256 and N % 256:
        pytest.skip("N not a multiple of 256")
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    assert ops.hip().decode_gemm_supported(w, False)
    _dg_census_reset()
    ops.hip().decode_gemm(out, x, w, _dg_ws(M, N), None, None, 1e-5, bn, splits)
    bn_eff = bn or 128
    S = min(splits, K // 64) if splits else _dg_split(N // bn_eff, K)
    _dg_census_check(_dg_key(M, bn_eff, "store" if S == 1 else "partial", S))
    _close(out, x.float().cpu() @ w.float().cpu().t(), 0.02, 0.02, name)


@pytest.mark.parametrize("M", _DG_ALL_M)   # o8b above 128 rows: 64-column tiles, 4 K splits
@pytest.mark.parametrize("name,N,K", [("o8b", 4096, 4096), ("down8b", 4096, 14336), ("o70b_tp8", 8192, 1024),
                                      ("o70b", 8192, 8192), ("down70b", 8192, 28672)])
def test_decode_gemm_add_rmsnorm(M, name, N, K):
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    res_exp = (res.float() + x.float() @ w.float().t()).cpu()   # fp32 reference (gfx950 has no xf32)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    _dg_census_reset()
    ops.hip().decode_gemm(out, x, w, _dg_ws(M, N), res, g, 1e-5)
    bn = 64 if (K <= 4096 and M > 128) else 128
    _dg_census_check(_dg_key(M, bn, "partial", _dg_split(N // bn, K)))
    _close(res, res_exp, 0.03, 0.03, "residual")
    rb = res_exp.to(torch.bfloat16).float()
    exp = rb * torch.rsqrt(rb.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float().cpu()
    _close(out, exp, 0.05, 0.05, "normed")


@pytest.mark.parametrize("M", _DG_SMALL_M + [129, 256])
@pytest.mark.parametrize("F,K,splits", [(14336, 4096, 2), (14336, 4096, 1), (3584, 8192, 2), (3584, 8192, 1),
                                        (384, 1024, 2), (28672, 8192, 1)])
def test_decode_gemm_silu(M, F, K, splits):
    """gate_up + SwiGLU: the 2-way K split with the in-launch combine (ticket parity,
    release/acquire hand-off) and the single-launch form; repeated calls exercise the
    monotonic tickets (no per-call reset)."""
    torch.manual_seed(M + F)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    tickets = torch.zeros(2 * (F // 128), device=DEV, dtype=torch.int32)
    err = torch.zeros(1, device=DEV, dtype=torch.int32)
    ws = torch.empty((F // 128) * 256 * 256, device=DEV, dtype=torch.float32)
    gu = (x.float() @ w.float().t()).cpu()
    exp = torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]
    for _ in range(3):
        out = torch.full((M, F), float("nan"), device=DEV, dtype=torch.bfloat16)
        _dg_census_reset()
        ops.hip().decode_gemm_silu(out, x, w, ws, tickets, err, splits)
        _dg_census_check(_dg_key(M, 256, "silu2", 2) if splits == 2 else _dg_key(M, 128, "silu", 1))
        _close(out, exp, 0.02, 0.02)
    assert err.item() == 0


@pytest.mark.parametrize("M", _DG_SMALL_M + [129, 256])
@pytest.mark.parametrize("Hq,Hkv,K", [(32, 8, 4096), (8, 1, 8192), (64, 8, 8192)])   # 8B; 70B TP=8 shard; 70B
def test_decode_gemm_qkv_rope(M, Hq, Hkv, K):
    """qkv split-K GEMM with RoPE + the paged K/V write fused into its reduction, against
    an fp32 projection rotated in fp32 and the same rows in the caches; rows with slot -1
    are not cached."""
    torch.manual_seed(M + Hq + K)
    D, BS = 128, 64
    N = (Hq + 2 * Hkv) * D
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32)
    half = torch.arange(0, D // 2, dtype=torch.float64)
    inv = 1.0 / (500000.0 ** (2 * half / D))
    ang = torch.arange(0, 4096, dtype=torch.float64)[:, None] * inv[None, :]
    cos_sin = torch.cat([ang.cos(), ang.sin()], 1).float().to(DEV)
    NB = 2 * M
    kc = torch.zeros(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, BS // 8, D, 8, device=DEV, dtype=torch.bfloat16)
    slots = torch.randperm(NB * BS, device=DEV)[:M].long()
    slots[M // 2] = -1
    qkv = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    _dg_census_reset()
    ops.hip().decode_gemm_qkv_rope(qkv, x, w, _dg_ws(M, N), pos, cos_sin, slots, kc, vc, Hq, Hkv)
    S = min(4, _dg_split(N // 128, K))
    _dg_census_check(_dg_key(M, 128, "partial" if S > 1 else "store", S))
    y = (x.float() @ w.float().t()).view(M, Hq + 2 * Hkv, D)
    cs = cos_sin[pos.long()]                                  # [M, D]
    co, si = cs[:, None, : D // 2], cs[:, None, D // 2:]
    a, b = y[:, : Hq + Hkv, : D // 2], y[:, : Hq + Hkv, D // 2:]
    rot = torch.cat([a * co - b * si, b * co + a * si], -1)
    exp = torch.cat([rot, y[:, Hq + Hkv:]], 1)
    _close(qkv.view(M, -1, D), exp, 0.03, 0.03, "qkv")
    got = qkv.view(M, -1, D)
    for m in range(M):
        s = int(slots[m])
        if s < 0:
            continue
        blk, off = s // BS, s % BS
        assert torch.equal(kc[blk, :, off, :], got[m, Hq: Hq + Hkv]), m
        assert torch.equal(vc[blk, :, off // 8, :, off % 8], got[m, Hq + Hkv:]), m
    assert int((kc != 0).any(-1).sum()) == (M - 1) * Hkv


@pytest.mark.parametrize("M", _DG_SMALL_M + [129, 256])
@pytest.mark.parametrize("bn", [128, 256])
def test_decode_gemm_f32_lm_head(M, bn):
    """The decode LM head: f32 logits straight from the 256-row decode GEMM at the
    Llama-3 vocabulary (128256 = 1002 x 128 = 501 x 256), against fp32."""
    torch.manual_seed(M + bn)
    N, K = 128256, 4096
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    assert ops.hip().decode_gemm_f32_supported(w, M)
    out = torch.full((M, N), float("nan"), device=DEV)
    _dg_census_reset()
    ops.hip().decode_gemm_f32(out, x, w, bn)
    _dg_census_check(_dg_key(M, bn, "partial", 1))
    ref = x.float() @ w.float().t()
    assert (out - ref).abs().max().item() < 2e-3 * ref.abs().max().item() + 1e-3


# ------------------------------------------------------------------ norm-deferred decode layer
# gemm_decode.hip DgArgs: split-K combine inside the launch (rendezvous of a tile's K
# slices), y = bf16(h * g) + per-tile sums of h^2 from the producer, 1/rms applied by the
# consumer's epilogue.  Repeated calls exercise the monotonic 64-bit counters.
def _rms_ref(h, g, eps=1e-5):
    return h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps) * g


@pytest.mark.parametrize("M", _DG_ALL_M)
@pytest.mark.parametrize("name,N,K", [("o8b", 4096, 4096), ("down8b", 4096, 14336), ("o70b", 8192, 8192)])
def test_decode_gemm_res_combine(M, name, N, K):
    torch.manual_seed(M + N + K)
    S = ops.hip().decode_gemm_cmb_splits(N, K)
    assert S > 1 and (N // 128) * S <= 256
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    cnt = torch.zeros(N // 128, device=DEV, dtype=torch.int64)
    err = torch.zeros(1, device=DEV, dtype=torch.int32)
    ws = torch.empty(S * M * N, device=DEV, dtype=torch.float32)
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    for it in range(3):
        h_exp = (res.float() + x.float() @ w.float().t()).to(torch.bfloat16)
        y = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        ss = torch.full((M, N // 128), float("nan"), device=DEV)
        ops.hip().decode_gemm_res(y, x, w, ws, cnt, res, g, ss, err)
        torch.cuda.synchronize()
        _close(res, h_exp.float().cpu(), 0.03, 0.03, f"residual it{it}")
        hf = res.float()
        _close(y, (hf * g.float()).cpu(), 0.01, 0.01, "y")
        assert torch.allclose(ss.sum(1), hf.pow(2).sum(1), rtol=1e-3), "sumsq"
        assert torch.allclose(ss[:, 3], hf[:, 384:512].pow(2).sum(1), rtol=1e-3)
    assert err.item() == 0 and int(cnt[0]) == 3 * S


@pytest.mark.parametrize("M", [129, 256])
@pytest.mark.parametrize("F,K", [(14336, 4096), (3584, 1024)])
def test_decode_gemm_silu_r(M, F, K):
    """gate_up on y = h * g with the producer's per-tile sums of h^2: silu(r g) * (r u)
    equals SwiGLU of the RMS-normed input."""
    torch.manual_seed(M + F)
    h = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    gnorm = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
    w = (torch.randn(2 * F, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    y = (h.float() * gnorm.float()).to(torch.bfloat16)
    parts = h.float().pow(2).view(M, K // 128, 128).sum(-1).contiguous()
    out = torch.full((M, F), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.hip().decode_gemm_silu_r(out, y, w, parts, 1e-5)
    xn = _rms_ref(h.float(), gnorm.float())
    gu = xn @ w.float().t()
    _close(out, torch.nn.functional.silu(gu[:, :F]) * gu[:, F:], 0.03, 0.03)


@pytest.mark.parametrize("M", [129, 256])
@pytest.mark.parametrize("Hq,Hkv,K", [(32, 8, 4096), (64, 8, 8192)])   # Llama-3-8B; Llama-3-70B at TP=1
def test_decode_gemm_qkv_combine(M, Hq, Hkv, K):
    """qkv on y = h * g: in-launch combine, 1/rms from the producer's partials, RoPE,
    paged K / V write (slot -1 rows not cached), against fp32 rmsnorm -> projection ->
    rotation."""
    torch.manual_seed(M + Hq + K)
    D, BS = 128, 64
    N = (Hq + 2 * Hkv) * D
    S = ops.hip().decode_gemm_cmb_splits(N, K)
    assert S >= 1
    h = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    gnorm = (1 + 0.1 * torch.randn(K, device=DEV)).to(torch.bfloat16)
    y = (h.float() * gnorm.float()).to(torch.bfloat16)
    parts = h.float().pow(2).view(M, K // 128, 128).sum(-1).contiguous()
    w = (torch.randn(N, K, device=DEV) / K ** 0.5).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32)
    half = torch.arange(0, D // 2, dtype=torch.float64)
    inv = 1.0 / (500000.0 ** (2 * half / D))
    ang = torch.arange(0, 4096, dtype=torch.float64)[:, None] * inv[None, :]
    cos_sin = torch.cat([ang.cos(), ang.sin()], 1).float().to(DEV)
    NB = 2 * M
    kc = torch.zeros(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros(NB, Hkv, BS // 8, D, 8, device=DEV, dtype=torch.bfloat16)
    slots = torch.randperm(NB * BS, device=DEV)[:M].long()
    slots[M // 2] = -1
    cnt = torch.zeros(N // 128, device=DEV, dtype=torch.int64)
    err = torch.zeros(1, device=DEV, dtype=torch.int32)
    ws = torch.empty(S * M * N, device=DEV, dtype=torch.float32)
    xn = _rms_ref(h.float(), gnorm.float())
    yp = (xn @ w.float().t()).view(M, Hq + 2 * Hkv, D)
    cs = cos_sin[pos.long()]
    co, si = cs[:, None, : D // 2], cs[:, None, D // 2:]
    a, b = yp[:, : Hq + Hkv, : D // 2], yp[:, : Hq + Hkv, D // 2:]
    exp = torch.cat([torch.cat([a * co - b * si, b * co + a * si], -1), yp[:, Hq + Hkv:]], 1)
    for _ in range(2):
        qkv = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
        ops.hip().decode_gemm_qkv_cmb(qkv, y, w, ws, cnt, parts, 1e-5, pos, cos_sin, slots, kc, vc, Hq, Hkv, err)
        _close(qkv.view(M, -1, D), exp, 0.03, 0.03, "qkv")
    got = qkv.view(M, -1, D)
    for m in range(0, M, 7):
        s = int(slots[m])
        if s < 0:
            continue
        blk, off = s // BS, s % BS
        assert torch.equal(kc[blk, :, off, :], got[m, Hq: Hq + Hkv]), m
        assert torch.equal(vc[blk, :, off // 8, :, off % 8], got[m, Hq + Hkv:]), m
    assert err.item() == 0


def test_rms_prep_and_rows_rms_scale():
    torch.manual_seed(3)
    M, N = 200, 4096
    h = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    y = torch.empty_like(h)
    ss = torch.empty(M, 1, device=DEV)
    ops.hip().rms_prep(y, ss, h, g)
    assert torch.allclose(ss[:, 0], h.float().pow(2).sum(1), rtol=1e-4)
    _close(y, (h.float() * g.float()).cpu(), 0.01, 0.01)
    out = torch.empty_like(h)
    ops.hip().rows_rms_scale(out, y, ss, 1e-5)
    _close(out, _rms_ref(h.float(), g.float()).cpu(), 0.02, 0.02)
