"""Per-op timing of one Llama-3-8B decode layer at batch B (HIP events, GPU only).

Prints one JSON line per op with microseconds and achieved HBM bandwidth, plus the
modelled per-step total (x num_layers) -- used to find which decode op is far from
its roofline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from langstream_amd import ops  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=512)
    ap.add_argument("--blas", default="", help="'rocblas' or 'hipblaslt' (torch preferred BLAS library)")
    a = ap.parse_args()
    if a.blas:
        torch.backends.cuda.preferred_blas_library(a.blas)
    B, ctx = a.batch, a.ctx
    H, Fi, Hq, Hkv, D, L = 4096, 14336, 32, 8, 128, 32
    dev = "cuda"
    bf = torch.bfloat16
    x = torch.randn(B, H, device=dev, dtype=bf)
    res = []

    def rec(name, us, bytes_):
        res.append({"op": name, "us": round(us, 2), "GBps": round(bytes_ / us / 1e3, 1)})

    for name, n, k in (("qkv", (Hq + 2 * Hkv) * D, H), ("o", H, Hq * D), ("gate_up", 2 * Fi, H), ("down", H, Fi)):
        w = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        inp = torch.randn(B, k, device=dev, dtype=bf)
        rec(f"linear_{name}", timeit(lambda: F.linear(inp, w)), n * k * 2 + B * (n + k) * 2)
    gu = torch.randn(B, 2 * Fi, device=dev, dtype=bf)
    out = torch.empty(B, Fi, device=dev, dtype=bf)
    rec("silu_and_mul", timeit(lambda: ops.hip().silu_and_mul(out, gu)), B * Fi * 6)
    r = torch.randn(B, H, device=dev, dtype=bf)
    w = torch.ones(H, device=dev, dtype=bf)
    rec("fused_add_rmsnorm", timeit(lambda: ops.hip().fused_add_rmsnorm(x, r, w, 1e-5)), B * H * 2 * 4)
    # attention + rope over a paged cache
    nb = (ctx + 63) // 64
    nblocks = B * nb
    kc = torch.randn(nblocks, Hkv, 64, D, device=dev, dtype=bf)
    vc = torch.randn(nblocks, Hkv, 8, D, 8, device=dev, dtype=bf)
    bt = torch.arange(nblocks, device=dev, dtype=torch.int32).view(B, nb)
    ctx_l = torch.full((B,), ctx, device=dev, dtype=torch.int32)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev, dtype=bf)
    pos = torch.full((B,), ctx - 1, device=dev, dtype=torch.int32)
    slots = (bt[:, -1].long() * 64 + (ctx - 1) % 64)
    cs = torch.randn(8192, D, device=dev, dtype=torch.float32)
    rec("rope_and_cache", timeit(lambda: ops.hip().rope_and_cache(qkv, pos, cs, slots, kc, vc, Hq, Hkv, True)),
        B * (Hq + 2 * Hkv) * D * 2 * 2)
    nsplit, bps = ops.decode_splits(64)
    ws = torch.empty(B * Hq * nsplit * (D + 2), device=dev, dtype=torch.float32)
    q = qkv[:, : Hq * D]
    o = torch.empty(B, Hq * D, device=dev, dtype=bf)
    rec("decode_attention", timeit(lambda: ops.hip().paged_decode_attention(o, q, kc, vc, bt, ctx_l, 0.088, nsplit,
                                                                            min(bps, nb), ws)),
        B * ctx * Hkv * D * 2 * 2)
    per_layer = sum(r_["us"] for r_ in res)
    for r_ in res:
        print(json.dumps(r_))
    print(json.dumps({"per_layer_us": round(per_layer, 1), "per_step_ms_est": round(per_layer * L / 1000, 2),
                      "batch": B, "ctx": ctx}))


if __name__ == "__main__":
    main()
