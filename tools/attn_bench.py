"""Decode-attention timing over (batch, context) shapes + a correctness spot check.

usage (GPU box): python tools/attn_bench.py [--shapes 256x448,64x2048,8x4000]

"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from langstream_amd import ops  # noqa: E402
from langstream_amd.ops import reference as ref  # noqa: E402


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
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="256x448,256x410,256x1024,128x448,64x2048,16x4096,4x4096,1x4096")
    ap.add_argument("--check-all", action="store_true")
    ap.add_argument("--ragged", type=float, default=0.0,
                    help="per-sequence context drawn uniformly from ctx*(1 +- ragged) (mean ctx)")
    ap.add_argument("--ring", type=int, default=1,
                    help="rotate over this many KV pools per call (> 256 MB Infinity Cache in total: cold "
                         "caches, as in an engine step that streams 32 layers between two calls)")
    ap.add_argument("--interleave-copy", action="store_true",
                    help="copy 235 MB (the decode gate_up weight bytes, no MFMA) before every call: separates "
                         "the cache / TLB effect of an interleaved GEMM from its power / clock effect")
    ap.add_argument("--interleave-gemm", action="store_true",
                    help="run a decode-sized gate_up GEMM before every call (engine-like power / cache state); "
                         "time the attention kernel with rocprofv3 in this mode")
    ap.add_argument("--pool-gb", type=float, default=0.0,
                    help="scatter the blocks over a KV pool of this size (TLB reach), like a real engine")
    ap.add_argument("--uniform-lo", type=int, default=0,
                    help="per-sequence context drawn uniformly from [uniform-lo, ctx] (e.g. the RAG bench's "
                         "prompt lengths 201..502 plus the tokens generated so far)")
    ap.add_argument("--seq-blocks", action="store_true",
                    help="each sequence's blocks are consecutive ids (a fresh burst through the engine's "
                         "block allocator) instead of scattered over the pool")
    ap.add_argument("--sorted", action="store_true",
                    help="rows ordered by context length, longest first (as the engine schedules them)")
    ap.add_argument("--shared-first", type=int, default=0,
                    help="the first N blocks of every sequence are the SAME physical blocks (a template "
                         "prefix shared through the prefix cache)")
    ap.add_argument("--rope", action="store_true",
                    help="time the decode-only variant with RoPE + the KV write fused in "
                         "(paged_decode_attention_rope over an un-rotated qkv buffer, as the engine runs it)")
    a = ap.parse_args()
    Hq, Hkv, D = 32, 8, 128
    dev, bf = "cuda", torch.bfloat16
    nsplit, mbps = ops.decode_splits(64)
    for shp in a.shapes.split(","):
        B, ctx = (int(x) for x in shp.split("x"))
        g = torch.Generator(device="cpu").manual_seed(0)
        if a.ragged > 0:
            lo, hi = int(ctx * (1 - a.ragged)), int(ctx * (1 + a.ragged))
            ctxs = torch.randint(max(1, lo), hi + 1, (B,), generator=g)
        elif a.uniform_lo > 0:
            ctxs = torch.randint(a.uniform_lo, ctx + 1, (B,), generator=g)
        else:
            ctxs = torch.full((B,), ctx)
        if a.sorted:
            ctxs = ctxs.sort(descending=True).values
        nb = int((ctxs.max() + 63) // 64)
        # blocks scattered over a pool 2x the live size (like a busy engine), or --pool-gb
        blk_bytes = Hkv * 64 * D * 2 * 2
        pool = max(2 * B * nb, int(a.pool_gb * 1e9 // blk_bytes))
        perm = (torch.arange(B * nb) if a.seq_blocks else torch.randperm(pool, generator=g)[: B * nb]).to(torch.int32)
        bt = perm.view(B, nb).clone()
        if a.shared_first:
            bt[:, : a.shared_first] = bt[0, : a.shared_first]
        bt = bt.to(dev)
        if pool > 2 * B * nb:
            kc = torch.zeros(pool, Hkv, 64, D, device=dev, dtype=bf)
            vc = torch.zeros(pool, Hkv, 8, D, 8, device=dev, dtype=bf)
            idx = perm.long().to(dev)
            kc[idx] = torch.randn(len(idx), Hkv, 64, D, device=dev, dtype=bf)
            vc[idx] = torch.randn(len(idx), Hkv, 8, D, 8, device=dev, dtype=bf)
        else:
            kc = torch.randn(pool, Hkv, 64, D, device=dev, dtype=bf)
            vc = torch.randn(pool, Hkv, 8, D, 8, device=dev, dtype=bf)
        kvs = [(kc, vc)] + [(torch.randn_like(kc), torch.randn_like(vc)) for _ in range(a.ring - 1)]
        cl = ctxs.to(torch.int32).to(dev)
        q = torch.randn(B, Hq * D, device=dev, dtype=bf)
        ws = torch.empty(B * Hq * nsplit * (D + 2), device=dev, dtype=torch.float32)
        o = torch.empty(B, Hq * D, device=dev, dtype=bf)
        scale = 1 / math.sqrt(D)
        it = [0]
        if a.interleave_copy:
            csrc = torch.empty(235 * 2 ** 20 // 2, device=dev, dtype=bf)
            cdst = torch.empty_like(csrc)
        if a.interleave_gemm:
            gx = torch.randn(B, 4096, device=dev, dtype=bf)
            gw = torch.randn(28672, 4096, device=dev, dtype=bf) * 0.02

        if a.rope:
            qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev, dtype=bf)
            pos = (cl - 1).to(torch.int32)
            half = torch.arange(0, D // 2, device=dev, dtype=torch.float32)
            inv = 1.0 / (500000.0 ** (2 * half / D))
            ang = torch.arange(0, 8192, device=dev, dtype=torch.float32)[:, None] * inv[None, :]
            cos_sin = torch.cat([ang.cos(), ang.sin()], dim=1).contiguous()
            # the new token's cache slot: its position inside the sequence's last block
            lastblk = bt.gather(1, ((cl.long() - 1) // 64).view(-1, 1)).view(-1).long()
            slots = lastblk * 64 + (cl.long() - 1) % 64

        def call():
            if a.interleave_gemm:
                torch.nn.functional.linear(gx, gw)
            if a.interleave_copy:
                cdst.copy_(csrc)
            k_, v_ = kvs[it[0] % len(kvs)]
            it[0] += 1
            if a.rope:
                ops.hip().paged_decode_attention_rope(o, qkv, pos, cos_sin, slots, k_, v_, bt, cl, scale, nsplit,
                                                      mbps, ws)
            else:
                ops.hip().paged_decode_attention(o, q, k_, v_, bt, cl, scale, nsplit, mbps, ws)
        us = timeit(call)
        if not a.rope:
            ops.hip().paged_decode_attention(o, q, kc, vc, bt, cl, scale, nsplit, mbps, ws)
        byts = int(ctxs.sum()) * Hkv * D * 2 * 2
        rec = {"B": B, "ctx": ctx, "us": round(us, 2), "TBps": round(byts / us / 1e6, 2),
               "kernel": "decode_attn_kernel", "wpp": os.environ.get("LS_ATTN_WPP", "auto"),
               "pipe": os.environ.get("LS_ATTN_PIPE", "1"),
               "ragged": a.ragged, "pool_gb": a.pool_gb, "ring": a.ring, "rope": a.rope,
               "uniform_lo": a.uniform_lo, "sorted": a.sorted, "seq_blocks": a.seq_blocks,
               "shared_first": a.shared_first, "nt": os.environ.get("LS_ATTN_NT", "2"),
               "interleave_gemm": a.interleave_gemm}
        if not a.rope and (B <= 16 or (a.check_all and B * ctx <= 512 * 1024)) and a.pool_gb == 0:
            exp = ref.paged_decode_attention(q.float().cpu().reshape(B, Hq, D), kc.float().cpu(), vc.float().cpu(),
                                             bt.cpu(), cl.cpu(), scale).reshape(B, Hq * D)
            rec["max_err"] = round(float((o.float().cpu() - exp).abs().max()), 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
