"""Paged prefill attention (ops.paged_prefill_attention) at the RAG bench's prompt mix:
a 16384-token chunk of whole prompts with lengths drawn from the bench's spread (201-508,
mean ~347), Llama-3-8B heads (32 q / 8 kv, D 128), causal; also uniform lengths.
Reports time per call and the attention FLOP rate (causal: 2 * 2 * sum(L^2)/2 * D * Hq),
and checks one case against the fp32 reference op.

usage: python tools/prefill_attn_bench.py [--chunk 16384] [--iters 20]
"""
import argparse
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from langstream_amd import ops
from langstream_amd.ops import reference as ref


def build(lens, Hq=32, Hkv=8, D=128, BS=64, dev="cuda"):
    T = sum(lens)
    nblk = sum((n + BS - 1) // BS for n in lens)
    kc = torch.randn(nblk, Hkv, BS, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(nblk, Hkv, BS // 8, D, 8, device=dev).to(torch.bfloat16)
    maxb = max((n + BS - 1) // BS for n in lens)
    bt = torch.zeros(len(lens), maxb, dtype=torch.int32)
    b = 0
    for s, n in enumerate(lens):
        for j in range((n + BS - 1) // BS):
            bt[s, j] = b
            b += 1
    q = torch.randn(T, Hq * D, device=dev).to(torch.bfloat16)
    starts = [0]
    for n in lens[:-1]:
        starts.append(starts[-1] + n)
    i32 = dict(dtype=torch.int32, device=dev)
    meta = dict(block_tables=bt.to(dev), q_start=torch.tensor(starts, **i32), q_len=torch.tensor(lens, **i32),
                ctx_len=torch.tensor(lens, **i32), tiles=ops.prefill_tiles(lens, Hq // Hkv).to(dev))
    return q, kc, vc, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunk", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    rng = random.Random(0)
    Hq, D = 32, 128
    scale = D ** -0.5
    mixes = {}
    lens, tot = [], 0
    while True:
        n = rng.randint(201, 508)
        if tot + n > a.chunk:
            break
        lens.append(n)
        tot += n
    mixes["bench_mix"] = lens
    for L in (256, 512, 1024, 4096):
        mixes[f"uniform_{L}"] = [L] * (a.chunk // L)
    for name, lens in mixes.items():
        q, kc, vc, m = build(lens)
        out = ops.paged_prefill_attention(q, kc, vc, m["block_tables"], m["q_start"], m["q_len"], m["ctx_len"],
                                          m["tiles"], Hq, scale)
        err = None
        if name == "bench_mix":
            sub = 4   # check the first sequences against the fp32 reference
            r = ref.paged_prefill_attention(q[: sum(lens[:sub])].float().cpu(), kc.float().cpu(), vc.float().cpu(),
                                            m["block_tables"][:sub].cpu(), m["q_start"][:sub].cpu(),
                                            m["q_len"][:sub].cpu(), m["ctx_len"][:sub].cpu(), Hq, scale)
            err = float((out[: sum(lens[:sub])].float().cpu() - r).abs().max())
        torch.cuda.synchronize()
        for _ in range(3):
            ops.paged_prefill_attention(q, kc, vc, m["block_tables"], m["q_start"], m["q_len"], m["ctx_len"],
                                        m["tiles"], Hq, scale, out=out)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            ops.paged_prefill_attention(q, kc, vc, m["block_tables"], m["q_start"], m["q_len"], m["ctx_len"],
                                        m["tiles"], Hq, scale, out=out)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t) / a.iters * 1e6
        flops = sum(2 * 2 * (n * (n + 1) / 2) * D * Hq for n in lens)
        print(json.dumps({"mix": name, "seqs": len(lens), "tokens": sum(lens), "us": round(us, 1),
                          "TFLOPs": round(flops / us / 1e6, 1), "max_abs_err_vs_fp32": err}), flush=True)


if __name__ == "__main__":
    main()
