"""Small-batch decode GEMV (ops/csrc/gemm_gemv.hip) vs hipBLASLt on the Llama-3-8B
projections, cache-cold (weights cycled through a ring larger than the Infinity Cache).

usage (GPU box): python tools/gemv_bench.py [--ts 1,2,4]
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

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
          "down": (4096, 14336, False)}


def timed(fn, ring, iters=4):
    for w in ring[:2]:
        fn(w)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        for w in ring:
            fn(w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / (iters * len(ring))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ts", default="1,2,4")
    args = ap.parse_args()
    h = ops.hip()
    dev = torch.device("cuda:0")
    for name, (N, K, silu) in SHAPES.items():
        copies = max(4, int(768e6 // (N * K * 2)) + 1)
        ring = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        for T in [int(t) for t in args.ts.split(",")]:
            x = torch.randn(T, K, device=dev).to(torch.bfloat16)
            out = torch.empty(T, N // 2 if silu else N, device=dev, dtype=torch.bfloat16)
            if silu:
                def base(w):
                    gu = F.linear(x, w)
                    ops.silu_and_mul(gu, out=out)
                def mine(w):
                    h.gemv_silu(out, x, w)
            else:
                def base(w):
                    F.linear(x, w)
                def mine(w):
                    h.gemv(out, x, w)
            b, g = timed(base, ring), timed(mine, ring)
            gb = N * K * 2 / 1e9
            row = {"gemm": name, "T": T, "N": N, "K": K, "hipblaslt_us": round(b, 1), "gemv_us": round(g, 1),
                   "speedup": round(b / g, 2), "gemv_TBps": round(gb / g * 1e3, 2)}
            if K <= 4096:
                # prologue-fused form (input = rmsnorm(o + res) * norm_w, computed in the kernel)
                o_, res = torch.randn(T, K, device=dev).to(torch.bfloat16), torch.randn(T, K, device=dev).to(torch.bfloat16)
                res_out, nw = torch.empty_like(res), torch.ones(K, device=dev, dtype=torch.bfloat16)
                fn = h.gemv_silu_norm if silu else h.gemv_norm
                p = timed(lambda w: fn(out, o_, res, res_out, nw, 1e-5, w), ring)
                row.update(pro_us=round(p, 1), pro_TBps=round(gb / p * 1e3, 2))
            print(json.dumps(row), flush=True)
        del ring


if __name__ == "__main__":
    sys.exit(main())
