"""Decode-shaped GEMMs: hipBLASLt (F.linear + the separate elementwise kernel) vs the
hand-written skinny MFMA GEMM with fused epilogues (ops/csrc/gemm_skinny.hip).

Weights rotate through a ring of copies larger than the 256 MB Infinity Cache, as in a
real decode step that streams all 32 layers.  usage (GPU): python tools/gemm_skinny_bench.py
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


def timeit(fn, n, iters=40):
    for i in range(4):
        fn(i % n)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for i in range(iters):
        fn(i % n)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="16,64,128,256")
    ap.add_argument("--only", default="", help="comma list of gemm names (qkv,o,gate_up,down)")
    ap.add_argument("--skinny-only", action="store_true", help="time only the skinny kernel (profiling)")
    a = ap.parse_args()
    H, Fi = 4096, 14336
    dev, bf = "cuda", torch.bfloat16
    h = ops.hip()
    shapes = {"qkv": (6144, H), "o": (H, H), "gate_up": (2 * Fi, H), "down": (H, Fi)}
    for name, (N, K) in shapes.items():
        if a.only and name not in a.only.split(","):
            continue
        ring = max(2, int(1.2e9 // (N * K * 2)))
        ws = [(torch.randn(N, K, device=dev) * 0.02).to(bf) for _ in range(ring)]
        for M in (int(v) for v in a.ms.split(",")):
            x = torch.randn(M, K, device=dev).to(bf)
            res = torch.randn(M, N, device=dev).to(bf)
            g = torch.ones(N, device=dev, dtype=bf)
            if name == "gate_up":
                out = torch.empty(M, Fi, device=dev, dtype=bf)
                base = 0.0 if a.skinny_only else timeit(lambda i: h.silu_and_mul(out, F.linear(x, ws[i])), ring)
                new = timeit(lambda i: h.skinny_gemm_silu(out, x, ws[i]), ring)
            elif name in ("o", "down"):
                out = torch.empty(M, N, device=dev, dtype=bf)
                base = 0.0 if a.skinny_only else timeit(
                    lambda i: h.fused_add_rmsnorm(F.linear(x, ws[i]), res, g, 1e-5), ring)
                new = timeit(lambda i: h.skinny_gemm_add_rmsnorm(out, x, ws[i], res, g, 1e-5), ring)
            else:
                out = torch.empty(M, N, device=dev, dtype=bf)
                base = 0.0 if a.skinny_only else timeit(lambda i: F.linear(x, ws[i]), ring)
                new = timeit(lambda i: h.skinny_gemm(out, x, ws[i]), ring)
            wbytes = N * K * 2
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(base, 1),
                              "skinny_us": round(new, 1), "speedup": round(base / new, 2),
                              "skinny_weight_TBps": round(wbytes / new / 1e6, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
