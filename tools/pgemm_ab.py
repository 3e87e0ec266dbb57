"""Prefill GEMM A/B on the Llama-3-8B projection shapes: hipBLASLt (+ the separate
silu_and_mul the engine runs after it for gate_up) vs gemm_prefill variants 0 (32-deep
ring) and 1 (ping-pong).  Random uniform operands; every variant checked against an fp32
GEMM first; all variants timed interleaved in one process (rounds x variants, median).

usage (GPU): python tools/pgemm_ab.py [--ms 2048,16384] [--only gate_up] [--variants 0,1]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from langstream_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
          "down": (4096, 14336, False)}


def time_it(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="2048,16384")
    ap.add_argument("--only", default="")
    ap.add_argument("--variants", default="1,3")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    dev = "cuda"
    for M in (int(v) for v in a.ms.split(",")):
        for name, (N, K, silu) in SHAPES.items():
            if a.only and name not in a.only.split(","):
                continue
            x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
            out = torch.empty(M, N // 2 if silu else N, device=dev, dtype=torch.bfloat16)
            var = {}
            if silu:
                def lib():
                    gu = F.linear(x, w)
                    ops.hip().silu_and_mul(out, gu)
            else:
                def lib():
                    torch.matmul(x, w.t(), out=out)
            var["hipblaslt"] = lib
            for v in (int(s) for s in a.variants.split(",")):
                var[f"pgemm_v{v}"] = (lambda v=v: ops.gemm_prefill(x, w, silu=silu, out=out, variant=v))
            ref = x.float() @ w.float().t()
            if silu:
                ref = F.silu(ref[:, : N // 2]) * ref[:, N // 2:]
            errs = {}
            for k, fn in var.items():
                out.zero_()
                fn()
                torch.cuda.synchronize()
                errs[k] = round(((out.float() - ref).abs().max() / ref.abs().max()).item(), 4)
            del ref
            flops = 2.0 * M * N * K
            iters = max(3, int(2e13 // flops))
            for fn in var.values():
                time_it(fn, 2)
            ts = {k: [] for k in var}
            for _ in range(a.rounds):
                for k, fn in var.items():
                    ts[k].append(time_it(fn, iters))
            us = {k: round(statistics.median(t), 1) for k, t in ts.items()}
            print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "us": us,
                              "tflops": {k: round(flops / t / 1e6, 1) for k, t in us.items()},
                              "rel_err": errs}), flush=True)


if __name__ == "__main__":
    main()
