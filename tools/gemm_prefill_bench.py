"""Prefill / encoder GEMM shapes: hipBLASLt (F.linear, + the separate epilogue kernel
the engine runs after it) vs the hand-written MFMA GEMM (ops.gemm) with fused
epilogues.  Random uniform operands (zero-filled operands read high on MFMA).

usage (GPU): python tools/gemm_prefill_bench.py [--ms 4096,16384] [--only gate_up,...] [--ours [--big]]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = {  # name: (N, K, epilogue)
    "llama_qkv": (6144, 4096, "none"),
    "llama_o": (4096, 4096, "none"),
    "llama_gate_up": (28672, 4096, "swiglu"),
    "llama_down": (4096, 14336, "none"),
    "bert_qkv": (1152, 384, "bias"),
    "bert_o": (384, 384, "bias_res"),
    "bert_ff1": (1536, 384, "bias_gelu"),
    "bert_ff2": (384, 1536, "bias_res"),
}


def timeit(fn, iters=20):
    for _ in range(3):
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
    ap.add_argument("--ms", default="2048,8192,16384")
    ap.add_argument("--only", default="")
    ap.add_argument("--ours", action="store_true", help="also time ops.gemm (hand-written)")
    ap.add_argument("--big", action="store_true",
                    help="llama shapes: time ops.gemm_prefill (256x256 tiles, SwiGLU epilogue) as 'ours'")
    a = ap.parse_args()
    from langstream_amd import ops
    dev = "cuda"
    only = set(filter(None, a.only.split(",")))
    for M in [int(x) for x in a.ms.split(",")]:
        for name, (N, K, epi) in SHAPES.items():
            if only and name not in only:
                continue
            x = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
            b = torch.rand(N, device=dev).bfloat16() if epi.startswith("bias") else None
            res = torch.rand(M, N, device=dev).bfloat16() if epi == "bias_res" else None
            flops = 2.0 * M * N * K
            if epi == "swiglu":
                def lib():
                    gu = F.linear(x, w)
                    ops.silu_and_mul(gu)
            elif epi == "bias_gelu":
                def lib():
                    h = F.linear(x, w)
                    ops.bias_gelu_(h, b)
            else:
                def lib():
                    F.linear(x, w, b)
            t_lib = timeit(lib)
            row = {"M": M, "gemm": name, "N": N, "K": K, "epi": epi, "hipblaslt_us": round(t_lib, 1),
                   "hipblaslt_tflops": round(flops / t_lib / 1e6, 1)}
            if a.ours:
                kw = {}
                if epi == "swiglu":
                    kw["act"] = "swiglu"
                elif epi == "bias_gelu":
                    kw.update(bias=b, act="gelu")
                elif epi == "bias":
                    kw.update(bias=b)
                elif epi == "bias_res":
                    kw.update(bias=b, residual=res)
                big = a.big and name.startswith("llama")
                fn = (lambda: ops.gemm_prefill(x, w, silu=epi == "swiglu")) if big else (lambda: ops.gemm(x, w, **kw))
                out = fn()
                ref = F.linear(x.float(), w.float(), None if b is None else b.float())
                if epi == "swiglu":
                    g, u = ref.chunk(2, -1)
                    ref = F.silu(g) * u
                elif epi == "bias_gelu":
                    ref = F.gelu(ref)
                elif epi == "bias_res":
                    ref = ref + res.float()
                err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                t_ours = timeit(fn)
                row.update(ours_us=round(t_ours, 1), ours_tflops=round(flops / t_ours / 1e6, 1),
                           speedup=round(t_lib / t_ours, 3), rel_err=round(err, 5))
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
