"""Time the Llama-3-8B projection GEMMs (out = x @ W^T, bf16) at decode and prefill M,
with hipBLASLt's default heuristic and after PyTorch TunableOp tuning, and write the
tuned solutions to ``langstream_amd/ops/tunableop_gfx950.csv``.

usage (GPU box): python tools/gemm_tune.py [--ms 64,128,256] [--no-tune]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "langstream_amd", "ops", "tunableop_gfx950.csv")

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,8,32,64,128,192,256,4096,16384")
    ap.add_argument("--no-tune", action="store_true")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    args = ap.parse_args()
    ms = [int(x) for x in args.ms.split(",")]
    dev = torch.device("cuda:0")
    ws = {k: torch.randn(*SHAPES[k], device=dev).to(torch.bfloat16) * 0.02 for k in args.shapes.split(",")}
    rows = []
    for name, w in ws.items():
        N, K = w.shape
        for M in ms:
            if name == "lm_head" and M > 256:
                continue
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            us = timeit(lambda: F.linear(x, w))
            rows.append({"gemm": name, "M": M, "N": N, "K": K, "default_us": round(us, 1)})
    if not args.no_tune:
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_filename(OUT, insert_device_ordinal=False)
        tun.set_max_tuning_duration(300)
        tun.set_max_tuning_iterations(60)
        for r in rows:
            w = ws[r["gemm"]]
            x = torch.randn(r["M"], r["K"], device=dev).to(torch.bfloat16)
            F.linear(x, w)
            torch.cuda.synchronize()
        tun.tuning_enable(False)
        print(json.dumps({'tuned': [list(map(str, r)) for r in tun.get_results()]}), flush=True)
        for r in rows:
            w = ws[r["gemm"]]
            x = torch.randn(r["M"], r["K"], device=dev).to(torch.bfloat16)
            r["tuned_us"] = round(timeit(lambda: F.linear(x, w)), 1)
    for r in rows:
        flop = 2.0 * r["M"] * r["N"] * r["K"]
        byts = 2.0 * (r["N"] * r["K"] + r["M"] * r["K"] + r["M"] * r["N"])
        best = min(r["default_us"], r.get("tuned_us", 1e30))
        r["TFLOPs"] = round(flop / best / 1e6, 1)
        r["TBps"] = round(byts / best / 1e6, 2)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    sys.exit(main())
