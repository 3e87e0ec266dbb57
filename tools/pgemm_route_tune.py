"""Measure the prefill routing table: hipBLASLt (F.linear) vs the hand-written
gemm_prefill (gemm_pp_kernel) for the plain Llama projections over 256-row M buckets.

usage (GPU): python tools/pgemm_route_tune.py [--out gpurun_out/pgemm_route_gfx950.csv]
then copy the CSV to langstream_amd/ops/pgemm_route_gfx950.csv (loaded at import).
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from langstream_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336)}   # Llama-3-8B


def timeit(fn, iters):
    for _ in range(2):
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
    ap.add_argument("--out", default="gpurun_out/pgemm_route_gfx950.csv")
    ap.add_argument("--m-min", type=int, default=1024)
    ap.add_argument("--m-max", type=int, default=16640)
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    dev = "cuda"
    with open(a.out, "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(["N", "K", "M", "lib_us", "pp_us"])
        for name, (N, K) in SHAPES.items():
            w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).bfloat16()
            xa = (torch.rand(a.m_max, K, device=dev) * 2 - 1).bfloat16()
            out = torch.empty(a.m_max, N, device=dev, dtype=torch.bfloat16)
            for M in range(a.m_min, a.m_max + 1, 256):
                x = xa[:M]
                o = out[:M]
                # interleaved repeats, median: single timings jitter by up to 40 % at some M
                libs, pps = [], []
                for _ in range(a.reps):
                    libs.append(timeit(lambda: torch.matmul(x, w.t(), out=o), a.iters))
                    pps.append(timeit(lambda: ops.gemm_prefill(x, w, out=o), a.iters))
                t_lib, t_pp = sorted(libs)[len(libs) // 2], sorted(pps)[len(pps) // 2]
                wr.writerow([N, K, M, round(t_lib, 2), round(t_pp, 2)])
                print(name, M, round(t_lib, 1), round(t_pp, 1), flush=True)


if __name__ == "__main__":
    main()
