"""Launch the prefill GEMM a few times on one shape (for rocprofv3 --pmc passes).

usage (GPU): python tools/pgemm_probe.py [--m 16384] [--n 28672] [--k 4096] [--silu] [--lib]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=28672)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--silu", action="store_true")
    ap.add_argument("--lib", action="store_true", help="hipBLASLt (F.linear) instead")
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    from langstream_amd import ops
    x = (torch.rand(a.m, a.k, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(a.n, a.k, device="cuda") * 2 - 1) / a.k ** 0.5).bfloat16()
    for _ in range(a.iters):
        if a.lib:
            torch.nn.functional.linear(x, w)
        else:
            ops.gemm_prefill(x, w, silu=a.silu)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
