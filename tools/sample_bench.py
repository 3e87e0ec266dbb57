"""Time the token sampler (ops/csrc/sampling.hip) on Llama-3 sized rows (V = 128256).

usage (GPU box): python tools/sample_bench.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from langstream_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    V = 128256
    for B in (1, 256):
        for std in (0.1, 3.0):
            logits = torch.randn(B, V, device=dev) * std
            for mode, (t, k, p) in {"greedy": (0.0, 0, 1.0), "T1": (1.0, 0, 1.0), "top_p": (0.8, 0, 0.95),
                                    "top_k": (0.8, 50, 1.0)}.items():
                temp = torch.full((B,), t, device=dev)
                tk = torch.full((B,), k, device=dev, dtype=torch.int32)
                tp = torch.full((B,), p, device=dev)
                seeds = torch.arange(B, device=dev, dtype=torch.int64)
                steps = torch.zeros(B, device=dev, dtype=torch.int64)
                for _ in range(3):
                    ops.sample(logits, temp, tk, tp, seeds, steps)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    ops.sample(logits, temp, tk, tp, seeds, steps)
                e.record()
                torch.cuda.synchronize()
                print(json.dumps({"B": B, "std": std, "mode": mode, "us": round(s.elapsed_time(e) * 50, 1)}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
