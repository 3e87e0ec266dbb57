"""Micro-benchmark of the fused RoPE + paged-KV write (ops.rope_and_cache) at decode
shapes: Llama-3-8B heads, B tokens at random cache slots in a large block pool.

    python tools/rope_bench.py [--B 256] [--blocks 20000]

Prints one JSON line per variant: full kernel, no cache write (slots = -1), and the
bytes-moved lower bound.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from langstream_amd import ops  # noqa: E402
from langstream_amd.ops import reference as ref  # noqa: E402


def timeit(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--blocks", type=int, default=20000)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    Hq, Hkv, D, BS = 32, 8, 128, 64
    B = a.B
    torch.manual_seed(0)
    qkv = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (B,), device=dev, dtype=torch.int32)
    inv = 1.0 / (500000.0 ** (torch.arange(0, D, 2, device=dev).float() / D))
    ang = torch.arange(8192, device=dev).float()[:, None] * inv[None]
    cos_sin = torch.cat([ang.cos(), ang.sin()], -1).contiguous()
    kc = torch.zeros(a.blocks, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(a.blocks, Hkv, BS // 8, D, 8, device=dev, dtype=torch.bfloat16)
    blk = torch.randperm(a.blocks, device=dev)[:B].long()
    slots = blk * BS + torch.randint(0, BS, (B,), device=dev)
    none = torch.full_like(slots, -1)
    if a.check:
        q2, k2, v2 = qkv.clone(), kc.clone(), vc.clone()
        ops.rope_and_cache(q2, pos, cos_sin, slots, k2, v2, Hq, Hkv)
        q3, k3, v3 = qkv.clone(), kc.clone(), vc.clone()
        ref.rope_and_cache(q3, pos, cos_sin, slots, k3, v3, Hq, Hkv, True)
        err = max((q2.float() - q3.float()).abs().max().item(), (k2.float() - k3.float()).abs().max().item(),
                  (v2.float() - v3.float()).abs().max().item())
        print(json.dumps({"check_max_err": err}))
    full = timeit(lambda: ops.rope_and_cache(qkv, pos, cos_sin, slots, kc, vc, Hq, Hkv))
    nowrite = timeit(lambda: ops.rope_and_cache(qkv, pos, cos_sin, none, kc, vc, Hq, Hkv))
    byts = B * (Hq + 2 * Hkv) * D * 2 * 2 + B * 2 * Hkv * D * 2
    print(json.dumps({"B": B, "us_full": round(full, 2), "us_no_cache_write": round(nowrite, 2),
                      "bytes": byts, "floor_us_at_6TBps": round(byts / 6e12 * 1e6, 2)}))


if __name__ == "__main__":
    main()
