"""GPU-side gap between back-to-back replays of a HIP graph of N small kernels, and
with a host->device copy enqueued between replays (run under rocprofv3 --kernel-trace
and read the gaps with tools/rocpd_stats.py / a timeline query)."""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=400)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    x = torch.zeros(1 << 16, device="cuda")
    host = torch.zeros(1 << 16, pin_memory=True)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(a.nodes):
                x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(a.nodes):
            x.add_(1.0)
    torch.cuda.synchronize()
    for mode in ("replay", "copy+replay"):
        t0 = time.perf_counter()
        for _ in range(a.reps):
            if mode == "copy+replay":
                x[: host.numel()].copy_(host, non_blocking=True)
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps
        print(f"{mode}: {dt * 1e6:.1f} us per replay ({a.nodes} nodes)", flush=True)


if __name__ == "__main__":
    main()
