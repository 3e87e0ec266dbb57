"""Search latency under LLM load: a vector-store search on the high-priority search
stream while the default stream runs back-to-back large GEMMs (a prefill step's worth,
~150 ms) -- or the high-priority auxiliary stream or a pool stream runs them -- with the D2H of results through freshly allocated pinned buffers
(utils/gpu.to_host), through a reused pinned buffer, and through pageable memory.

usage (GPU): python tools/search_latency_probe.py
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> int:
    from langstream_amd.engine.vector_store import VectorStore
    from langstream_amd.utils import gpu
    dev = "cuda"
    store = VectorStore(384, device=dev)
    n = 50000
    g = torch.Generator(device="cpu").manual_seed(0)
    store.upsert([f"d{i}" for i in range(n)], torch.randn(n, 384, generator=g).to(dev), [{"text": "x"}] * n)
    torch.cuda.synchronize()
    a = torch.randn(16384, 4096, device=dev, dtype=torch.bfloat16)
    w = torch.randn(14336, 4096, device=dev, dtype=torch.bfloat16)
    q = torch.randn(64, 384)

    from langstream_amd import ops
    wg = torch.randn(2 * 14336, 4096, device=dev, dtype=torch.bfloat16)
    kind = {"k": "matmul"}

    side = torch.cuda.Stream()

    def load(stop):
        # the load's stream: the default stream (the LLM engine's), the high-priority
        # auxiliary stream (ingest embeddings / upserts), or a pool stream
        st = {"aux": gpu.aux_stream(dev), "side": side}.get(kind.get("stream"), torch.cuda.current_stream())
        with torch.cuda.stream(st):
            while not stop.is_set():
                for _ in range(40):
                    if kind["k"] == "matmul":
                        torch.matmul(a, w.t())
                    else:   # the engine's prefill gate_up kernel: 160 KB of LDS per workgroup
                        ops.gemm_prefill(a, wg, silu=True)
                torch.cuda.synchronize()

    res = {}
    for mode in ("idle", "loaded", "loaded_pp", "loaded_aux", "loaded_side"):
        kind["k"] = "pp" if mode == "loaded_pp" else "matmul"
        kind["stream"] = mode[len("loaded_"):] if mode in ("loaded_aux", "loaded_side") else None
        stop = threading.Event()
        th = threading.Thread(target=load, args=(stop,), daemon=True)
        if mode != "idle":
            th.start()
            time.sleep(0.5)
        for variant in ("default", "vectors"):
            lat = []
            for _ in range(15):
                t = time.perf_counter()
                store.search(q.tolist(), 20, with_vectors=(variant == "vectors"))
                lat.append((time.perf_counter() - t) * 1e3)
                time.sleep(0.02)
            res[f"{mode}_{variant}_ms"] = [round(statistics.median(lat), 2), round(max(lat), 2)]
        stop.set()
        if mode != "idle":
            th.join()
    # the raw copy paths under load
    stop = threading.Event()
    th = threading.Thread(target=load, args=(stop,), daemon=True)
    th.start()
    time.sleep(0.5)
    x = torch.randn(1280, 384, device=dev)
    pinned = torch.empty(1280, 384, pin_memory=True)
    for variant in ("to_host_fresh_pinned", "reused_pinned", "pageable"):
        lat = []
        for _ in range(15):
            with gpu.on_search(dev):
                t = time.perf_counter()
                if variant == "to_host_fresh_pinned":
                    gpu.to_host(x)
                elif variant == "reused_pinned":
                    pinned.copy_(x, non_blocking=True)
                    ev = torch.cuda.Event(blocking=True)
                    ev.record()
                    ev.synchronize()
                else:
                    x.cpu()
                lat.append((time.perf_counter() - t) * 1e3)
            time.sleep(0.02)
        res[f"loaded_copy_{variant}_ms"] = [round(statistics.median(lat), 2), round(max(lat), 2)]
    stop.set()
    th.join()
    print(json.dumps(res), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
