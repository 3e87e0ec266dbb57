"""Host-path probe for config 2 (bench/embed.py) without a GPU: the same pipeline,
broker process and load process, but the embeddings engine is a null engine that
returns a constant 384-float vector per text at once.  What it measures is the agent
process's own per-record cost (Kafka fetch -> record -> template -> batch -> JSON with
384 floats -> produce -> ordered commit), the part that bounds one agent replica.

  python tools/embed_host_bench.py [--batch 8192] [--steps 3] [--profile]
"""
from __future__ import annotations

import argparse
import os
import sys
from concurrent.futures import Future

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class NullEngine:
    """Completes every batch on its own thread, as the GPU engine's loop does."""

    def __init__(self, dim=384):
        import queue
        import threading
        import torch
        # float32 values, as the engine's host tensor holds them (tolist -> doubles)
        from langstream_amd.utils.fastjson import f32_rows
        # float32 rows, as the engine hands them out
        self.vec = f32_rows((torch.randn(1, dim) * 0.05))[0]
        self.q = queue.Queue()
        threading.Thread(target=self._loop, daemon=True).start()

    def _loop(self):
        while True:
            f, n = self.q.get()
            f.set_result([self.vec] * n)

    def embed_async(self, texts):
        f: Future = Future()
        self.q.put((f, len(texts)))
        return f

    def start(self):
        pass

    def stop(self):
        pass


_names = {}


def _thread_cpu():
    """CPU seconds (user + system) of every live thread of this process, by native id."""
    import threading
    out = {}
    tick = os.sysconf("SC_CLK_TCK")
    for t in threading.enumerate():
        _names[t.native_id] = t.name
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                parts = f.read().rsplit(")", 1)[1].split()
            out[int(tid)] = (int(parts[11]) + int(parts[12])) / tick
        except OSError:
            pass
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--embed-batch", type=int, default=256)
    ap.add_argument("--profile", action="store_true", help="cProfile the agent process (all threads)")
    a = ap.parse_args()
    from langstream_amd import services as svc
    svc.ServiceRegistry.embedding_engine = lambda self, model, cfg=None: NullEngine()
    from langstream_amd.bench import embed
    args = argparse.Namespace(batch=a.batch, steps=a.steps, warmup=a.warmup, embed_replicas=1,
                              embed_model="bge-small-en", embed_batch=a.embed_batch, timeout=300.0)
    if a.profile:
        import cProfile
        import pstats
        import threading
        prof = cProfile.Profile()
        threading.setprofile(lambda *x: None)
        profs = []

        def tp(frame, event, arg):
            p = cProfile.Profile()
            profs.append(p)
            p.enable()
            threading.setprofile(None)
        threading.setprofile(tp)
        prof.enable()
    import threading
    import time
    cpu_before = _thread_cpu()
    last = dict(cpu_before)
    done = threading.Event()

    def monitor():   # threads end before the run returns: keep the last value seen
        while not done.is_set():
            last.update(_thread_cpu())
            time.sleep(0.2)
    if os.environ.get("THREAD_CPU"):
        threading.Thread(target=monitor, daemon=True).start()
    embed.run(args, 0, 1, lambda: None, lambda x: x, gpu_init=lambda: False)
    done.set()
    if os.environ.get("THREAD_CPU"):
        after = last
        names = dict(_names)
        rows = sorted(((after[k] - cpu_before.get(k, 0.0), names.get(k, str(k))) for k in after), reverse=True)
        for cpu, name in rows[:12]:
            print(f"thread cpu {cpu:8.2f} s  {name}")
    if a.profile:
        prof.disable()
        st = pstats.Stats(prof)
        for p in profs:
            p.disable()
            st.add(p)
        st.sort_stats("tottime").print_stats(40)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
