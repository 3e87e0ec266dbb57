"""Load generator for the config-2 bench (bench/embed.py): the Kafka clients OUTSIDE the
agent pod -- the application that writes ``input-topic`` and the one that reads
``output-topic`` -- in their own interpreter, as they are separate processes in a real
deployment (the reference measures its agent pod, not the clients feeding it).

Protocol on stdin/stdout, one line per command:
  ``produce <step>``  -> write this rank's B records of that step, wait for the acks, ``ok``
  ``wait <total>``    -> read ``output-topic`` until ``total`` records were seen, ``ok <n>``
  ``quit``
"""
from __future__ import annotations

import argparse
import json
import sys
import time


def make_records(corpus, rank: int, world: int, B: int, step: int):
    from ..api.record import SimpleRecord
    out = []
    for j in range(B):
        g = (step * world + rank) * B + j
        text = " ".join(corpus[(g * 7 + k) % len(corpus)] for k in range(3))
        out.append(SimpleRecord.of(f"r{rank}-{g}", json.dumps({"text": text})))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--bootstrap", required=True)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--read", action="store_true", help="also count output-topic (rank 0)")
    ap.add_argument("--timeout", type=float, default=900.0)
    a = ap.parse_args(argv)
    from ..api.topics import TopicOffsetPosition
    from ..tokenizers import builtin_corpus
    from ..topics.kafka import KafkaProducer, KafkaReader
    corpus = builtin_corpus(20000)
    prod = KafkaProducer(a.bootstrap, "input-topic")
    reader = None
    if a.read:
        reader = KafkaReader(a.bootstrap, "output-topic", TopicOffsetPosition.EARLIEST, poll_ms=50)
        reader.start()
    seen = 0
    print("ready", flush=True)
    for line in sys.stdin:
        cmd = line.split()
        if not cmd:
            continue
        if cmd[0] == "quit":
            break
        if cmd[0] == "produce":
            # one queued unit behind one future (KafkaProducer.write_many), as a batching
            # Kafka client application would send them
            prod.write_many(make_records(corpus, a.rank, a.world, a.batch, int(cmd[1]))).result(60)
            print("ok", flush=True)
        elif cmd[0] == "wait":
            total = int(cmd[1])
            deadline = time.time() + a.timeout
            while seen < total and time.time() < deadline:
                seen += len(reader.read().records)
            print(f"ok {seen}", flush=True)
    prod.close()
    if reader is not None:
        reader.close()
    return 0


class LoadProcess:
    def __init__(self, bootstrap: str, rank: int, world: int, batch: int, read: bool, timeout: float):
        from ..utils.procs import spawn_module
        args = ["--bootstrap", bootstrap, "--rank", str(rank), "--world", str(world), "--batch", str(batch),
                "--timeout", str(timeout)] + (["--read"] if read else [])
        self.proc = spawn_module("langstream_amd.bench.embed_load", args)
        self._expect("ready")

    def _expect(self, prefix: str) -> str:
        line = self.proc.stdout.readline().strip()
        if not line.startswith(prefix):
            raise RuntimeError(f"embed load process: expected {prefix!r}, got {line!r} "
                               f"(exit {self.proc.poll()})")
        return line

    def produce(self, step: int) -> None:
        self.proc.stdin.write(f"produce {step}\n")
        self.proc.stdin.flush()
        self._expect("ok")

    def wait(self, total: int) -> int:
        self.proc.stdin.write(f"wait {total}\n")
        self.proc.stdin.flush()
        return int(self._expect("ok").split()[1])

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.proc.stdin.write("quit\n")
                self.proc.stdin.flush()
            except Exception:  # noqa: BLE001
                pass
        from ..utils.procs import close_stdin_and_wait
        close_stdin_and_wait(self.proc, 30.0)


if __name__ == "__main__":
    raise SystemExit(main())
