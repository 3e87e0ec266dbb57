"""BASELINE config 1: the text-splitter agent on an in-memory topic, the way
``langstream docker run`` runs an application on one host (here: ``LocalApplicationRunner``
on the ``memory`` streaming cluster, as ``python -m langstream_amd.cli run`` does).  CPU
only -- the plumbing of the runtime, no GPU.

The reference application shape (examples/applications/text-processing: text-splitter
with RecursiveCharacterTextSplitter, cl100k_base lengths) reads ``input-topic`` and writes
one record per chunk to ``output-topic``.  A step = B documents written at once; it ends
when every chunk of those documents has been read back from ``output-topic``.  The chunk
count a step must produce is computed up front with the agent's own splitter, so the
step boundary is exact.
"""
from __future__ import annotations

import json
import time

PIPE = """
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
  - name: "output-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "split"
    id: "split"
    type: "text-splitter"
    input: "input-topic"
    output: "output-topic"
    configuration:
      splitter_type: "RecursiveCharacterTextSplitter"
      chunk_size: {chunk}
      chunk_overlap: {overlap}
      length_function: "cl100k_base"
"""

INSTANCE = """
instance:
  streamingCluster:
    type: "memory"
  computeCluster:
    type: "none"
"""

METRIC = "records/sec (input documents), text-splitter agent on an in-memory topic, CPU only"
CHUNK, OVERLAP = 400, 100


def make_docs(corpus, B: int, paragraphs: int = 12, sentences: int = 5):
    """B synthetic documents of ``paragraphs`` paragraphs (blank-line separated, the
    splitter's first separator), ~2.5 KB each; the same texts every step."""
    docs = []
    for d in range(B):
        paras = []
        for p in range(paragraphs):
            base = (d * paragraphs + p) * sentences
            paras.append(" ".join(corpus[(base + k) % len(corpus)] for k in range(sentences)))
        docs.append("\n\n".join(paras))
    return docs


def run(args) -> None:
    from ..agents.text import TextSplitterAgent
    from ..api.record import SimpleRecord
    from ..runtime.local import LocalApplicationRunner
    from ..tokenizers import builtin_corpus
    B = args.batch
    docs = make_docs(builtin_corpus(20000), B)
    ref = TextSplitterAgent()
    ref.init({"chunk_size": CHUNK, "chunk_overlap": OVERLAP, "length_function": "cl100k_base"})
    per_step = sum(len(ref.splitter.split_text(d)) for d in docs)

    t_setup = time.time()
    runner = LocalApplicationRunner.from_yaml({"pipeline.yaml": PIPE.format(chunk=CHUNK, overlap=OVERLAP)},
                                              instance=INSTANCE, application_id="split-bench")
    runner.start()
    prod = runner.producer("input-topic")
    reader = runner.reader("output-topic")
    setup_s = time.time() - t_setup
    seen = 0
    step_s = []
    try:
        for step in range(args.warmup + args.steps):
            t0 = time.perf_counter()
            futs = [prod.write(SimpleRecord.of(f"s{step}-d{j}", d)) for j, d in enumerate(docs)]
            for f in futs:
                f.result(60)
            want = (step + 1) * per_step
            deadline = time.time() + args.timeout
            while seen < want:
                if runner.errors:
                    raise runner.errors[0]
                if time.time() > deadline:
                    raise TimeoutError(f"split bench: {seen} of {want} chunks after {args.timeout} s")
                seen += len(reader.read().records)
            if step >= args.warmup:
                step_s.append(time.perf_counter() - t0)
    finally:
        prod.close()
        reader.close()
        runner.stop()
    total = sum(step_s)
    docs_s = B * args.steps / total
    print(json.dumps({
        "metric": METRIC, "value": round(docs_s, 1), "unit": "records/s", "n_gpus": 0,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(total / args.steps * 1000, 2),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "n/a (CPU only)",
        "data": "synthetic documents (12 paragraphs, ~2.5 KB each)",
        "config": {"agent": "text-splitter", "streaming": "memory", "documents_per_step": B,
                   "chunk_size": CHUNK, "chunk_overlap": OVERLAP, "length_function": "cl100k_base"},
        "chunks_per_s": round(per_step * args.steps / total, 1), "chunks_per_document": round(per_step / B, 2),
        "setup_s": round(setup_s, 2)}), flush=True)
