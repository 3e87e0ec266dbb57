"""Headline benchmark: full RAG pipeline, Llama-3-8B, records/sec (whole node) + p50 e2e latency.

BASELINE.json config 4 ("full RAG pipeline (crawl->split->embed->vector-write;
query->vector-query->chat) Llama-3-8B, 8 agent replicas DP on 8xMI355X"), run through
the framework itself (YAML app -> planner -> fused composite agents -> AgentRunner on
memory topics), both pipelines concurrently in every timed step:

  ingest: documents -> text-splitter (cl100k length) -> document-to-json
          -> compute-ai-embeddings (bge-small-en, GPU) -> vector-db-sink (HBM store)
  query:  questions -> document-to-json -> compute-ai-embeddings (GPU)
          -> query-vector-db (GPU kNN top-20) -> re-rank (MMR, top-5)
          -> ai-chat-completions (Llama-3-8B, GPU, streamed to answers-topic)
          -> drop-fields -> log-topic

One process per GPU (torchrun), each an independent agent replica (data parallel,
weak scaling: a fixed batch per GPU per step).  Before timing, each rank loads a
synthetic corpus through the GPU encoder into its vector store (untimed).  A step =
produce B questions + D documents (the crawled pages), wait for all B answers and for
every chunk of the D documents to be indexed; time K steps after W warmup steps.
value = answered questions per second over all ranks (max time over ranks); the
ingest rate is reported alongside.  Weights are random-init (no checkpoints offline);
data is synthetic.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

APP = """
topics:
  - name: "questions-topic"
    creation-mode: create-if-not-exists
    partitions: 4
  - name: "answers-topic"
    creation-mode: create-if-not-exists
  - name: "log-topic"
    creation-mode: create-if-not-exists
errors:
  on-failure: "fail"
pipeline:
  - name: "convert-to-structure"
    type: "document-to-json"
    input: "questions-topic"
    configuration:
      text-field: "question"
  - name: "compute-embeddings"
    type: "compute-ai-embeddings"
    configuration:
      model: "{embed_model}"
      embeddings-field: "value.question_embeddings"
      text: "{{{{ value.question }}}}"
      batch-size: 64
      concurrency: 4
      flush-interval: 5
  - name: "lookup-related-documents"
    type: "query-vector-db"
    configuration:
      datasource: "LocalVectors"
      query: '{{"collection-name": "documents", "vector": ?, "top-k": 20, "include-vector": true}}'
      fields:
        - "value.question_embeddings"
      output-field: "value.related_documents"
  - name: "re-rank documents with MMR"
    type: "re-rank"
    configuration:
      max: 5
      field: "value.related_documents"
      query-text: "value.question"
      query-embeddings: "value.question_embeddings"
      output-field: "value.related_documents"
      text-field: "record.text"
      embeddings-field: "record.vector"
      algorithm: "MMR"
      lambda: 0.5
      k1: 1.2
      b: 0.75
  - name: "ai-chat-completions"
    type: "ai-chat-completions"
    configuration:
      model: "{chat_model}"
      completion-field: "value.answer"
      log-field: "value.prompt"
      stream-to-topic: "answers-topic"
      stream-response-completion-field: "value"
      min-chunks-per-message: 20
      max-tokens: {max_tokens}
      ignore-eos: true
      messages:
        - role: system
          content: |
              An user is going to perform a questions, The documents below may help you in answering to their questions.
              Please try to leverage them in your answer as much as possible.
              Documents:
              {{{{# value.related_documents}}}}
              {{{{ text}}}}
              {{{{/ value.related_documents}}}}
        - role: user
          content: "{{{{ value.question}}}}"
  - name: "cleanup-response"
    type: "drop-fields"
    output: "log-topic"
    configuration:
      fields:
        - "question_embeddings"
        - "related_documents"
"""

INGEST = """
topics:
  - name: "documents-topic"
    creation-mode: create-if-not-exists
    partitions: 2
pipeline:
  - name: "split"
    type: "text-splitter"
    input: "documents-topic"
    configuration:
      chunk_size: 256
      chunk_overlap: 32
      length_function: "cl100k_base"
  - name: "to-json"
    type: "document-to-json"
    configuration:
      text-field: "text"
  - name: "embed-chunks"
    type: "compute-ai-embeddings"
    configuration:
      model: "{embed_model}"
      embeddings-field: "value.embeddings"
      text: "{{{{ value.text }}}}"
      batch-size: 64
      concurrency: 4
      flush-interval: 5
  - name: "write"
    type: "vector-db-sink"
    configuration:
      datasource: "LocalVectors"
      collection-name: "documents"
      fields:
        - name: "id"
          expression: "fn:concat(key, '-', properties.chunk_id)"
        - name: "vector"
          expression: "value.embeddings"
        - name: "text"
          expression: "value.text"
"""

CONFIGURATION = """
configuration:
  resources:
    - type: "local-gpu-configuration"
      name: "local"
      configuration:
        chat-model: "{chat_model}"
        embeddings-model: "{embed_model}"
        max-batch: {max_batch}
        max-model-len: {max_len}
        max-prefill-tokens: {prefill}
    - type: "vector-database"
      name: "LocalVectors"
      configuration:
        service: "local"
        collection-name: "documents"
"""


def _env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="questions per GPU per step")
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--corpus", type=int, default=50000, help="documents in each rank's vector store")
    ap.add_argument("--docs", type=int, default=32, help="documents ingested per GPU per step (0: query only)")
    ap.add_argument("--chat-model", default="llama-3-8b")
    ap.add_argument("--embed-model", default="bge-small-en")
    ap.add_argument("--device", default=None)
    ap.add_argument("--timeout", type=float, default=900.0)
    args = ap.parse_args()

    rank, world, local = _env_int("RANK", 0), _env_int("WORLD_SIZE", 1), _env_int("LOCAL_RANK", 0)
    import torch
    import torch.distributed as dist
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl" if use_gpu else "gloo")

    def barrier():
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize()

    from langstream_amd.engine.vector_store import VectorStoreRegistry
    from langstream_amd.runtime.local import LocalApplicationRunner
    from langstream_amd.services import ServiceRegistry
    from langstream_amd.tokenizers import builtin_corpus

    device = args.device or (f"cuda:{local}" if use_gpu else "cpu")
    chat_model, embed_model = args.chat_model, args.embed_model
    if not use_gpu and args.chat_model == "llama-3-8b":
        chat_model, embed_model = "llama-tiny", "bert-tiny"  # CPU plumbing mode only
    fmt = dict(chat_model=chat_model, embed_model=embed_model, max_tokens=args.max_tokens,
               max_batch=max(args.batch, 1), max_len=4096, prefill=16384)
    files = {"pipeline.yaml": APP.format(**fmt), "ingest.yaml": INGEST.format(**fmt),
             "configuration.yaml": CONFIGURATION.format(**fmt)}
    services = ServiceRegistry({"device": device})
    ServiceRegistry.set_default(services)

    # ---- untimed setup: engines, corpus ingest into the HBM vector store
    t_setup = time.time()
    emb = services.embedding_engine(embed_model, {"embeddings-model": embed_model})
    corpus = builtin_corpus(max(4000, args.corpus // 4 + 1))
    docs = [" ".join(corpus[(i * 7 + j) % len(corpus)] for j in range(4)) for i in range(args.corpus)]
    store = VectorStoreRegistry.get("documents", emb.dim, device=device)
    for i in range(0, len(docs), 8192):
        chunk = docs[i: i + 8192]
        vec = emb.embed_tensor(chunk)
        store.upsert(list(range(i, i + len(chunk))), vec, [{"text": t} for t in chunk])
    llm = services.llm_engine(chat_model, {"chat-model": chat_model, "max-batch": fmt["max_batch"],
                                           "max-model-len": 4096, "max-prefill-tokens": 16384})
    runner = LocalApplicationRunner.from_yaml(files, application_id="rag-bench", services=services)
    runner.start()
    prod = runner.producer("questions-topic")
    doc_prod = runner.producer("documents-topic")
    reader = runner.reader("log-topic")
    setup_s = time.time() - t_setup

    from langstream_amd.agents.text import RecursiveCharacterTextSplitter
    from langstream_amd.api.record import SimpleRecord
    from langstream_amd.tokenizers import cl100k_counter
    splitter = RecursiveCharacterTextSplitter(["\n\n", "\n", " ", ""], False, 256, 32, cl100k_counter())
    qwords = corpus
    seq = [0]
    ingested = {"docs": 0, "chunks": 0}

    def make_doc(i: int) -> str:  # a crawled page: ~12 paragraphs of corpus sentences
        return "\n\n".join(" ".join(corpus[(i * 31 + p * 7 + j) % len(corpus)] for j in range(5))
                           for p in range(12))

    def run_step(n, n_docs):
        sent = {}
        t0 = time.time()
        base = len(store)
        expect = 0
        for d in range(n_docs):
            text = make_doc(seq[0] * 7 + d)
            expect += len(splitter.split_text(text))
            doc_prod.write(SimpleRecord.of(f"doc-{rank}-{seq[0]}-{d}", text))
        for i in range(n):
            k = f"{rank}-{seq[0]}"
            seq[0] += 1
            q = qwords[(seq[0] * 13) % len(qwords)]
            sent[k] = time.time()
            prod.write(SimpleRecord.of(k, q))
        lats = []
        got = 0
        deadline = time.time() + args.timeout
        while got < n or len(store) < base + expect:
            if runner.errors:
                raise runner.errors[0]
            if time.time() > deadline:
                raise TimeoutError(f"only {got}/{n} records and {len(store) - base}/{expect} chunks completed")
            for r in reader.read().records:
                t = sent.pop(r.key(), None)
                if t is not None:
                    got += 1
                    lats.append(time.time() - t)
        ingested["docs"] += n_docs
        ingested["chunks"] += expect
        return time.time() - t0, lats

    for _ in range(args.warmup):
        run_step(args.batch, args.docs)
    barrier()
    from langstream_amd.utils import threads as _threads
    cpu0 = _threads.snapshot()
    t0 = time.time()
    all_lats = []
    for _ in range(args.steps):
        _, lats = run_step(args.batch, args.docs)
        all_lats.extend(lats)
    barrier()
    elapsed = time.time() - t0
    if os.environ.get("LANGSTREAM_THREAD_CPU"):
        print(json.dumps({"thread_cpu_s": _threads.diff(cpu0, _threads.snapshot())}), file=sys.stderr, flush=True)
    p50 = statistics.median(all_lats) if all_lats else 0.0
    if world > 1:
        t = torch.tensor([elapsed, p50], dtype=torch.float64, device=device if use_gpu else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, p50 = float(t[0]), float(t[1])
    total = args.batch * args.steps * world
    value = total / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "records/sec (whole node) + p50 end-to-end latency, RAG pipeline Llama-3-8B",
            "value": round(value, 3), "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "p50_latency_s": round(p50, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if use_gpu else "fp32", "data": "synthetic questions + synthetic corpus, random-init weights",
            "config": {"model": chat_model, "embedding_model": embed_model, "global_batch": args.batch * world,
                       "seq_len": 4096, "max_new_tokens": args.max_tokens, "corpus_docs_per_gpu": args.corpus,
                       "top_k": 20, "rerank": 5, "ingest_docs_per_gpu_per_step": args.docs,
                       "parallelism": f"dp{world}"},
            "ingest": {"docs_per_s": round(args.docs * args.steps * world / elapsed, 2),
                       "chunks_per_s_rank0": round(ingested["chunks"] * args.steps / max(1, args.steps + args.warmup)
                                                   / elapsed, 2)},
            "setup_s": round(setup_s, 1),
            "engine": dict(llm.stats, exec_ms=dict(zip(("upload", "enqueue", "download", "wait"),
                                                       (round(x, 1) for x in llm.exec.timings())))),
        }), flush=True)
    runner.stop(timeout=10)
    services.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
