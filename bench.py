"""Headline benchmark: full RAG pipeline, Llama-3-8B, records/sec (whole node) + p50 e2e latency.

BASELINE.json config 4 ("full RAG pipeline (crawl->split->embed->vector-write;
query->vector-query->chat) Llama-3-8B, 8 agent replicas DP on 8xMI355X"), run through
the framework itself (YAML app -> planner -> fused composite agents -> AgentRunner),
all three pipelines concurrently in every timed step:

  crawl:  webcrawler-source (rank 0 only, like the reference's single crawler replica)
          fetching the step's new pages from a local HTTP site -> documents-topic
  ingest: documents -> text-extractor -> text-splitter (cl100k length) -> document-to-json
          -> compute-ai-embeddings (bge-small-en, GPU) -> vector-db-sink (HBM shard)
  query:  questions -> document-to-json -> compute-ai-embeddings (GPU)
          -> query-vector-db (GPU kNN top-20 over EVERY rank's shard) -> re-rank (MMR, top-5)
          -> ai-chat-completions (Llama-3-8B, GPU, streamed to answers-topic)
          -> drop-fields -> log-topic

Data parallelism is the reference's: one process per GPU, every process
running a replica of each agent, the replicas of an agent forming ONE consumer group
over the partitions of its input topic.  Topics live in the cross-process shared-memory
log (``shm`` streaming type), so any replica may answer any rank's question; the vector
store is sharded (each rank indexes the chunks it consumed) and query-vector-db returns
the global top-k through the sharded kNN service (RCCL all-gather / all-to-all).

``python bench.py --gpus N`` (no torchrun environment) launches N rank processes with
torch.distributed.run itself before anything touches the GPU; under torchrun
(WORLD_SIZE set) ``--gpus`` must equal WORLD_SIZE.

Weak scaling: per GPU per step, B answered questions and D crawled pages; before timing
each rank loads a synthetic corpus into its shard (untimed).  Load (``--load``): by
default bursts -- B questions written at the start of each step; ``--load stream`` runs
a closed loop instead (B questions in flight per GPU, a new one as each answer
arrives).  Measured on one MI355X the conservative stream window is slower (89.9 / 97.6
records/s over 3 / 6 steps vs 105.9 burst, profiles/bench_r2k_*): every request
generates exactly max-tokens, so the loop stays phase-locked and the window pays its
drain.  Burst: a step ends when the rank has its
B answers and every page crawled so far is fully indexed (committed by the ingest
consumer group).  Stream: the timed window counts only questions sent inside it (K x B
per GPU), keeps B in flight until all are sent, then drains them, so the window never
does less work than it counts.  K steps are timed after W warmup steps, bracketed by a barrier
and a device synchronize on both sides; value = answered questions per second over all
ranks (max elapsed over ranks).  Weights are random-init (no checkpoints offline); data
is synthetic.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import threading
import time
import uuid
import zlib

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

APP = """
topics:
  - name: "questions-topic"
    creation-mode: create-if-not-exists
    partitions: {q_parts}
  - name: "answers-topic"
    creation-mode: create-if-not-exists
  - name: "log-topic"
    creation-mode: create-if-not-exists
errors:
  on-failure: "fail"
pipeline:
  - name: "convert-to-structure"
    id: "query"
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
    partitions: {d_parts}
pipeline:
  - name: "extract"
    id: "ingest"
    type: "text-extractor"
    input: "documents-topic"
  - name: "split"
    type: "text-splitter"
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

CRAWL = """
topics:
  - name: "documents-topic"
    creation-mode: create-if-not-exists
    partitions: {d_parts}
pipeline:
  - name: "crawl"
    id: "crawler"
    type: "webcrawler-source"
    output: "documents-topic"
    configuration:
      seed-urls: ["{site}/step/0/index.html"]
      allowed-domains: ["{site}"]
      max-urls: 10000000
      max-depth: 10000000
      handle-robots-file: false
      min-time-between-requests: 0
      http-timeout: 1800000
      state-storage: disk
      max-unflushed-pages: 1000
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

INSTANCE = """
instance:
  streamingCluster:
    type: "shm"
    configuration:
      name: "{shm}"
      size-mb: {shm_mb}
  computeCluster:
    type: "none"
"""

METRIC = "records/sec (whole node) + p50 end-to-end latency, RAG pipeline Llama-3-8B"


def _env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(argv, n: int) -> int:
    """Start N ranks with torch.distributed.run (this process never touches the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def balanced_key(prefix: str, target: int, parts: int) -> str:
    """A record key whose crc32 partition (the producers' key hash) is ``target``: keys
    are spread evenly over the partitions, so every consumer-group member gets the same
    share of each step."""
    salt = 0
    while True:
        k = f"{prefix}.{salt}"
        if zlib.crc32(k.encode()) % parts == target:
            return k
        salt += 1


def _pcts(xs):
    """min / p10 / p50 / p90 / p99 / max of a list (the decode attention launch ends with the longest context)."""
    if not xs:
        return None
    xs = sorted(xs)
    return {k: xs[min(len(xs) - 1, int(q * len(xs)))] for k, q in
            (("min", 0.0), ("p10", 0.1), ("p50", 0.5), ("p90", 0.9), ("p99", 0.99), ("max", 1.0))}


def _stream_summary(gathered, args, world):
    """The closed-loop window run after the burst window (--also-stream): records/s over
    the slowest rank, p50 latency; None when it did not run."""
    if not gathered or gathered[0].get("stream") is None:
        return None
    el = max(g["stream"]["elapsed"] for g in gathered)
    lats = [x for g in gathered for x in g["stream"]["lats"]]
    n = args.also_stream * args.batch * world
    return {"value": round(n / el, 3), "unit": "records/s", "steps": args.also_stream,
            "ms_per_step": round(1000 * el / args.also_stream, 2),
            "p50_latency_s": round(statistics.median(lats), 3) if lats else None,
            "load": f"closed loop, {args.batch} questions in flight per GPU; only questions sent inside the "
                    f"window count, the window drains them"}


from langstream_amd.bench.site import Site, SiteProcess, make_page  # noqa: E402


def _bringup(rank: int, world: int, use_gpu: bool, args):
    """Multi-rank bring-up: a per-rank watchdog (a rank that stops making progress ends
    every rank with exit 3 and one JSON line naming the stalled phase and the suspect
    rank) and the collective self-check on the job's group (a wrong RCCL / gloo sum ends
    the run with exit 2 and the failing phase, before any timing)."""
    from langstream_amd.parallel.bringup import CollectiveCheckError, check_collectives
    from langstream_amd.parallel.watchdog import RankWatchdog
    wd = RankWatchdog(rank, world, prefix="bench-watchdog").start()
    try:
        res = check_collectives(device=f"cuda:{torch_current_device()}" if use_gpu else "cpu", graphs=False,
                                watchdog=wd, limit_s=_env_int("LS_BRINGUP_LIMIT_S", 300))
    except CollectiveCheckError as e:
        print(json.dumps({"error": "collective self-check failed", "rank": rank, "detail": str(e)}),
              file=sys.stderr, flush=True)
        os._exit(2)
    if rank == 0:
        print(json.dumps({"bringup": res, "world": world}), file=sys.stderr, flush=True)
    return wd


def torch_current_device() -> int:
    import torch
    return torch.cuda.current_device()


def _phase(wd, name: str, limit_s: float) -> None:
    if wd is not None:
        wd.phase(name, _env_int("LS_WATCHDOG_LIMIT_S", 0) or limit_s)


def _beat(wd) -> None:
    if wd is not None:
        wd.beat()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="questions per GPU per step")
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--corpus", type=int, default=50000, help="documents in each rank's vector-store shard")
    ap.add_argument("--docs", type=int, default=32, help="pages crawled per GPU per step (0: query only)")
    ap.add_argument("--no-crawl", action="store_true", help="produce pages into documents-topic directly")
    ap.add_argument("--chat-model", default="llama-3-8b")
    ap.add_argument("--embed-model", default="bge-small-en")
    ap.add_argument("--device", default=None)
    ap.add_argument("--timeout", type=float, default=900.0)
    ap.add_argument("--prefill-chunk", type=int, default=16384,
                    help="engine max-prefill-tokens per step (chunked prefill)")
    ap.add_argument("--also-stream", type=int, default=3,
                    help="burst load: afterwards time this many steps' worth of questions under the closed-loop "
                         "load too and report it as stream_load (0: skip)")
    ap.add_argument("--load", choices=("stream", "burst"), default="burst",
                    help="stream: closed loop, --batch questions in flight per GPU, a new question as each "
                         "answer arrives, a step = --batch answers; burst: --batch questions at the start of "
                         "each step, the step ends when all are answered")
    ap.add_argument("--no-persist", action="store_true",
                    help="keep the vector store in HBM only (default: WAL + snapshots on local disk, the "
                         "durable default of a vector-db-sink pod)")
    ap.add_argument("--config", choices=("rag", "embed", "chat", "split"), default="rag",
                    help="rag: BASELINE config 4 (the headline, default); split: config 1 (text-splitter on an "
                         "in-memory topic, CPU only); embed: config 2 (compute-ai-embeddings "
                         "agent on Kafka records); chat: config 3 (ai-chat-completions through the websocket "
                         "gateway), and config 5 with --chat-model llama-3-70b --gpus 8 --tp 8")
    ap.add_argument("--tp", type=int, default=0, help="chat: tensor-parallel degree (= --gpus)")
    ap.add_argument("--embed-batch", type=int, default=64, help="embed: the agent's batch-size")
    ap.add_argument("--embed-replicas", type=int, default=3,
                    help="embed: agent replicas per GPU (resources.parallelism); > 1 runs each as its own "
                         "agent-pod process sharing the GPU")
    args = ap.parse_args()
    try:
        # byte-compile the package up front (~0.3 s cold): modules imported lazily by
        # agents / codecs must not compile inside the timed window on a fresh checkout
        import compileall
        compileall.compile_dir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "langstream_amd"), quiet=1)
    except Exception:  # noqa: BLE001  (read-only tree: imports compile in memory as before)
        pass

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch(sys.argv[1:], args.gpus))
    rank, world, local = _env_int("RANK", 0), _env_int("WORLD_SIZE", 1), _env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.config == "split":
        from langstream_amd.bench import split
        return split.run(args)
    if args.config != "rag":
        return _other_config(args, rank, world, local)
    corpus_sentences = max(4000, args.corpus // 4 + 1)
    crawl = args.docs > 0 and not args.no_crawl
    site = None
    if crawl and rank == 0:
        # the crawl target runs in its own process (started before the GPU is touched);
        # LS_BENCH_SITE_INPROC=1 serves it from this rank's interpreter as before
        if os.environ.get("LS_BENCH_SITE_INPROC") == "1":
            from langstream_amd.tokenizers import builtin_corpus as _bc
            site = Site(_bc(corpus_sentences), args.docs * world)
        else:
            site = SiteProcess(args.docs * world, corpus_sentences)
    # the webcrawler source (once, on rank 0) in an interpreter of its own, as its own pod
    # would be: pre-started here, before the GPU is touched, and handed the app later;
    # LS_BENCH_CRAWLER_INPROC=1 runs it as a thread of rank 0's runner instead
    crawler_host = None
    if crawl and rank == 0 and os.environ.get("LS_BENCH_CRAWLER_INPROC") != "1":
        from langstream_amd.runtime.agent_host import AgentHostProcess
        crawler_host = AgentHostProcess()

    import torch
    import torch.distributed as dist
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local)
    ctrl = None
    # LS_BENCH_FORCE_DIST=1 (under torchrun): take the multi-rank code path even at world
    # size 1 -- RCCL/gloo groups, barriers, the sharded kNN service -- to rehearse it on one GPU
    multi = world > 1 or os.environ.get("LS_BENCH_FORCE_DIST") == "1" and "WORLD_SIZE" in os.environ
    wd = None
    if multi:
        dist.init_process_group("nccl" if use_gpu else "gloo")
        ctrl = dist.new_group(backend="gloo")   # barriers / small host exchanges
        wd = _bringup(rank, world, use_gpu, args)

    def barrier():
        if multi:
            if wd is not None:
                wd.arrive("barrier")
            dist.barrier(group=ctrl)
        if use_gpu:
            torch.cuda.synchronize()

    def bcast(obj):
        if world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0, group=ctrl)
        return box[0]

    from langstream_amd.engine import dist_knn
    from langstream_amd.engine.vector_store import VectorStoreRegistry
    from langstream_amd.runtime import composite as _composite
    from langstream_amd.runtime.local import LocalApplicationRunner
    from langstream_amd.services import ServiceRegistry
    from langstream_amd.tokenizers import builtin_corpus
    from langstream_amd.topics.shm import unlink_shmlog

    device = args.device or (f"cuda:{local}" if use_gpu else "cpu")
    chat_model, embed_model = args.chat_model, args.embed_model
    if not use_gpu and args.chat_model == "llama-3-8b":
        chat_model, embed_model = "llama-tiny", "bert-tiny"  # CPU plumbing mode only
    q_parts, d_parts = max(4, 2 * world), max(2, 2 * world)
    shm = bcast(f"bench-{uuid.uuid4().hex[:12]}")
    shm_mb = 2048 + 512 * world
    fmt = dict(chat_model=chat_model, embed_model=embed_model, max_tokens=args.max_tokens,
               max_batch=max(args.batch, 1), max_len=4096, prefill=args.prefill_chunk, q_parts=q_parts, d_parts=d_parts,
               shm=shm, shm_mb=shm_mb)
    corpus = builtin_corpus(corpus_sentences)
    files = {"pipeline.yaml": APP.format(**fmt), "ingest.yaml": INGEST.format(**fmt),
             "configuration.yaml": CONFIGURATION.format(**fmt)}
    if crawl:
        files["crawl.yaml"] = CRAWL.format(site=bcast(site.url if site else None), d_parts=d_parts)
    services = ServiceRegistry({"device": device})
    ServiceRegistry.set_default(services)

    # ---- untimed setup: engines, corpus ingest into this rank's HBM shard
    t_setup = time.time()
    _phase(wd, "setup", 1800)
    persist_dir = None
    if not args.no_persist:
        import tempfile
        persist_dir = tempfile.mkdtemp(prefix=f"rag-bench-store-r{rank}-")
        import atexit
        import shutil
        # removed on every exit path (a failed or interrupted run too), not only at the end
        atexit.register(shutil.rmtree, persist_dir, True)
        VectorStoreRegistry.configure(persist_dir=persist_dir)   # every upsert WAL-logged before its ack
    emb = services.embedding_engine(embed_model, {"embeddings-model": embed_model})
    docs = [" ".join(corpus[(i * 7 + j) % len(corpus)] for j in range(4)) for i in range(args.corpus)]
    store = VectorStoreRegistry.get("documents", emb.dim, device=device)
    for i in range(0, len(docs), 8192):
        chunk = docs[i: i + 8192]
        vec = emb.embed_tensor(chunk)
        store.upsert([f"c{rank}-{j}" for j in range(i, i + len(chunk))], vec, [{"text": t} for t in chunk])
    llm = services.llm_engine(chat_model, {"chat-model": chat_model, "max-batch": fmt["max_batch"],
                                           "max-model-len": 4096, "max-prefill-tokens": args.prefill_chunk})
    if multi:
        dist_knn.start(device=device)
    # the crawler runs once (rank 0), in its own process unless LS_BENCH_CRAWLER_INPROC=1
    only = None if rank == 0 and crawler_host is None else ["query", "ingest"]
    if os.environ.get("LS_STAGE_TRACE", "0") != "0":
        _composite.STAGE_TRACE = []
        from langstream_amd.engine import vector_store as _vs
        _vs.SEARCH_TRACE = []
    runner = LocalApplicationRunner.from_yaml(files, instance=INSTANCE.format(**fmt), application_id="rag-bench",
                                              services=services, agents=only)
    runner.start()
    if crawler_host is not None:
        import atexit
        import shutil
        import tempfile
        crawler_state = tempfile.mkdtemp(prefix="rag-bench-crawler-")
        atexit.register(shutil.rmtree, crawler_state, True)
        crawler_host.start(files, INSTANCE.format(**fmt), "rag-bench", ["crawler"], state_dir=crawler_state)
    log = runner.topic_runtime.log
    barrier()
    prod = runner.producer("questions-topic")
    doc_prod = runner.producer("documents-topic")
    reader = runner.reader("log-topic")
    ingest_group = "langstream-agent-ingest"
    setup_s = time.time() - t_setup

    seq = [0]
    steps_done = [0]

    def ingest_done(expected_docs: int) -> bool:
        end = log.end_offsets("documents-topic")
        return sum(end) >= expected_docs and log.committed("documents-topic", ingest_group) == end

    def send_question():
        g = seq[0] * world + rank
        k = balanced_key(f"{rank}-{seq[0]}", g % q_parts, q_parts)
        seq[0] += 1
        sent[k] = time.time()
        prod.write(_rec(k, corpus[(g * 13) % len(corpus)]))
        return k

    sent = {}
    phases = []
    stage_trace = []

    def publish_pages(step):
        if args.docs <= 0:
            return
        if crawl:
            if site is not None:
                site.publish(step)
        else:
            for d in range(args.docs):
                i = (step * world + rank) * args.docs + d
                doc_prod.write(_rec(balanced_key(f"doc-{i}", i % d_parts, d_parts), make_page(i, corpus)))

    def thread_cpu():
        out = {}
        for th in threading.enumerate():
            try:
                out[th.name] = time.clock_gettime(time.pthread_getcpuclockid(th.ident))
            except (OSError, TypeError, AttributeError):
                pass
        return out

    def cpu_window(store, delay):
        # per-thread CPU seconds over the step's first `delay` s (the question front:
        # embed -> kNN -> MMR -> prompt), top threads -- who competes for the GIL there
        a = thread_cpu()
        time.sleep(delay)
        b = thread_cpu()
        d = sorted(((round(1e3 * (b[k] - a.get(k, 0.0)), 1), k) for k in b), reverse=True)[:10]
        store.append(d)

    cpu_front = []

    def run_step():
        step = steps_done[0]
        t0 = time.time()
        if _composite.STAGE_TRACE is not None:
            threading.Thread(target=cpu_window, args=(cpu_front, 0.6), daemon=True, name="cpu-window").start()
        publish_pages(step)
        step_keys = set()
        if args.load == "burst" or step == 0:
            for _ in range(args.batch):
                step_keys.add(send_question())
        expect_docs = (step + 1) * args.docs * world
        lats = []
        t_first = t_all = None
        deadline = time.time() + args.timeout
        while len(lats) < args.batch or (args.docs > 0 and not ingest_done(expect_docs)):
            if t_all is None and len(lats) >= args.batch:
                t_all = time.time()
            if runner.errors:
                raise runner.errors[0]
            if crawler_host is not None and not crawler_host.alive():
                raise RuntimeError("the crawler agent process exited")
            if time.time() > deadline:
                raise TimeoutError(f"rank {rank}: {args.batch - len(lats)} answers missing; documents end "
                                   f"{log.end_offsets('documents-topic')} committed "
                                   f"{log.committed('documents-topic', ingest_group)} (expected {expect_docs})")
            for r in reader.read().records:
                t = sent.pop(r.key(), None)
                if t is not None:
                    lats.append(time.time() - t)
                    if t_first is None:
                        t_first = time.time()
                    if args.load == "stream":
                        send_question()   # closed loop: keep --batch questions in flight
        steps_done[0] += 1
        t_end = time.time()
        # (first answer, last answer, step end incl. waiting for the crawled pages' indexing,
        # first / last prompt reaching the LLM scheduler), s
        arr = [a for a in list(llm.arrival_log) if t0 <= a <= t_end]
        phases.append([round((t_first or t_end) - t0, 3), round((t_all or t_end) - t0, 3), round(t_end - t0, 3),
                       round(min(arr) - t0, 3) if arr else None, round(max(arr) - t0, 3) if arr else None])
        if _composite.STAGE_TRACE is not None:
            # per stage of the fused question chain: [p10, p50, max] of entry time - t0, s
            by = {}
            for k, name, t in list(_composite.STAGE_TRACE):
                if k in step_keys and t >= t0:
                    by.setdefault(name, []).append(t - t0)
            stage_trace.append({n: [round(sorted(v)[min(len(v) - 1, int(q * len(v)))], 3) for q in (0.1, 0.5, 1.0)]
                                for n, v in by.items()})
            _composite.STAGE_TRACE.clear()
            from langstream_amd.engine import vector_store as _vs
            if _vs.SEARCH_TRACE is not None:
                # searches of this step: [start, lock wait, lock->host top-k, results build, n] (s, ms, ms, ms)
                stage_trace[-1]["searches"] = [[round(a - t0, 3), round(1e3 * (b - a), 1), round(1e3 * (c - b), 1),
                                                round(1e3 * (d - c), 1), n] for a, b, c, d, n in list(_vs.SEARCH_TRACE)
                                               if a >= t0]
                _vs.SEARCH_TRACE.clear()
            if cpu_front:
                # per-thread CPU ms over the first 0.6 s of the step: [[ms, thread], ...]
                stage_trace[-1]["thread_cpu_ms_front"] = cpu_front.pop()
        return t_end - t0, lats

    def run_window(k_steps):
        """Timed region of the streaming load.  Only questions SENT inside the window
        count: the closed loop keeps --batch in flight until k_steps * batch window
        questions have been sent, then drains them; answers to questions sent during the
        warmup (in flight when the window opens) are processed but not counted.  So the
        window's GPU work is at least the counted records' work (conservative), and the
        crawled pages of the k_steps steps are published as each batch of window
        questions starts and must be indexed before the window closes."""
        first = steps_done[0]
        quota = k_steps * args.batch
        window = set()
        lats = []
        n_sent = 0

        def send_w():
            nonlocal n_sent
            if n_sent % args.batch == 0:
                publish_pages(first + n_sent // args.batch)
            window.add(send_question())
            n_sent += 1

        while len(sent) < args.batch and n_sent < quota:
            send_w()
        expect_docs = (first + k_steps) * args.docs * world
        deadline = time.time() + args.timeout * k_steps
        while len(lats) < quota or (args.docs > 0 and not ingest_done(expect_docs)):
            if runner.errors:
                raise runner.errors[0]
            if time.time() > deadline:
                raise TimeoutError(f"rank {rank}: {quota - len(lats)} window answers missing")
            _beat(wd)
            for r in reader.read().records:
                t = sent.pop(r.key(), None)
                if t is None:
                    continue
                if r.key() in window:
                    window.discard(r.key())
                    lats.append(time.time() - t)
                if n_sent < quota:
                    send_w()
        steps_done[0] += k_steps
        return lats

    _phase(wd, "warmup", args.timeout + 300)
    for _ in range(args.warmup):
        run_step()
        _beat(wd)
    chunks0 = len(store)
    _phase(wd, "timed", args.timeout + 300)
    barrier()
    from langstream_amd.utils import threads as _threads
    cpu0 = _threads.snapshot()
    stats0 = dict(llm.stats)
    phases.clear()
    import gc
    gc_t = {"start": 0.0, "ms": 0.0, "n": [0, 0, 0]}

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t["start"] = time.perf_counter()
        else:
            gc_t["ms"] += 1000 * (time.perf_counter() - gc_t["start"])
            gc_t["n"][info["generation"]] += 1
    gc.callbacks.append(_gc_cb)
    t0 = time.time()
    my_lats = []
    if args.load == "stream":
        my_lats = run_window(args.steps)
    else:
        for _ in range(args.steps):
            _, lats = run_step()
            my_lats.extend(lats)
            _beat(wd)
    barrier()
    elapsed = time.time() - t0
    gc.callbacks.remove(_gc_cb)
    chunks = len(store) - chunks0
    if os.environ.get("LANGSTREAM_THREAD_CPU"):
        print(json.dumps({"thread_cpu_s": _threads.diff(cpu0, _threads.snapshot())}), file=sys.stderr, flush=True)
    stats = {k: v - stats0.get(k, 0) if isinstance(v, (int, float)) else v for k, v in llm.stats.items()}
    assign = {}
    for r in runner.runners:   # partitions this rank's replicas own (disjoint across ranks)
        c = getattr(getattr(r, "source", None), "consumer", None)
        if c is not None and hasattr(c, "get_info"):
            info = c.get_info()
            assign[info["topic"]] = info.get("assignment")
    stream_res = None
    if args.load == "burst" and args.also_stream > 0:
        # the same pipeline under the closed-loop load, reported beside the burst number
        barrier()
        ts0 = time.time()
        s_lats = run_window(args.also_stream)
        barrier()
        stream_res = {"elapsed": time.time() - ts0, "lats": s_lats}
    mine = {"elapsed": elapsed, "lats": my_lats, "chunks": chunks, "assign": assign, "stream": stream_res,
            "prefill_tokens": stats.get("prefill_tokens", 0), "requests": stats.get("requests", 0),
            "prompt_tokens": stats.get("prompt_tokens", 0),
            "phases": phases, "stage_trace": stage_trace, "gc": {"pause_ms": round(gc_t["ms"], 1), "collections_by_gen": gc_t["n"]},
            "knn_rounds": dist_knn.active().rounds if dist_knn.active() else 0,
            "knn_stats": ({k: (round(v, 3) if isinstance(v, float) else v) for k, v in dist_knn.active().stats.items()}
                          if dist_knn.active() else None)}
    _phase(wd, "report", 600)
    if multi:
        gathered = [None] * world
        dist.all_gather_object(gathered, mine, group=ctrl)
    else:
        gathered = [mine]
    elapsed = max(g["elapsed"] for g in gathered)
    all_lats = [x for g in gathered for x in g["lats"]]
    p50 = statistics.median(all_lats) if all_lats else 0.0
    reqs = sum(g["requests"] for g in gathered)
    # seq_len: the mean prompt length of a request (what the model attends over); the
    # prefill tokens actually computed are fewer by the prefix-KV hits, reported beside it
    prompt_toks = sum(g["prompt_tokens"] for g in gathered)
    prefill_toks = sum(g["prefill_tokens"] for g in gathered)
    mean_prompt = prompt_toks / reqs if reqs else 0.0
    hit_frac = (prompt_toks - prefill_toks) / prompt_toks if prompt_toks else 0.0
    total = args.batch * args.steps * world
    value = total / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(value, 3), "unit": "records/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "p50_latency_s": round(p50, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if use_gpu else "fp32",
            "data": "synthetic questions + synthetic crawled pages + synthetic corpus, random-init weights",
            "config": {"model": chat_model, "embedding_model": embed_model, "global_batch": args.batch * world,
                       "seq_len": round(mean_prompt, 1), "max_model_len": 4096,
                       "prefix_hit_tokens_frac": round(hit_frac, 4),
                       "prefill_tokens_per_request": round(prefill_toks / reqs, 1) if reqs else 0.0,
                       "prefill_chunk": args.prefill_chunk, "max_new_tokens": args.max_tokens,
                       "corpus_docs_per_gpu": args.corpus, "top_k": 20, "rerank": 5,
                       "crawled_pages_per_gpu_per_step": args.docs, "crawl": crawl,
                       "topics": "shm (cross-process consumer groups)",
                       "vector_store": ("HBM shard, WAL + snapshots on local disk (fsync off)" if persist_dir
                                        else "HBM shard, not persisted"),
                       "load": (f"closed loop, {args.batch} questions in flight per GPU; only questions sent "
                                f"inside the timed window count, the window drains them"
                                if args.load == "stream" else f"bursts of {args.batch} questions per GPU per step"),
                       "parallelism": f"dp{world}"},
            "ingest": {"pages_per_s": round(args.docs * args.steps * world / elapsed, 2),
                       "chunks_per_s": round(sum(g["chunks"] for g in gathered) / elapsed, 2)},
            "latency_samples": len(all_lats), "step_phases_rank0_s": gathered[0]["phases"],
            **({"stage_trace_rank0_s": gathered[0]["stage_trace"]} if gathered[0]["stage_trace"] else {}), "gc_rank0": gathered[0]["gc"], "knn_rounds_per_rank": [g["knn_rounds"] for g in gathered],
            "knn_stats_rank0": gathered[0]["knn_stats"],
            "partitions_per_rank": [g["assign"] for g in gathered],
            "setup_s": round(setup_s, 1),
            "engine_rank0": dict(stats, exec_ms=dict(zip(("upload", "enqueue", "download", "wait"),
                                                         (round(x, 1) for x in llm.exec.timings())))),
            "stream_load": _stream_summary(gathered, args, world),
            "prompt_len_pcts_rank0": _pcts(list(llm.prompt_lens)),
            "prefill_step_tokens_rank0": list(llm.prefill_step_tokens)[-40:],
        }), flush=True)
    barrier()
    if crawler_host is not None:
        crawler_host.stop()
    runner.stop(timeout=10)
    if multi:
        dist_knn.stop()
    services.shutdown()
    if site is not None:
        site.close()
    barrier()
    if rank == 0:
        unlink_shmlog(shm, size_mb=shm_mb)
    if persist_dir:
        import shutil
        VectorStoreRegistry.reset()
        shutil.rmtree(persist_dir, ignore_errors=True)
    if multi:
        dist.destroy_process_group()


def _other_config(args, rank: int, world: int, local: int) -> None:
    """BASELINE configs 2, 3 and 5 (langstream_amd/bench/)."""
    import torch
    import torch.distributed as dist
    if args.config == "chat":
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        from langstream_amd.bench import chat
        chat.run(args, rank, world, None)
        if dist.is_initialized():
            dist.destroy_process_group()
        return
    # config 2 starts its broker and load-generator processes before anything touches
    # the GPU (gloo needs no GPU), then initialises the device
    ctrl = None
    if world > 1:
        dist.init_process_group("gloo")
        ctrl = dist.group.WORLD
    gpu = [False]

    def gpu_init() -> bool:
        gpu[0] = torch.cuda.is_available()
        if gpu[0]:
            torch.cuda.set_device(local)
        return gpu[0]

    def barrier():
        if ctrl is not None:
            dist.barrier(group=ctrl)
        if gpu[0]:
            torch.cuda.synchronize()

    def bcast(obj):
        if world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=0, group=ctrl)
        return box[0]

    from langstream_amd.bench import embed
    embed.run(args, rank, world, barrier, bcast, gpu_init)
    if ctrl is not None:
        dist.destroy_process_group()


def _rec(key, value):
    from langstream_amd.api.record import SimpleRecord
    return SimpleRecord.of(key, value)


if __name__ == "__main__":
    main()
