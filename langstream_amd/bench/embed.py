"""BASELINE config 2: the compute-ai-embeddings agent (bge-small-en bf16 on the GPU)
over batched records on a Kafka topic.

The pipeline is the reference's embeddings step shape (ComputeAIEmbeddingsStep.java:
66-250: Mustache text -> OrderedAsyncBatchExecutor(batch-size, flush-interval,
concurrency) -> one computeEmbeddings call per batch) reading ``input-topic`` and
writing ``output-topic`` of the in-tree Kafka-protocol broker (streaming type
``kafka``; rank 0 hosts the broker, every rank's agent replica joins the consumer group
``langstream-agent-embed`` -- replica DP as the reference scales).  A step = B records
per GPU produced at once; the step ends when all of them are committed by the group.
The broker and the clients that feed and count the topics (bench/embed_load.py) run in
their own processes, as Kafka and the applications around an agent pod do; set
``LS_EMBED_INPROC=1`` to put all of them in the agent's interpreter instead.
"""
from __future__ import annotations

import json
import os
import time

PIPE = """
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
    partitions: {parts}
  - name: "output-topic"
    creation-mode: create-if-not-exists
    partitions: {parts}
pipeline:
  - name: "compute-embeddings"
    id: "embed"
    type: "compute-ai-embeddings"
    input: "input-topic"
    output: "output-topic"
    configuration:
      model: "{model}"
      embeddings-field: "value.embeddings"
      text: "{{{{ value.text }}}}"
      batch-size: {batch_size}
      concurrency: 4
      flush-interval: 5
    resources:
      parallelism: {replicas}
"""

CONFIG = """
configuration:
  resources:
    - type: "local-gpu-configuration"
      name: "local"
      configuration:
        embeddings-model: "{model}"
"""

INSTANCE = """
instance:
  streamingCluster:
    type: "kafka"
    configuration:
      admin:
        bootstrap.servers: "{bootstrap}"
  computeCluster:
    type: "none"
"""

METRIC = "records/sec (whole node), compute-ai-embeddings agent on Kafka records, bge-small-en"


def run(args, rank: int, world: int, barrier, bcast, gpu_init=None) -> None:
    broker = None
    inproc = bool(os.environ.get("LS_EMBED_INPROC"))
    if rank == 0:
        # the broker runs in its own interpreter, as the reference's Kafka runs in its
        # own JVM; like the load generator it starts before anything touches the GPU
        from ..topics.kafka.broker import BrokerProcess, KafkaBroker
        parts0 = max(2, 2 * world * args.embed_replicas)
        broker = KafkaBroker(default_partitions=parts0).start() if inproc else BrokerProcess(partitions=parts0)
    bootstrap = bcast(broker.bootstrap if broker else None)
    B = args.batch
    load = None
    if not inproc:
        from .embed_load import LoadProcess
        load = LoadProcess(bootstrap, rank, world, B, read=rank == 0, timeout=args.timeout)
    import torch
    from ..runtime.local import LocalApplicationRunner
    from ..services import ServiceRegistry
    R = args.embed_replicas
    if R > 1:
        # the replicas are agent-pod processes with their own engines: this process never
        # touches the GPU (so it may start them), it only counts devices
        use_gpu = torch.cuda.device_count() > 0
    else:
        use_gpu = gpu_init() if gpu_init is not None else torch.cuda.is_available()
    model = args.embed_model if use_gpu else "bert-tiny"
    parts = max(2, 2 * world * R)
    services = ServiceRegistry({"device": f"cuda:{int(os.environ.get('LOCAL_RANK', '0') or 0)}" if use_gpu else "cpu"})
    ServiceRegistry.set_default(services)
    if R == 1:
        services.embedding_engine(model, {"embeddings-model": model})
    files = {"pipeline.yaml": PIPE.format(model=model, parts=parts, batch_size=args.embed_batch, replicas=R),
             "configuration.yaml": CONFIG.format(model=model)}
    runner = LocalApplicationRunner.from_yaml(files, instance=INSTANCE.format(bootstrap=bootstrap),
                                              application_id="embed-bench", services=services,
                                              replica_processes=True).start(wait=600.0)
    if inproc:
        # LS_EMBED_INPROC=1: clients and broker share the agent's interpreter (GIL)
        from ..tokenizers import builtin_corpus
        from .embed_load import make_records
        corpus = builtin_corpus(20000)
        prod = runner.producer("input-topic")
        reader = runner.reader("output-topic") if rank == 0 else None   # rank 0 counts every replica's output
    seen = [0]

    def step(i):
        if load is not None:
            load.produce(i)
            return
        prod.write_many(make_records(corpus, rank, world, B, i)).result(60)

    def wait_all(total):
        if rank != 0:
            return
        deadline = time.time() + args.timeout
        if load is not None:
            seen[0] = load.wait(total)
            if runner.errors:
                raise runner.errors[0]
            if seen[0] < total:
                raise TimeoutError(f"embed bench: {seen[0]} of {total} embedded records")
            return
        while seen[0] < total:
            if runner.errors:
                raise runner.errors[0]
            if time.time() > deadline:
                raise TimeoutError(f"embed bench: {seen[0]} of {total} embedded records")
            seen[0] += len(reader.read().records)

    for w in range(args.warmup):
        step(w)
        barrier()
        wait_all((w + 1) * B * world)
    barrier()
    t0 = time.time()
    for s in range(args.steps):
        step(args.warmup + s)
    wait_all((args.warmup + args.steps) * B * world)
    barrier()
    elapsed = time.time() - t0
    if rank == 0:
        total = args.steps * B * world
        print(json.dumps({
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "records/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if use_gpu else "fp32", "data": "synthetic text records (builtin corpus), random-init weights",
            "config": {"model": model, "records_per_gpu_per_step": B, "batch-size": args.embed_batch,
                       "concurrency": 4, "topics": "kafka (in-tree broker, own process)",
                       "agent_replicas_per_gpu": R, "parallelism": f"dp{world}"}}),
              flush=True)
    barrier()
    runner.stop(10)
    services.shutdown()
    if load is not None:
        load.close()
    if broker is not None:
        broker.stop()
