"""BASELINE config 2: the compute-ai-embeddings agent (bge-small-en bf16 on the GPU)
over batched records on a Kafka topic.

The pipeline is the reference's embeddings step shape (ComputeAIEmbeddingsStep.java:
66-250: Mustache text -> OrderedAsyncBatchExecutor(batch-size, flush-interval,
concurrency) -> one computeEmbeddings call per batch) reading ``input-topic`` and
writing ``output-topic`` of the in-tree Kafka-protocol broker (streaming type
``kafka``; rank 0 hosts the broker, every rank's agent replica joins the consumer group
``langstream-agent-embed`` -- replica DP as the reference scales).  A step = B records
per GPU produced at once; the step ends when all of them are committed by the group.
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


def run(args, rank: int, world: int, barrier, bcast) -> None:
    import torch
    from ..api.record import SimpleRecord
    from ..runtime.local import LocalApplicationRunner
    from ..services import ServiceRegistry
    from ..tokenizers import builtin_corpus
    use_gpu = torch.cuda.is_available()
    model = args.embed_model if use_gpu else "bert-tiny"
    broker = None
    if rank == 0:
        from ..topics.kafka.broker import KafkaBroker
        broker = KafkaBroker(default_partitions=max(2, 2 * world)).start()
    bootstrap = bcast(broker.bootstrap if broker else None)
    parts = max(2, 2 * world)
    services = ServiceRegistry({"device": f"cuda:{int(os.environ.get('LOCAL_RANK', '0') or 0)}" if use_gpu else "cpu"})
    ServiceRegistry.set_default(services)
    services.embedding_engine(model, {"embeddings-model": model})
    files = {"pipeline.yaml": PIPE.format(model=model, parts=parts, batch_size=args.embed_batch),
             "configuration.yaml": CONFIG.format(model=model)}
    runner = LocalApplicationRunner.from_yaml(files, instance=INSTANCE.format(bootstrap=bootstrap),
                                              application_id="embed-bench", services=services).start()
    corpus = builtin_corpus(20000)
    prod = runner.producer("input-topic")
    reader = runner.reader("output-topic") if rank == 0 else None   # rank 0 counts every replica's output
    B = args.batch
    seen = [0]

    def step(i):
        futs = []
        for j in range(B):
            g = (i * world + rank) * B + j
            text = " ".join(corpus[(g * 7 + k) % len(corpus)] for k in range(3))
            futs.append(prod.write(SimpleRecord.of(f"r{rank}-{g}", json.dumps({"text": text}))))
        for f in futs:
            f.result(60)

    def wait_all(total):
        if reader is None:
            return
        deadline = time.time() + args.timeout
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
                       "concurrency": 4, "topics": "kafka (in-tree broker)", "parallelism": f"dp{world}"}}),
              flush=True)
    barrier()
    runner.stop(10)
    services.shutdown()
    if broker is not None:
        broker.stop()
