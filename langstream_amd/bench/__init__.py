"""Driver-runnable benchmarks of the BASELINE configs other than the headline RAG
pipeline (bench.py --config ...):

* ``embed`` -- config 2: the compute-ai-embeddings agent (bge-small-en, GPU) over
  records on a Kafka topic (the in-tree Kafka-protocol broker), records/s.
* ``chat``  -- config 3 (``--tp 1``): ai-chat-completions through the WebSocket chat
  gateway, TTFT and tokens/s; config 5 is the same path with ``--model llama-3-70b
  --gpus 8 --tp 8`` (one tensor-parallel chat agent over 8 GPUs, RCCL all-reduces).
"""
