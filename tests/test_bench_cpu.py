"""bench.py contract on CPU (gloo): ``--gpus 2`` self-launches two rank processes whose
agent replicas share the topics through the shared-memory log as ONE consumer group
(disjoint partitions), with the crawl stage and the sharded kNN in the loop."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_consumer_group_dp(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
                        "--batch", "4", "--max-tokens", "4", "--corpus", "1000", "--docs", "2"],
                       cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(line) == 1, r.stdout[-2000:]
    d = json.loads(line[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["value"] > 0
    assert d["latency_samples"] == 2 * 4
    a, b = d["partitions_per_rank"]
    for topic in ("questions-topic", "documents-topic"):
        assert a[topic] and b[topic] and not set(a[topic]) & set(b[topic])
    assert all(n > 0 for n in d["knn_rounds_per_rank"])   # queries went through the sharded kNN
    assert d["config"]["crawl"] and d["ingest"]["chunks_per_s"] > 0


def _run(args, tmp_path, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and '"metric"' in ln]
    assert len(line) == 1, r.stdout[-2000:]
    return json.loads(line[0])


def test_bench_config2_embeddings_agent_on_kafka_two_ranks(tmp_path):
    """BASELINE config 2 shape: compute-ai-embeddings agent replicas (3 agent-pod processes
    per rank, the bench default) as ONE consumer group on a Kafka topic of the in-tree
    broker (its own process); the load clients run in their own processes too."""
    d = _run(["--config", "embed", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "32"], tmp_path)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["value"] > 0
    assert d["config"]["agent_replicas_per_gpu"] == 3
    assert "Kafka" in d["metric"] and d["config"]["topics"].startswith("kafka")


def test_bench_config5_shape_tensor_parallel_chat_gateway(tmp_path):
    """BASELINE config 3/5 path: a TP=2 chat agent (rank 0 serves the websocket gateway +
    scheduler, rank 1 mirrors every engine step) answering streamed chat sessions."""
    d = _run(["--config", "chat", "--gpus", "2", "--tp", "2", "--steps", "1", "--warmup", "1", "--batch", "2",
              "--max-tokens", "6"], tmp_path)
    assert d["config"]["parallelism"] == "tp2" and d["answers"] == 2 and d["value"] > 0
    assert d["ttft_p50_ms"] > 0 and d["unit"] == "tokens/s"


def test_bench_stage_trace(tmp_path, monkeypatch):
    """LS_STAGE_TRACE=1: per-step entry times of every processor of the fused question
    chain and the per-batch kNN search timings come back in the JSON line."""
    monkeypatch.setenv("LS_STAGE_TRACE", "1")
    d = _run(["--steps", "1", "--warmup", "1", "--batch", "8", "--max-tokens", "4", "--corpus", "1000",
              "--docs", "2"], tmp_path)
    st = d["stage_trace_rank0_s"]
    assert len(st) == 2
    for step in st:
        assert any("query-vector-db" in k for k in step) and "end" in step
        p10, p50, mx = step["end"]
        assert 0 <= p10 <= p50 <= mx
        assert step["searches"] and sum(s[4] for s in step["searches"]) >= 8


def test_bench_eight_ranks_dp8_disjoint_partitions(tmp_path):
    """World 8 (the driver's scaling size) on CPU: bench.py --gpus 8 self-launches 8
    ranks whose replicas consume DISJOINT partitions of the question and document topics
    (one consumer group), every rank owns partitions, and every query went through the
    8-shard kNN service (global top-k: tests/test_distributed_cpu.py at world 8)."""
    d = _run(["--gpus", "8", "--steps", "1", "--warmup", "1", "--batch", "2", "--max-tokens", "2",
              "--corpus", "400", "--docs", "1"], tmp_path, timeout=900)
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8" and d["value"] > 0
    assert d["latency_samples"] == 8 * 2
    parts = d["partitions_per_rank"]
    assert len(parts) == 8
    for topic in ("questions-topic", "documents-topic"):
        owned = [set(p[topic]) for p in parts]
        assert all(owned), (topic, owned)
        for i in range(8):
            for j in range(i + 1, 8):
                assert not owned[i] & owned[j], (topic, i, j)
    assert all(n > 0 for n in d["knn_rounds_per_rank"])


def test_bench_config1_text_splitter_on_memory_topic(tmp_path):
    """BASELINE config 1 (CPU only): the text-splitter agent on the in-memory streaming
    cluster; every chunk the agent's own splitter predicts is read back per step."""
    d = _run(["--config", "split", "--steps", "2", "--warmup", "1", "--batch", "16"], tmp_path, timeout=300)
    assert d["n_gpus"] == 0 and d["value"] > 0 and d["steps"] == 2
    assert d["config"]["agent"] == "text-splitter" and d["config"]["streaming"] == "memory"
    assert d["chunks_per_document"] > 1 and d["chunks_per_s"] > d["value"]
