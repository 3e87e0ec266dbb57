"""Multi-process tests on CPU with the gloo backend (world_size 2).

Tensor parallelism: a TP=2 engine (rank 0 schedules, rank 1 mirrors steps through the
executor's worker loop; all-reduce after o/down, all-gather of vocab-sharded logits)
must produce the same greedy tokens as the TP=1 engine with the same full weights.
Data parallelism: each rank runs its own replica over disjoint requests; results are
gathered and must match the single-process run.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

PROMPTS = [list(range(3, 3 + n)) for n in (5, 64, 97)]
MAXTOK = 6


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _full_model():
    from langstream_amd.models.llama import LlamaModel, PRESETS
    return LlamaModel(PRESETS["llama-tiny"], device="cpu", dtype=torch.float32, seed=5)


def _single_run():
    from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
    eng = LLMEngine(_full_model(), None, num_blocks=64, max_model_len=512)
    sp = SamplingParams(max_tokens=MAXTOK, temperature=0.0, ignore_eos=True)
    return [r.output_ids for r in eng.generate(PROMPTS, sp)]


def _tp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
        from langstream_amd.models.llama import LlamaModel, PRESETS, TPInfo
        from langstream_amd.models.loader import shard_llama
        cfg = PRESETS["llama-tiny"]
        full = _full_model()
        m = LlamaModel(cfg, device="cpu", dtype=torch.float32, tp=TPInfo(rank, world, None))
        m.load_state_dict(shard_llama(full.state_dict(), cfg, rank, world))
        eng = LLMEngine(m, None, num_blocks=64, max_model_len=512)
        if rank == 0:
            sp = SamplingParams(max_tokens=MAXTOK, temperature=0.0, ignore_eos=True)
            out = [r.output_ids for r in eng.generate(PROMPTS, sp)]
            eng.stop()
            q.put(out)
        else:
            eng.worker_loop()
    finally:
        dist.destroy_process_group()


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
        eng = LLMEngine(_full_model(), None, num_blocks=64, max_model_len=512)
        mine = PROMPTS[rank::world]
        sp = SamplingParams(max_tokens=MAXTOK, temperature=0.0, ignore_eos=True)
        out = [r.output_ids for r in eng.generate(mine, sp)]
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        if rank == 0:
            res = [None] * len(PROMPTS)
            for r in range(world):
                for i, o in zip(range(r, len(PROMPTS), world), gathered[r]):
                    res[i] = o
            q.put(res)
    finally:
        dist.destroy_process_group()


def _spawn(fn, world=2, *extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q, *extra)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return out


def test_tensor_parallel_matches_single():
    assert _spawn(_tp_worker) == _single_run()


SMALL_PROMPTS = [list(range(3, 3 + n)) for n in (7, 70)]


def _small_full(cfg_name: str = "llama-small"):
    from langstream_amd.models.llama import LlamaModel
    return LlamaModel(_cfg(cfg_name), device="cpu", dtype=torch.float32, seed=9)


def _cfg(name: str):
    """llama-small, or "llama-kv8": 8 KV heads so TP=8 gives every rank exactly one KV
    head -- the Llama-3-70B TP=8 layout (64 q / 8 kv heads) at test size."""
    from langstream_amd.models.llama import LlamaConfig, PRESETS
    if name == "llama-kv8":
        return LlamaConfig(name="llama-kv8", vocab_size=2048, hidden_size=512, intermediate_size=1024, num_layers=2,
                           num_heads=16, num_kv_heads=8, head_dim=32, max_position=2048, bos_token_id=1,
                           eos_token_ids=(2,))
    return PRESETS[name]


def _small_run(model, sampled=False):
    from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
    eng = LLMEngine(model, None, num_blocks=32, max_model_len=512)
    if sampled:
        sp = SamplingParams(max_tokens=6, temperature=0.9, top_k=40, top_p=0.9, seed=123, ignore_eos=True,
                            logprobs=3)
    else:
        sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True, logprobs=2)
    tops = {}
    reqs = [eng.submit(p, sp, callback=lambda ev: tops.setdefault(ev.request_id, []).append(ev.top))
            for p in SMALL_PROMPTS]
    while not all(r.finished for r in reqs):
        eng.step()
    res = [(r.output_ids, r.output_logprobs, tops.get(r.request_id)) for r in reqs]
    return eng, res


def _tp_small_worker(rank, world, port, q, sampled=False, cfg_name="llama-small"):
    """llama-small sharded TP=world (KV heads replicated when world > 2); rank 0 reports
    tokens + logprobs."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.models.llama import LlamaModel, TPInfo
        from langstream_amd.models.loader import shard_llama
        cfg = _cfg(cfg_name)
        m = LlamaModel(cfg, device="cpu", dtype=torch.float32, tp=TPInfo(rank, world, None))
        m.load_state_dict(shard_llama(_small_full(cfg_name).state_dict(), cfg, rank, world))
        if rank == 0:
            eng, res = _small_run(m, sampled)
            eng.stop()
            q.put(res)
        else:
            from langstream_amd.engine.llm_engine import LLMEngine
            LLMEngine(m, None, num_blocks=32, max_model_len=512).worker_loop()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sampled", [(2, False), (4, False), (2, True)])
def test_tp_llama_small_logprobs_match_tp1(world, sampled):
    """TP=2 and TP=4 (2 KV heads -> replicated at TP=4) tokens, their logprobs and the
    top-n alternatives equal the TP=1 engine on the same full weights -- greedy, and
    seeded top-k/top-p sampling.  The TP engine never all-gathers full logit rows for
    greedy rows: ops.sample_vocab_parallel exchanges row statistics and candidates."""
    _, ref_res = _small_run(_small_full(), sampled)
    got = _spawn(_tp_small_worker, world, sampled)
    for (ids_a, lp_a, top_a), (ids_b, lp_b, top_b) in zip(got, ref_res):
        assert ids_a == ids_b
        assert max(abs(a - b) for a, b in zip(lp_a, lp_b)) < 1e-3
        if top_b is not None:
            assert _top_close(top_a, top_b)


def test_tp8_one_kv_head_per_rank_logprobs_match_tp1():
    """World 8, the only multi-GPU size the driver runs: Llama with 8 KV heads sharded
    TP=8 (one KV head and 2 q heads per rank, vocabulary in 8 slices, row-parallel o /
    down all-reduced over 8 ranks) gives the TP=1 tokens, log-probs and top-n."""
    _, ref_res = _small_run(_small_full("llama-kv8"))
    got = _spawn(_tp_small_worker, 8, False, "llama-kv8")
    for (ids_a, lp_a, top_a), (ids_b, lp_b, top_b) in zip(got, ref_res):
        assert ids_a == ids_b
        assert max(abs(a - b) for a, b in zip(lp_a, lp_b)) < 1e-3
        assert _top_close(top_a, top_b)


def _top_close(a, b) -> bool:
    """Per-step top-n alternatives [(token_id, logprob)]: same ids, log-probs within 1e-3."""
    if a is None or b is None or len(a) != len(b):
        return False
    for sa, sb in zip(a, b):
        if len(sa) != len(sb):
            return False
        for (ka, va), (kb, vb) in zip(sa, sb):
            if ka != kb or abs(float(va) - float(vb)) > 1e-3:
                return False
    return True


def test_data_parallel_replicas_match_single():
    assert _spawn(_dp_worker) == _single_run()


def test_shard_llama_roundtrip_shapes():
    from langstream_amd.models.llama import PRESETS
    from langstream_amd.models.loader import shard_llama
    cfg = PRESETS["llama-tiny"]
    sd = _full_model().state_dict()
    parts = [shard_llama(sd, cfg, r, 2) for r in range(2)]
    # concatenating the row-parallel shards restores the full matrix
    assert torch.equal(torch.cat([p["layers.0.o_w"] for p in parts], 1), sd["layers.0.o_w"])
    assert torch.equal(torch.cat([p["embed"] for p in parts], 0)[: cfg.vocab_size], sd["embed"])


TP_AGENT_CFG = {"steps": [{"type": "ai-chat-completions", "model": "llama-tiny"}],
                "local": {"chat-model": "llama-tiny", "device": "cpu", "num-blocks": 64,
                          "max-model-len": 512, "max-batch": 8}}


def _tp_pod_worker(rank, world, port, q):
    """The TP pod wiring: parallel.init_tensor_parallel from torchrun env, rank 0 serves
    the chat agent's completions service, rank 1 runs pod.serve_tp_worker."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from langstream_amd.parallel import init_tensor_parallel
    from langstream_amd.runtime.pod import serve_tp_worker
    from langstream_amd.services import ServiceRegistry
    reg = ServiceRegistry()
    reg.tp = init_tensor_parallel()
    try:
        if rank == 0:
            from langstream_amd.agents.genai.services import ChatMessage
            svc = reg.completions_service(TP_AGENT_CFG, "llama-tiny")
            chunks = []
            res = svc.get_chat_completions(
                [ChatMessage("user", "tell me about streaming")],
                lambda aid, i, text, last: chunks.append((i, last)),
                {"max-tokens": 7, "temperature": 0.0, "ignore-eos": True,
                 "min-chunks-per-message": 2}).result(120)
            reg.shutdown()   # stops the engine -> releases rank 1's worker loop
            q.put((res.completion_tokens, len(res.content) > 0, chunks[-1][1]))
        else:
            serve_tp_worker(TP_AGENT_CFG, reg)
    finally:
        dist.destroy_process_group()


def test_tp_pod_serves_chat_agent():
    ntok, has_text, last = _spawn(_tp_pod_worker)
    assert ntok == 7 and has_text and last


def _knn_corpus():
    g = torch.Generator().manual_seed(11)
    vecs = torch.randn(600, 48, generator=g)
    queries = torch.randn(10, 48, generator=g)
    return vecs, queries


def _sharded_knn_worker(rank, world, port, q):
    """Each rank holds a disjoint shard (rows i % world == rank) of one collection and
    asks a different subset of the queries; the service returns global top-k."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine import dist_knn
        from langstream_amd.engine.vector_store import VectorStoreRegistry
        vecs, queries = _knn_corpus()
        rows = [i for i in range(vecs.shape[0]) if i % world == rank]
        VectorStoreRegistry.get("docs", 48, device="cpu").upsert(
            [f"d{i}" for i in rows], vecs[rows].tolist(), [{"text": f"t{i}", "owner": rank} for i in rows])
        svc = dist_knn.start(device="cpu")
        mine = list(range(rank, queries.shape[0], world))
        # several concurrent requests of different k -> one round may carry them all
        futs = [svc.search("docs", queries[i:i + 1].tolist(), 7 + (i % 3), with_vectors=(i % 2 == 0)) for i in mine]
        res = {i: f.result(60)[0] for i, f in zip(mine, futs)}
        # a query for a collection nobody has
        assert svc.search("nope", queries[:1].tolist(), 3).result(60) == [[]]
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        dist_knn.stop()
        if rank == 0:
            allres = {}
            for g in gathered:
                allres.update(g)
            q.put(allres)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_knn_equals_single_store(world):
    from langstream_amd.engine.vector_store import VectorStore
    out = _spawn(_sharded_knn_worker, world)
    vecs, queries = _knn_corpus()
    single = VectorStore(48, device="cpu")          # same bf16 rows as the shards
    single.upsert([f"d{i}" for i in range(vecs.shape[0])], vecs.tolist())
    for i in range(queries.shape[0]):
        k = 7 + (i % 3)
        want = single.search(queries[i:i + 1].tolist(), k, with_vectors=True)[0]
        got = out[i]
        assert len(got) == len(want) == k
        assert all(abs(a["similarity"] - b["similarity"]) < 1e-4 for a, b in zip(got, want))
        # identical ranking except within exact score ties
        for a, b in zip(got, want):
            assert a["id"] == b["id"] or abs(a["similarity"] - b["similarity"]) < 1e-6
        assert all(d["text"] == "t" + d["id"][1:] for d in got)
        assert len({d["owner"] for d in got}) >= min(2, len(got))   # results span shards
        if i % 2 == 0:
            assert all(len(d["vector"]) == 48 for d in got)


def _allgather_bytes_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine.dist_knn import ShardedKnn
        x = ShardedKnn.__new__(ShardedKnn)       # only the byte collectives
        x.world, x.meta = world, dist.new_group(backend="gloo")
        r1 = x._allgather_bytes(b"a" * (10 if rank == 0 else 5000))   # one rank overflows the slot
        r2 = x._allgather_bytes(b"" if rank == 0 else b"xyz")          # fast path, an empty entry
        if rank == 0:
            q.put(([len(a) for a in r1], r2))
    finally:
        dist.destroy_process_group()


def test_sharded_knn_header_allgather_slot_and_overflow():
    lens, r2 = _spawn(_allgather_bytes_worker)
    assert lens == [10, 5000] and r2 == [b"", b"xyz"]


def _sharded_knn_fail_worker(rank, world, port, q):
    """Rank 1's local search raises in the first round: its own requests fail with that
    error, rank 0's requests still complete (with rank 0's rows), nobody hangs, and the
    next round is healthy on both ranks (identical collective sequence)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine import dist_knn
        from langstream_amd.engine.vector_store import VectorStoreRegistry
        vecs, queries = _knn_corpus()
        rows = [i for i in range(vecs.shape[0]) if i % world == rank]
        st = VectorStoreRegistry.get("docs", 48, device="cpu")
        st.upsert([f"d{i}" for i in rows], vecs[rows].tolist(), [{"owner": rank} for i in rows])
        orig = st.topk_rows
        calls = {"n": 0}
        if rank == 1:
            def boom(*a, **k):
                calls["n"] += 1
                if calls["n"] == 1:
                    raise MemoryError("simulated OOM in the kNN kernel")
                return orig(*a, **k)
            st.topk_rows = boom
        svc = dist_knn.start(device="cpu")
        dist.barrier()
        f1 = svc.search("docs", queries[rank:rank + 1].tolist(), 5)
        out = {}
        try:
            r = f1.result(60)[0]
            out["first"] = ("ok", sorted({d["owner"] for d in r}), len(r))
        except Exception as e:  # noqa: BLE001
            out["first"] = ("err", type(e).__name__)
        dist.barrier()
        r2 = svc.search("docs", queries[rank:rank + 1].tolist(), 5).result(60)[0]
        out["second"] = ("ok", sorted({d["owner"] for d in r2}), len(r2))
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        dist_knn.stop()
        VectorStoreRegistry.reset()
        if rank == 0:
            q.put(gathered)
    finally:
        dist.destroy_process_group()


def test_sharded_knn_local_failure_keeps_collectives_in_step():
    g = _spawn(_sharded_knn_fail_worker)
    assert g[1]["first"] == ("err", "MemoryError")
    assert g[0]["first"][0] == "ok" and g[0]["first"][2] == 5
    for r in range(2):
        assert g[r]["second"] == ("ok", [0, 1], 5)


def _slow_rank_knn_worker(rank, world, port, q):
    """A slow agent on one rank (blocked in a sleep, then busy in pure-Python work holding
    the GIL for most of each switch interval) must not stall the other ranks' kNN
    rounds: the service thread of the slow rank keeps taking part in every round."""
    import time as _t
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine import dist_knn
        from langstream_amd.engine.vector_store import VectorStoreRegistry
        vecs, queries = _knn_corpus()
        rows = [i for i in range(vecs.shape[0]) if i % world == rank]
        VectorStoreRegistry.get("docs", 48, device="cpu").upsert(
            [f"d{i}" for i in rows], vecs[rows].tolist(), [{"text": f"t{i}"} for i in rows])
        svc = dist_knn.start(device="cpu")
        slow = world - 1
        out = {}
        for phase in ("none", "sleep", "busy"):
            dist.barrier()
            t0 = _t.time()
            if rank == slow:
                if phase == "none":
                    pass
                elif phase == "sleep":
                    _t.sleep(_SLOW_S)                   # an agent blocked on a slow call
                else:
                    x = 0
                    while _t.time() - t0 < _SLOW_S:     # an agent burning CPU in Python
                        for i in range(1000):
                            x += i * i
                # the slow rank's own query still works once its agent comes back
                assert len(svc.search("docs", queries[:1].tolist(), 5).result(60)[0]) == 5
                out[phase] = {"end": _t.time()}
            else:
                lat = []
                for j in range(_FAST_QUERIES):
                    ts = _t.time()
                    res = svc.search("docs", queries[(rank + j) % 10:(rank + j) % 10 + 1].tolist(), 5).result(60)
                    lat.append(_t.time() - ts)
                    assert len(res[0]) == 5
                out[phase] = {"lat": lat, "done": _t.time()}
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        dist_knn.stop()
        if rank == 0:
            q.put(gathered)
    finally:
        dist.destroy_process_group()


_SLOW_S = 4.0
_FAST_QUERIES = 8


def test_sharded_knn_slow_rank_does_not_stall_others():
    """world-8 gloo with one slow rank; every other rank's queries finish
    while the slow rank's agent is still blocked / busy, with bounded per-query latency."""
    world = 8
    g = _spawn(_slow_rank_knn_worker, world)
    slow = g[world - 1]
    p50 = {}
    for phase in ("none", "sleep", "busy"):
        lats = sorted(x for r in g[:-1] for x in r[phase]["lat"])
        p50[phase] = lats[len(lats) // 2]
        print(phase, "p50 %.3f s  max %.3f s" % (p50[phase], lats[-1]))
        assert lats[-1] < 1.5, (phase, lats[-5:])
        if phase == "sleep":
            # an agent blocked outside the GIL costs the others nothing
            assert p50[phase] < 3 * p50["none"] + 0.1, (phase, p50)
        if phase == "busy":
            # an agent holding the GIL delays each of the slow rank's GIL hand-offs in a
            # round by up to the 1 ms switch interval the service sets: bounded, not stalled
            assert p50[phase] < 0.5, (phase, p50)
        if phase != "none":
            # every fast rank finished its queries before the slow rank's agent came back
            assert max(r[phase]["done"] for r in g[:-1]) < slow[phase]["end"], phase


def _prefix_prompts():
    g = torch.Generator().manual_seed(21)
    head = torch.randint(3, 250, (70,), generator=g).tolist()
    return [head + torch.randint(3, 250, (int(n),), generator=g).tolist() for n in (9, 33, 21, 50, 14, 40)]


def _tp_prefix_worker(rank, world, port, q):
    """TP engine whose later prompts hit the prefix cache: the KV block copies ride in
    the broadcast arena, so every rank copies its own KV shard."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
        from langstream_amd.models.llama import LlamaModel, PRESETS, TPInfo
        from langstream_amd.models.loader import shard_llama
        cfg = PRESETS["llama-tiny"]
        full = _full_model()
        m = LlamaModel(cfg, device="cpu", dtype=torch.float32, tp=TPInfo(rank, world, None))
        m.load_state_dict(shard_llama(full.state_dict(), cfg, rank, world))
        eng = LLMEngine(m, None, num_blocks=64, max_model_len=512, max_prefill_tokens=96, prefix_cache=True)
        if rank == 0:
            sp = SamplingParams(max_tokens=MAXTOK, temperature=0.0, ignore_eos=True)
            out = [r.output_ids for r in eng.generate(_prefix_prompts(), sp)]
            hits = eng.prefix.stats["hits"]
            eng.stop()
            q.put((out, hits))
        else:
            eng.worker_loop()
    finally:
        dist.destroy_process_group()


def test_tensor_parallel_prefix_cache_matches_single():
    from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
    out, hits = _spawn(_tp_prefix_worker)
    assert hits >= 2
    eng = LLMEngine(_full_model(), None, num_blocks=64, max_model_len=512, prefix_cache=False)
    sp = SamplingParams(max_tokens=MAXTOK, temperature=0.0, ignore_eos=True)
    assert out == [r.output_ids for r in eng.generate(_prefix_prompts(), sp)]
