"""End-to-end numerics of the GPU models/engines against the same weights on CPU
(fp32 PyTorch reference ops)."""
import pytest
import torch

from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
from langstream_amd.models.bert import BertEncoder, PRESETS as BERT_PRESETS
from langstream_amd.models.llama import AttnMeta, LlamaModel, PRESETS
from langstream_amd import ops

pytestmark = pytest.mark.gpu


def _cos(a, b):
    a, b = a.float().flatten().cpu(), b.float().flatten().cpu()
    return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-12))


def _cpu_copy(model: LlamaModel) -> LlamaModel:
    cpu = LlamaModel(model.cfg, device="cpu", dtype=torch.float32)
    cpu.load_state_dict({k: v.float().cpu() for k, v in model.state_dict().items()})
    return cpu


def _first_token_tops(e: LLMEngine, prompts, n_top=20):
    """First sampled token of each prompt with its top-n (id, logprob) alternatives."""
    events = {}
    reqs = [e.submit(p, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True, logprobs=n_top),
                     callback=lambda ev, i=i: events.setdefault(i, ev)) for i, p in enumerate(prompts)]
    while not all(r.finished for r in reqs):
        e.step()
    e._flush()
    return [events[i] for i in range(len(prompts))]


def test_llama_prefill_logits_match_cpu():
    cfg = PRESETS["llama-small"]
    gpu = LlamaModel(cfg, device="cuda")
    cpu = _cpu_copy(gpu)
    prompts = [list(range(5, 5 + n)) for n in (7, 70, 130)]
    eg = _first_token_tops(LLMEngine(gpu, None, num_blocks=64, max_model_len=1024), prompts)
    ec = _first_token_tops(LLMEngine(cpu, None, num_blocks=64, max_model_len=1024), prompts)
    for g, c in zip(eg, ec):
        cmap = dict(c.top)
        # bf16 vs fp32: the GPU's argmax is (near-)argmax on the CPU, same max log-prob
        assert g.token_id in cmap and cmap[g.token_id] >= c.top[0][1] - 0.05
        assert abs(g.top[0][1] - c.top[0][1]) < 0.05
        assert len(set(t for t, _ in g.top) & set(cmap)) >= 10


def _step_tops(e: LLMEngine, prompts, n_gen: int, n_top=10):
    """Per prompt, the top-n (id, logprob) alternatives of each generated token."""
    events = {}
    reqs = [e.submit(p, SamplingParams(max_tokens=n_gen, temperature=0.0, ignore_eos=True, logprobs=n_top),
                     callback=lambda ev, i=i: events.setdefault(i, []).append(ev)) for i, p in enumerate(prompts)]
    while not all(r.finished for r in reqs):
        e.step()
    e._flush()
    return [events[i] for i in range(len(prompts))]


def _close_tops(g, c, tol=0.05):
    cmap = dict(c.top)
    assert g.token_id in cmap and cmap[g.token_id] >= c.top[0][1] - tol
    assert abs(g.top[0][1] - c.top[0][1]) < tol


@pytest.mark.parametrize("M", [5, 33, 64, 100, 128, 300, 700])
def test_runner_projection_routing_at_m_rows_matches_fp32(M):
    """Every projection route of LlamaRunner at M rows against the same weights in fp32 on
    the CPU: a prefill step of M tokens (one prompt) and a decode-only step of M rows (M
    sequences).  5..128 rows run the 256-row decode GEMM (rows past M read as zeros) and
    the skinny kernels, 300 / 700 the decode GEMM in 256-row blocks; no library GEMM."""
    cfg = PRESETS["llama-small"]
    gpu = LlamaModel(cfg, device="cuda")
    cpu = _cpu_copy(gpu)
    torch.manual_seed(M)
    # prefill of M rows
    prompt = [[int(t) for t in torch.randint(5, 30000, (M,))]]
    kw = dict(num_blocks=2048, max_model_len=1024, max_batch=1024, max_prefill_tokens=4096)
    g = _first_token_tops(LLMEngine(gpu, None, **kw), prompt)[0]
    c = _first_token_tops(LLMEngine(cpu, None, **kw), prompt)[0]
    _close_tops(g, c)
    # decode-only step of M rows: M prompts of 3 tokens prefilled together, then every
    # sequence decodes its second token in one step
    prompts = [[int(t) for t in torch.randint(5, 30000, (3,))] for _ in range(M)]
    eg = _step_tops(LLMEngine(gpu, None, use_graphs=False, **kw), prompts, 2)
    ec = _step_tops(LLMEngine(cpu, None, **kw), prompts, 2)
    same = 0
    for a, b in zip(eg, ec):
        _close_tops(a[0], b[0])
        if a[0].token_id == b[0].token_id:   # else a near-tie split the inputs of step 2
            _close_tops(a[1], b[1])
            same += 1
    assert same >= 0.8 * M


def test_native_runner_matches_python_forward():
    """The C++ LlamaRunner and the Python op-by-op forward issue the same kernels:
    logits must agree to bf16 rounding on a two-sequence prefill."""
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    kv = [ops.new_kv_cache(16, model.hkv, cfg.head_dim, "cuda", model.dtype) for _ in range(cfg.num_layers)]
    lens = [70, 100]
    T = sum(lens)
    ids = torch.randint(5, 1000, (T,), dtype=torch.int32, device="cuda")
    pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens]).cuda()
    bt = torch.tensor([[0, 1, 0, 0], [2, 3, 0, 0]], dtype=torch.int32, device="cuda")
    slots = torch.cat([bt[s].long()[torch.arange(n) // 64].cpu() * 64 + torch.arange(n) % 64
                       for s, n in enumerate(lens)]).cuda()
    G = model.hq // model.hkv
    meta = AttnMeta(positions=pos, slots=slots, num_decode=0, num_prefill_tokens=T, p_block_tables=bt,
                    q_start=torch.tensor([0, 70], dtype=torch.int32, device="cuda"),
                    q_len=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                    ctx_len=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                    tiles=ops.prefill_tiles(lens, G).cuda())
    rows = torch.tensor([69, 169], dtype=torch.long, device="cuda")
    a = model.forward_logits(ids, meta, kv, rows).float().cpu()
    b = model.logits(model.forward(ids, meta, kv).index_select(0, rows)).float().cpu()
    for i in range(2):
        assert _cos(a[i], b[i]) > 0.999


def _run_tops(e: LLMEngine, prompts, sp: SamplingParams):
    """Run to completion; per request the output ids and each step's top-n alternatives
    (None when sp.logprobs == 0 -- the only mode the decode graphs serve)."""
    tops = {}
    reqs = [e.submit(p, sp, callback=lambda ev, i=i: tops.setdefault(i, []).append(ev.top))
            for i, p in enumerate(prompts)]
    while not all(r.finished for r in reqs):
        e.step()
    e._flush()
    return [(r.output_ids, tops.get(i)) for i, r in enumerate(reqs)]


def _same_or_near_tie(a, b, gap: float = 0.1) -> None:
    """Greedy sequences from two bf16 paths agree over their WHOLE length, except that
    they may part at a genuine near-tie: at the first differing position both tokens are
    in b's top-2 and within `gap` nats of each other (random-init weights have top-2 gaps
    of ~1e-3 nats, so rounding may flip argmax there).  After such a split the sequences
    condition on different tokens and are not compared."""
    (ids_a, _), (ids_b, tops_b) = a, b
    assert len(ids_a) == len(ids_b)
    for t, (x, y) in enumerate(zip(ids_a, ids_b)):
        if x == y:
            continue
        alt = dict(tops_b[t])
        assert x in alt and y in alt and abs(alt[x] - alt[y]) < gap, (t, x, y, tops_b[t])
        return


def test_native_executor_matches_python_executor():
    """Whole-step native executor (arena upload, feedback gather, graphs, sampling)
    against the Python executor driving the same model on the same GPU."""
    from langstream_amd.engine.arena import PyStepExecutor
    from langstream_amd.engine.llm_engine import NSLOTS
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    prompts = [list(range(3, 3 + n)) for n in (5, 33, 64, 65, 200)]
    sp = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True)
    sp_ref = SamplingParams(max_tokens=16, temperature=0.0, ignore_eos=True, logprobs=2)
    e1 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, max_batch=8)
    out1 = _run_tops(e1, prompts, sp)
    assert e1.stats["graph_steps"] > 0
    e2 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, max_batch=8, use_graphs=False)
    e2.exec = PyStepExecutor(model, e2.kv_caches, e2.layout, NSLOTS, e2.nsplit, e2.bps, e2.device)
    out2 = _run_tops(e2, prompts, sp_ref)
    for a, b in zip(out1, out2):
        _same_or_near_tie(a, b)


@pytest.mark.parametrize("n", [1, 2, 3, 4])
def test_batch_le4_fused_gemv_decode_matches_python_executor(n):
    """Decode batches of 1-4 rows take the runner's fused GEMV layer (gemm_gemv.hip: qkv
    with RoPE + KV write, o, gate_up with SwiGLU, down; the add + RMSNorm in the next
    GEMV's prologue up to 2 rows, a separate fused_add_rmsnorm above): greedy tokens of
    the native executor (graphs) against the Python executor.  The model's dimensions are
    multiples of 512 (llama-small's 2816-wide MLP is not, so it never reaches this path)."""
    from langstream_amd.engine.arena import PyStepExecutor
    from langstream_amd.engine.llm_engine import NSLOTS
    from langstream_amd.models.llama import LlamaConfig
    cfg = LlamaConfig(name="llama-gemv", vocab_size=32000, hidden_size=1024, intermediate_size=3072, num_layers=4,
                      num_heads=8, num_kv_heads=2, head_dim=128, max_position=4096, bos_token_id=1, eos_token_ids=(2,))
    model = LlamaModel(cfg, device="cuda")
    prompts = [list(range(3 + 7 * i, 3 + 7 * i + n_tok)) for i, n_tok in enumerate((5, 70, 129, 300)[:n])]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    sp_ref = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True, logprobs=2)
    e1 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, max_batch=8)
    out1 = _run_tops(e1, prompts, sp)
    assert e1.stats["graph_steps"] > 0
    e2 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, max_batch=8, use_graphs=False)
    e2.exec = PyStepExecutor(model, e2.kv_caches, e2.layout, NSLOTS, e2.nsplit, e2.bps, e2.device)
    out2 = _run_tops(e2, prompts, sp_ref)
    for a, b in zip(out1, out2):
        _same_or_near_tie(a, b)


def test_llama_graph_decode_matches_eager():
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    prompts = [list(range(3, 3 + n)) for n in (5, 33, 64, 65, 200)]
    sp = SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True)
    e1 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, use_graphs=True, max_batch=8)
    out1 = _run_tops(e1, prompts, sp)
    assert e1.stats["graph_steps"] > 0
    e2 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, use_graphs=False, max_batch=8)
    out2 = _run_tops(e2, prompts, SamplingParams(max_tokens=24, temperature=0.0, ignore_eos=True, logprobs=2))
    # the same kernels replayed from a graph: identical over the whole length (a split
    # is only tolerated at a genuine near-tie)
    for a, b in zip(out1, out2):
        _same_or_near_tie(a, b, gap=0.02)


def test_llama_chunked_prefill_consistent():
    """Whole vs 100-token-chunked prefill: the prefill's and the first decode step's
    top-20 distributions agree to bf16 noise.  (Greedy token equality is not asserted:
    random-init logits have top-2 gaps of 1e-3 nats, so argmax flips on rounding.)"""
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    prompt = list(range(10, 10 + 300))

    def run(chunk):
        events = []
        e = LLMEngine(model, None, num_blocks=64, max_model_len=1024, max_prefill_tokens=chunk)
        r = e.submit(prompt, SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True, logprobs=20),
                     callback=events.append)
        while not r.finished:
            e.step()
        e._flush()
        return events

    ea, eb = run(4096), run(100)
    for step in range(2):
        ta, tb = dict(ea[step].top), dict(eb[step].top)
        common = set(ta) & set(tb)
        assert len(common) >= 15, (step, ta, tb)
        assert max(abs(ta[t] - tb[t]) for t in common) < 0.05, (step, ta, tb)
        if ea[0].token_id != eb[0].token_id:
            break  # the decode step conditions on different tokens


def test_bert_encoder_matches_cpu():
    cfg = BERT_PRESETS["bge-small-en"]
    gpu = BertEncoder(cfg, device="cuda")
    cpu = BertEncoder(cfg, device="cpu", dtype=torch.float32)
    cpu.load_state_dict({k: v.float().cpu() for k, v in gpu.state_dict().items()})
    toks = [[101] + list(range(1000, 1000 + n)) + [102] for n in (3, 50, 200)]
    eg = gpu.encode_tokens(toks)
    ec = cpu.encode_tokens(toks)
    for i in range(len(toks)):
        assert _cos(eg[i], ec[i]) > 0.995
    assert torch.allclose(eg.norm(dim=-1).cpu(), torch.ones(3), atol=1e-3)


def test_vector_store_search():
    from langstream_amd.engine.vector_store import VectorStore
    vs = VectorStore(384, device="cuda")
    torch.manual_seed(0)
    v = torch.randn(3000, 384)
    vs.upsert(list(range(3000)), v, [{"text": f"doc{i}"} for i in range(3000)])
    vs.delete([5, 17])
    res = vs.search(v[[7, 100]], k=3)
    assert res[0][0]["id"] == 7 and res[0][0]["text"] == "doc7"
    assert res[1][0]["id"] == 100
    assert abs(res[0][0]["similarity"] - 1.0) < 1e-2
    assert vs.search(v[[5]], k=1)[0][0]["id"] != 5


@pytest.mark.parametrize("oneshot", [False, True])
def test_native_executor_tp_path_world1_rccl(oneshot, monkeypatch):
    """The TP code path of the native executor at world size 1 over a real RCCL process
    group: all-reduces inside the graph-captured forward, and the vocab-parallel sampler
    (statistics / histogram / candidate exchanges) instead of the single-GPU sampler.
    Same greedy tokens and log-probs as the non-TP executor on the same weights.
    oneshot: the per-layer all-reduces go through allreduce.hip (LS_ONESHOT_AR=1)."""
    import socket
    if oneshot:
        monkeypatch.setenv("LS_ONESHOT_AR", "1")
    import torch.distributed as dist
    from langstream_amd.models.llama import TPInfo
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        cfg = PRESETS["llama-small"]
        m0 = LlamaModel(cfg, device="cuda")
        m1 = LlamaModel(cfg, device="cuda", tp=TPInfo(0, 1, None, force_pg=True))
        m1.load_state_dict(m0.state_dict())
        prompts = [list(range(3, 3 + n)) for n in (5, 33, 64, 200)]
        e0 = LLMEngine(m0, None, num_blocks=128, max_model_len=1024, max_batch=8)
        e1 = LLMEngine(m1, None, num_blocks=128, max_model_len=1024, max_batch=8)
        e1.capture_graphs()
        a, b = _first_token_tops(e0, prompts, 5), _first_token_tops(e1, prompts, 5)
        for x, y in zip(a, b):
            assert x.token_id == y.token_id
            assert abs(x.logprob - y.logprob) < 0.05
            assert [t for t, _ in x.top[:2]] == [t for t, _ in y.top[:2]]
        out1 = _run_tops(e1, prompts, SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))
        out0 = _run_tops(e0, prompts, SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True, logprobs=2))
        assert e1.stats["graph_steps"] > 0
        for x, y in zip(out1, out0):
            _same_or_near_tie(x, y)
        spr = SamplingParams(max_tokens=8, temperature=0.8, top_k=20, top_p=0.9, seed=5, ignore_eos=True)
        for r in e1.generate(prompts, spr):
            assert len(r.output_ids) == 8 and all(0 <= t < cfg.vocab_size for t in r.output_ids)
        e0.stop()
        e1.stop()
    finally:
        dist.destroy_process_group()


def test_prefill_gate_up_gemm_in_model(monkeypatch):
    """A prefill step of >= 8192 tokens (3 sequences of 2800, within llama-small's 4096
    positions) runs gate_up on gemm_prefill.hip with the SwiGLU epilogue (native runner
    and Python forward); its logits match the hipBLASLt + silu_and_mul forward."""
    import langstream_amd.models.llama as llama_mod
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    lens = [2800, 2800, 2800]
    n = sum(lens)
    bps = (max(lens) + 63) // 64
    nblk = bps * len(lens)
    assert max(lens) <= cfg.max_position
    kv = [ops.new_kv_cache(nblk, model.hkv, cfg.head_dim, "cuda", model.dtype) for _ in range(cfg.num_layers)]
    ids = torch.randint(5, 1000, (n,), dtype=torch.int32, device="cuda")
    pos = torch.cat([torch.arange(m, dtype=torch.int32) for m in lens]).cuda()
    bt = torch.arange(nblk, dtype=torch.int32, device="cuda").view(len(lens), bps)
    slots = torch.cat([bt[s].long()[torch.arange(m) // 64].cpu() * 64 + torch.arange(m) % 64
                       for s, m in enumerate(lens)]).cuda()
    G = model.hq // model.hkv
    starts = [sum(lens[:i]) for i in range(len(lens))]
    meta = AttnMeta(positions=pos, slots=slots, num_decode=0, num_prefill_tokens=n, p_block_tables=bt,
                    q_start=torch.tensor(starts, dtype=torch.int32, device="cuda"),
                    q_len=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                    ctx_len=torch.tensor(lens, dtype=torch.int32, device="cuda"),
                    tiles=ops.prefill_tiles(lens, G).cuda())
    rows = torch.tensor([s + m - 1 for s, m in zip(starts, lens)], dtype=torch.long, device="cuda")
    assert llama_mod._pgemm(torch.empty(n, cfg.hidden_size, device="cuda", dtype=torch.bfloat16),
                            model.layers[0].gate_up_w, True)
    native = model.forward_logits(ids, meta, kv, rows).float().cpu()
    fused = model.logits(model.forward(ids, meta, kv).index_select(0, rows)).float().cpu()
    monkeypatch.setattr(llama_mod, "_PGEMM", 0)
    lib = model.logits(model.forward(ids, meta, kv).index_select(0, rows)).float().cpu()
    for i in range(len(lens)):
        assert _cos(fused[i], lib[i]) > 0.999
        assert _cos(native[i], lib[i]) > 0.999


# ------------------------------------------------------------------ native TP, 2 ranks
_TP_PROMPTS = [list(range(3, 3 + n)) for n in (5, 33, 64, 200)]


def _tp_native_worker(rank, world, port, q, oneshot=False, graphs=False):
    """One TP rank on cuda:0 over a gloo process group: the NATIVE step executor (C++
    forward, per-layer all-reduces through c10d, vocab-parallel sampling); rank 0 drives
    the engine, the other ranks run StepExecutor::worker_loop (pure C++)."""
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if oneshot:
        os.environ["LS_ONESHOT_AR"] = "1"   # read when the runner is built
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from langstream_amd.models.llama import TPInfo
        from langstream_amd.models.loader import shard_llama
        cfg = PRESETS["llama-small"]
        full = LlamaModel(cfg, device="cpu", dtype=torch.float32, seed=9)
        m = LlamaModel(cfg, device="cuda", tp=TPInfo(rank, world, None))
        m.load_state_dict(shard_llama(full.state_dict(), cfg, rank, world))
        eng = LLMEngine(m, None, num_blocks=128, max_model_len=1024, max_batch=8, use_graphs=graphs)
        if rank == 0:
            # decode graphs serve logprobs == 0 steps only (the reference run keeps top-2)
            sp = SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True, logprobs=0 if graphs else 2)
            out = _run_tops(eng, _TP_PROMPTS, sp)
            stats = dict(eng.stats)
            eng.stop()
            q.put((out, stats))
        else:
            eng.worker_loop()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("oneshot,graphs", [(False, False), (True, False), (True, True)])
def test_native_executor_tp2_two_ranks_one_gpu(oneshot, graphs):
    """TP = 2 with two real ranks (two processes sharing cuda:0, gloo collectives on GPU
    tensors): the native executor's worker loop, arena broadcast, per-layer all-reduces
    and vocab-parallel sampling produce the TP = 1 engine's greedy tokens (up to genuine
    near-ties) on the same full weights.  RCCL cannot put two ranks on one GPU; this is
    the multi-rank run of the C++ TP path available on a 1-GPU box.  oneshot: the
    per-layer all-reduces run allreduce.hip between the two processes (IPC-mapped
    buffers, the xGMI one-shot protocol) instead of c10d, and so do the sampler's
    all-gathers and histogram all-reduce; with graphs, whole TP decode steps -- every
    collective included -- are captured and replayed on both ranks."""
    import multiprocessing as mp
    import socket
    cfg = PRESETS["llama-small"]
    full = LlamaModel(cfg, device="cpu", dtype=torch.float32, seed=9)
    m0 = LlamaModel(cfg, device="cuda")
    m0.load_state_dict(full.state_dict())
    e0 = LLMEngine(m0, None, num_blocks=128, max_model_len=1024, max_batch=8, use_graphs=False)
    ref = _run_tops(e0, _TP_PROMPTS, SamplingParams(max_tokens=10, temperature=0.0, ignore_eos=True, logprobs=2))
    e0.stop()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_native_worker, args=(r, 2, port, q, oneshot, graphs)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got, stats = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert stats["decode_steps"] > 0
    if graphs:
        assert stats["graph_steps"] > 0, stats
    for a, b in zip(got, ref):
        _same_or_near_tie(a, b)


def test_norm_deferred_decode_layer_matches_python_executor():
    """Decode batches of 129..256 rows run the norm-deferred layer (LlamaRunner::
    forward_dgemm: in-launch split-K combines, 1/rms in the consumer epilogues): greedy
    tokens against the Python executor's op-by-op path over 160 concurrent sequences."""
    from langstream_amd.engine.arena import PyStepExecutor
    from langstream_amd.engine.llm_engine import NSLOTS
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    prompts = [list(range(3 + i % 50, 3 + i % 50 + 5 + i % 37)) for i in range(160)]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    e1 = LLMEngine(model, None, num_blocks=512, max_model_len=512, max_batch=256)
    out1 = _run_tops(e1, prompts, sp)
    assert e1.stats["graph_steps"] > 0
    e2 = LLMEngine(model, None, num_blocks=512, max_model_len=512, max_batch=256, use_graphs=False)
    e2.exec = PyStepExecutor(model, e2.kv_caches, e2.layout, NSLOTS, e2.nsplit, e2.bps, e2.device)
    out2 = _run_tops(e2, prompts, SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True, logprobs=2))
    for a, b in zip(out1, out2):
        _same_or_near_tie(a, b)


def test_prefix_cache_native_matches_no_cache():
    """Prefix KV reuse on the native executor: the KV block copies ride in the step
    arena (kv_block_copy_kernel ahead of the forward); greedy outputs match the engine
    without the cache (bf16: equal up to near-ties), and the reused tokens were not
    prefilled again."""
    import numpy as np
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    rng = np.random.default_rng(7)
    head = rng.integers(3, 30000, 150).tolist()
    prompts = [head + rng.integers(3, 30000, int(rng.integers(10, 200))).tolist() for _ in range(12)]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    sp_ref = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True, logprobs=2)
    kw = dict(num_blocks=256, max_model_len=1024, max_batch=16, max_prefill_tokens=256)
    on = LLMEngine(model, None, prefix_cache=True, **kw)
    out_on = _run_tops(on, prompts, sp)
    off = LLMEngine(model, None, prefix_cache=False, **kw)
    out_off = _run_tops(off, prompts, sp_ref)
    for a, b in zip(out_on, out_off):
        _same_or_near_tie(a, b)
    assert on.prefix.stats["hits"] >= 4 and on.stats["prefix_hit_tokens"] >= 4 * 128
    assert off.stats["prefill_tokens"] - on.stats["prefill_tokens"] == on.stats["prefix_hit_tokens"]
    held = sum(len(e.blocks) for e in on.prefix.entries)
    assert on.allocator.num_free() + held == 256
