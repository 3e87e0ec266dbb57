"""LLM engine scheduler on CPU (llama-tiny, fp32): the same arena/scheduler code the GPU
path uses, run by the Python step executor.  Checks continuous batching, chunked
prefill, lookahead, preemption, stop conditions, penalties and logprobs against a
plain full-recompute reference."""
import numpy as np
import pytest
import torch

from langstream_amd import ops
from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams
from langstream_amd.models.llama import AttnMeta, LlamaModel, PRESETS


@pytest.fixture(scope="module")
def model():
    return LlamaModel(PRESETS["llama-tiny"], device="cpu", dtype=torch.float32, seed=3)


def _greedy_reference(model, prompt, n):
    """Greedy decode by recomputing the whole sequence every token (no KV reuse)."""
    cfg = model.cfg
    kv = []
    nb = 16
    for _ in range(cfg.num_layers):
        kv.append(ops.new_kv_cache(nb, model.hkv, cfg.head_dim, "cpu", torch.float32))
    ids = list(prompt)
    out = []
    for _ in range(n):
        T = len(ids)
        slots = torch.arange(T, dtype=torch.int64)
        meta = AttnMeta(positions=torch.arange(T, dtype=torch.int32), slots=slots, num_decode=0,
                        num_prefill_tokens=T, p_block_tables=torch.arange(nb, dtype=torch.int32)[None],
                        q_start=torch.tensor([0], dtype=torch.int32), q_len=torch.tensor([T], dtype=torch.int32),
                        ctx_len=torch.tensor([T], dtype=torch.int32), tiles=ops.prefill_tiles([T], 1))
        lg = model.forward_logits(torch.tensor(ids, dtype=torch.int32), meta, kv,
                                  torch.tensor([T - 1], dtype=torch.long))
        t = int(lg[0].argmax())
        out.append(t)
        ids.append(t)
    return out


def _prefix_blocks(eng):
    return sum(len(e.blocks) for e in eng.prefix.entries) if eng.prefix is not None else 0


def test_greedy_matches_full_recompute(model):
    prompts = [list(range(3, 3 + n)) for n in (5, 64, 65, 130)]
    sp = SamplingParams(max_tokens=8, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, None, num_blocks=64, max_model_len=512, max_batch=8, max_prefill_tokens=96)
    got = [r.output_ids for r in eng.generate(prompts, sp)]
    for p, g in zip(prompts, got):
        assert g == _greedy_reference(model, p, 8)
    assert eng.stats["finished"] == 4
    # every block returned (the prefix cache keeps its captured prefixes' blocks)
    assert eng.allocator.num_free() + _prefix_blocks(eng) == 64


def test_lookahead_equals_synchronous(model):
    prompts = [list(range(7, 7 + n)) for n in (3, 40, 100)]
    sp = SamplingParams(max_tokens=10, temperature=0.8, top_k=20, top_p=0.9, seed=11, ignore_eos=True)
    a = [r.output_ids for r in LLMEngine(model, None, num_blocks=64, max_model_len=512,
                                         lookahead=True).generate(prompts, sp)]
    b = [r.output_ids for r in LLMEngine(model, None, num_blocks=64, max_model_len=512,
                                         lookahead=False).generate(prompts, sp)]
    assert a == b


def test_graph_bucket_padding_path(model):
    """CPU executor emulates the padded graph steps: same tokens as eager steps."""
    prompts = [list(range(11, 11 + n)) for n in (9, 17, 33)]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    e1 = LLMEngine(model, None, num_blocks=64, max_model_len=512, max_batch=8)
    e1.use_graphs = True  # force the bucketed decode path through the CPU executor
    a = [r.output_ids for r in e1.generate(prompts, sp)]
    assert e1.stats["graph_steps"] > 0
    b = [r.output_ids for r in LLMEngine(model, None, num_blocks=64, max_model_len=512,
                                         max_batch=8).generate(prompts, sp)]
    assert a == b


def test_preemption_under_block_pressure(model):
    prompts = [list(range(5, 5 + 60)) for _ in range(6)]
    sp = SamplingParams(max_tokens=70, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, None, num_blocks=10, max_model_len=512, max_batch=8)
    reqs = eng.generate(prompts, sp)
    assert all(len(r.output_ids) == 70 for r in reqs)
    assert eng.stats["preemptions"] > 0
    ref = _greedy_reference(model, prompts[0], 70)
    assert all(r.output_ids == ref for r in reqs)


def test_stop_tokens_min_tokens_and_logprobs(model):
    eng = LLMEngine(model, None, num_blocks=32, max_model_len=512)
    base = eng.generate([[1, 2, 3, 4]], SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True))[0]
    stop_tok = base.output_ids[2]
    r = eng.generate([[1, 2, 3, 4]], SamplingParams(max_tokens=6, temperature=0.0, stop_token_ids=[stop_tok]))[0]
    assert r.finish_reason == "stop" and r.output_ids[-1] == stop_tok
    assert len(r.output_ids) == base.output_ids.index(stop_tok) + 1
    # min_tokens suppresses EOS
    eos = model.cfg.eos_token_ids[0]
    r = eng.generate([[1, 2, 3]], SamplingParams(max_tokens=5, min_tokens=5, temperature=0.0,
                                                 logit_bias={eos: 100.0}))[0]
    assert len(r.output_ids) == 5 and eos not in r.output_ids
    # logprobs: top alternatives come back with each token
    events = []
    req = eng.submit([1, 2, 3], SamplingParams(max_tokens=3, temperature=0.0, logprobs=3, ignore_eos=True),
                     callback=events.append)
    while not req.finished:
        eng.step()
    eng._flush()
    assert len(events) == 3 and all(len(e.top) == 3 for e in events)
    assert all(e.top[0][0] == e.token_id for e in events)
    assert all(abs(e.top[0][1] - e.logprob) < 1e-4 for e in events)


def test_presence_penalty_changes_output(model):
    eng = LLMEngine(model, None, num_blocks=32, max_model_len=512)
    plain = eng.generate([[9, 9, 9]], SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True))[0]
    pen = eng.generate([[9, 9, 9]], SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True,
                                                   presence_penalty=50.0))[0]
    assert len(set(pen.output_ids)) == len(pen.output_ids)  # a huge penalty forbids repeats
    assert len(set(plain.output_ids)) < len(plain.output_ids) or plain.output_ids != pen.output_ids


def test_prefill_tiles_np_matches_torch():
    for q, pre in (([5, 300, 64], [0, 10, 500]), ([1], [0]), ([129, 128, 127], [3, 0, 64])):
        for G in (1, 4):
            a = ops.prefill_tiles(q, G, pre).numpy()
            b = ops.prefill_tiles_np(q, G, pre)
            assert sorted(map(tuple, a.tolist())) == sorted(map(tuple, b.tolist()))
            # heaviest-first order by work = prefix + last row // G
            w = lambda t: pre[t[0]] + (min(t[1] + ops.PREFILL_ROWS, q[t[0]] * G) - 1) // G  # noqa: E731
            ws = [w(t) for t in b.tolist()]
            assert ws == sorted(ws, reverse=True)


def test_full_prefill_steps_are_256_aligned(model):
    """A step whose prefill budget is used up carries decode rows + prefill tokens in a
    multiple of 256 (the prefill GEMMs run whole 256-row tiles), and the outputs equal an
    engine with a small unaligned budget (chunking does not change greedy tokens)."""
    V = model.cfg.vocab_size
    prompts = [[3 + (7 * i + n) % (V - 3) for i in range(n)] for n in (300, 700, 650, 1500, 1800, 1700, 1200, 40, 510)]
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, None, num_blocks=256, max_model_len=2048, max_batch=16, max_prefill_tokens=4608)
    reqs = [eng.submit(p, sp) for p in prompts[:3]]
    for _ in range(3):       # some decode rows running before the large prompts arrive
        eng.step()
    reqs += [eng.submit(p, sp) for p in prompts[3:]]
    while not all(r.finished for r in reqs):
        eng.step()
    eng._flush()
    full = [t for t in eng.prefill_step_tokens if t > 4608 - 256]
    assert full and all(t % 256 == 0 for t in full), list(eng.prefill_step_tokens)
    ref = LLMEngine(model, None, num_blocks=256, max_model_len=2048, max_batch=16, max_prefill_tokens=333)
    assert [r.output_ids for r in reqs] == [r.output_ids for r in ref.generate(prompts, sp)]


def _shared_prefix_prompts(n=8, plen=70, seed=5):
    rng = np.random.default_rng(seed)
    head = rng.integers(3, 250, plen).tolist()
    return [head + rng.integers(3, 250, int(rng.integers(8, 60))).tolist() for _ in range(n)]


def test_prefix_cache_is_exact_and_hits(model):
    """Prompts sharing a 70-token template prefix: with the prefix cache the later prompts
    start their prefill after the cached prefix (KV block copies in the step arena) and
    the greedy outputs equal both the cache-off engine and the full-recompute reference."""
    prompts = _shared_prefix_prompts()
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    on = LLMEngine(model, None, num_blocks=96, max_model_len=512, max_batch=8, max_prefill_tokens=96,
                   prefix_cache=True)
    off = LLMEngine(model, None, num_blocks=96, max_model_len=512, max_batch=8, max_prefill_tokens=96,
                    prefix_cache=False)
    a = [r.output_ids for r in on.generate(prompts, sp)]
    b = [r.output_ids for r in off.generate(prompts, sp)]
    assert a == b
    assert a[0] == _greedy_reference(model, prompts[0], 6) and a[-1] == _greedy_reference(model, prompts[-1], 6)
    st = on.prefix.stats
    assert st["captures"] >= 1 and st["hits"] >= 3 and on.stats["prefix_hit_tokens"] >= 3 * 64
    # fewer tokens prefilled by exactly the reused ones
    assert off.stats["prefill_tokens"] - on.stats["prefill_tokens"] == on.stats["prefix_hit_tokens"]
    assert on.allocator.num_free() + _prefix_blocks(on) == 96 and off.allocator.num_free() == 96


def test_prefix_cache_sampled_and_preempted(model):
    """Seeded sampling and recompute-preemption under block pressure: the same tokens
    with and without the cache (a preempted request re-enters through the cache)."""
    prompts = _shared_prefix_prompts(n=10, plen=80, seed=9)
    sp = SamplingParams(max_tokens=24, temperature=0.9, top_k=30, seed=4, ignore_eos=True)
    kw = dict(num_blocks=24, max_model_len=512, max_batch=8, max_prefill_tokens=128)
    on = LLMEngine(model, None, prefix_cache=True, **kw)
    off = LLMEngine(model, None, prefix_cache=False, **kw)
    assert [r.output_ids for r in on.generate(prompts, sp)] == [r.output_ids for r in off.generate(prompts, sp)]
    assert on.prefix.stats["hits"] >= 1
    assert on.allocator.num_free() + _prefix_blocks(on) == 24


def test_prefix_cache_lru_bound(model):
    """Many distinct template prefixes: at most max_entries are kept (LRU), the rest are
    evicted and their blocks returned."""
    rng = np.random.default_rng(2)
    prompts = []
    for g in range(12):
        head = rng.integers(3, 250, 40).tolist()
        prompts += [head + rng.integers(3, 250, 10).tolist() for _ in range(2)]
    sp = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, None, num_blocks=128, max_model_len=512, max_batch=4, max_prefill_tokens=64,
                    prefix_cache=True)
    eng.prefix.max_entries = 3
    for i in range(0, len(prompts), 2):
        eng.generate(prompts[i:i + 2], sp)
    assert len(eng.prefix.entries) <= 3 and eng.prefix.stats["evictions"] >= 1
    assert eng.allocator.num_free() + _prefix_blocks(eng) == 128


def test_prefix_cache_shares_full_blocks(model):
    """A hit's block table starts with the entry's FULL prefix blocks (shared, never
    written: the prompt writes from the prefix end on); only the partial block is
    copied.  Refcounts keep a shared entry from eviction and return to 0 at release."""
    prompts = _shared_prefix_prompts(n=6, plen=150, seed=12)
    sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True)
    eng = LLMEngine(model, None, num_blocks=96, max_model_len=512, max_batch=8, max_prefill_tokens=128,
                    prefix_cache=True)
    reqs = [eng.submit(p, sp) for p in prompts]
    seen = []
    while not all(r.finished for r in reqs):
        eng.step()
        for r in reqs:
            if r.shared_blocks and r.request_id not in [x[0] for x in seen]:
                e = r._prefix_entry
                seen.append((r.request_id, r.shared_blocks, list(r.blocks[:r.shared_blocks]) == e.blocks[:2],
                             e.refs))
    eng._flush()
    assert seen and all(nb == 2 and same and refs >= 1 for _, nb, same, refs in seen)   # 150 // 64 = 2
    assert all(e.refs == 0 for e in eng.prefix.entries)
    assert eng.allocator.num_free() + _prefix_blocks(eng) == 96
    off = LLMEngine(model, None, num_blocks=96, max_model_len=512, max_batch=8, max_prefill_tokens=128,
                    prefix_cache=False)
    assert [r.output_ids for r in reqs] == [r.output_ids for r in off.generate(prompts, sp)]


def test_prefix_cache_yields_blocks_under_pool_pressure(model):
    """idle cached prefixes never hold blocks a sequence needs.  A pool of
    max_model_len / BLOCK + 1 blocks, mostly held by captured prefixes, then one long
    request that needs nearly the whole pool: the scheduler reclaims the idle entries
    (LRU) instead of truncating the prompt with 'length', skipping its decode rows or
    preempting, and the tokens equal a cache-off engine's."""
    from langstream_amd.engine.llm_engine import BLOCK
    rng = np.random.default_rng(21)
    max_len = 8 * BLOCK
    nb = max_len // BLOCK + 1
    kw = dict(num_blocks=nb, max_model_len=max_len, max_batch=4, max_prefill_tokens=128)
    eng = LLMEngine(model, None, prefix_cache=True, **kw)
    sp2 = SamplingParams(max_tokens=2, temperature=0.0, ignore_eos=True)
    for _ in range(3):
        head = rng.integers(3, 250, 100).tolist()
        eng.generate([head + rng.integers(3, 250, 8).tolist() for _ in range(2)], sp2)
    held = _prefix_blocks(eng)
    assert held >= 4 and eng.allocator.num_free() + held == nb
    long_prompt = rng.integers(3, 250, 5 * BLOCK - 10).tolist()
    sp = SamplingParams(max_tokens=max_len - len(long_prompt) - 1, temperature=0.0, ignore_eos=True)
    r = eng.generate([long_prompt], sp)[0]
    off = LLMEngine(model, None, prefix_cache=False, **kw).generate([long_prompt], sp)[0]
    assert len(r.output_ids) == sp.max_tokens and r.output_ids == off.output_ids
    assert eng.prefix.stats.get("reclaimed_blocks", 0) >= 1 and eng.stats["preemptions"] == 0
    assert eng.allocator.num_free() + _prefix_blocks(eng) == nb


def test_prefix_capture_leaves_decode_headroom(model):
    """collect_captures(headroom=n_decode): a capture never takes the blocks the step's
    decoding sequences may need."""
    from langstream_amd.engine.prefix_cache import PrefixCache

    class Alloc:
        def __init__(self, n):
            self.free_ = list(range(n))

        def num_free(self):
            return len(self.free_)

        def can_allocate(self, n):
            return n <= len(self.free_)

        def allocate(self, n):
            out, self.free_ = self.free_[:n], self.free_[n:]
            return out

        def free(self, bl):
            self.free_ += list(bl)

    class R:
        def __init__(self, ids):
            self.prompt_ids, self.num_computed, self.finished = ids, len(ids), False
            self.blocks = [100, 101]

    a = Alloc(3)
    pc = PrefixCache(a, 64, min_len=32)
    head = list(range(3, 103))
    pc.observe(R(head + [1]))
    r2 = R(head + [2])
    pc.observe(r2)
    assert pc.pending
    pc.collect_captures(step=1, headroom=2)   # 3 free - 2 headroom < 2 blocks: no capture
    assert not pc.entries
    pc.collect_captures(step=1, headroom=1)
    assert len(pc.entries) == 1 and a.num_free() == 1
    assert pc.reclaimable(step=1) == 0          # captured this step: its copy reads it
    assert pc.reclaim(3, step=2) == 2 and a.num_free() == 3 and not pc.entries
