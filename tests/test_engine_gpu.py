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


def test_llama_prefill_logits_match_cpu():
    cfg = PRESETS["llama-small"]
    gpu = LlamaModel(cfg, device="cuda")
    cpu = _cpu_copy(gpu)
    prompts = [list(range(5, 5 + n)) for n in (7, 70, 130)]
    e_g = LLMEngine(gpu, None, num_blocks=64, max_model_len=1024, use_graphs=False)
    e_c = LLMEngine(cpu, None, num_blocks=64, max_model_len=1024)
    logits = []
    for e in (e_g, e_c):
        reqs = [e.submit(p, SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)) for p in prompts]
        e._drain_inbox()
        batch = e._schedule_prefill()
        captured = {}
        orig = e._sample_and_emit
        e._sample_and_emit = lambda lg, rs, c=captured, o=orig: (c.setdefault("lg", lg.clone()), o(lg, rs))
        e._run_prefill(batch)
        logits.append(captured["lg"])
    assert _cos(logits[0], logits[1]) > 0.995


def test_llama_graph_decode_matches_eager():
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    prompts = [list(range(3, 3 + n)) for n in (5, 33, 64, 65, 200)]
    sp = SamplingParams(max_tokens=12, temperature=0.0, ignore_eos=True)
    e1 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, use_graphs=True, max_batch=8)
    out1 = [r.output_ids for r in e1.generate(prompts, sp)]
    e2 = LLMEngine(model, None, num_blocks=128, max_model_len=1024, use_graphs=False, max_batch=8)
    out2 = [r.output_ids for r in e2.generate(prompts, sp)]
    # greedy decode with bf16: allow a late divergence on near-ties, first tokens must agree
    for a, b in zip(out1, out2):
        assert a[:4] == b[:4]


def test_llama_chunked_prefill_consistent():
    cfg = PRESETS["llama-small"]
    model = LlamaModel(cfg, device="cuda")
    prompt = list(range(10, 10 + 300))
    sp = SamplingParams(max_tokens=6, temperature=0.0, ignore_eos=True)
    a = LLMEngine(model, None, num_blocks=64, max_model_len=1024, max_prefill_tokens=4096).generate([prompt], sp)[0]
    b = LLMEngine(model, None, num_blocks=64, max_model_len=1024, max_prefill_tokens=100).generate([prompt], sp)[0]
    assert a.output_ids[:3] == b.output_ids[:3]


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
