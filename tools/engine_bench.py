"""Microbenchmarks of the GPU engines (not the driver's bench.py): Llama decode/prefill
throughput, BERT embedding throughput, kNN latency.  Prints one JSON line per test."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams  # noqa: E402
from langstream_amd.models.llama import LlamaModel, PRESETS  # noqa: E402


def sync():
    torch.cuda.synchronize()


def bench_llm(args):
    cfg = PRESETS[args.model]
    t0 = time.time()
    model = LlamaModel(cfg, device="cuda")
    sync()
    print(json.dumps({"event": "model_init", "s": round(time.time() - t0, 2)}), flush=True)
    eng = LLMEngine(model, None, max_model_len=args.max_len, max_batch=args.batch, max_prefill_tokens=args.prefill_chunk)
    t0 = time.time()
    eng.capture_graphs([b for b in eng.buckets if b <= args.batch])
    sync()
    print(json.dumps({"event": "graphs", "s": round(time.time() - t0, 2), "blocks": eng.num_blocks}), flush=True)
    sp = SamplingParams(max_tokens=args.gen, temperature=0.8, top_p=0.95, ignore_eos=True)
    prompts = [[(i * 31 + j) % 1000 + 100 for j in range(args.prompt)] for i in range(args.batch)]
    # warmup
    eng.generate(prompts[:4], SamplingParams(max_tokens=4, ignore_eos=True))
    sync()
    t0 = time.time()
    reqs = [eng.submit(p, sp) for p in prompts]
    eng._drain_inbox()
    # prefill phase
    while eng.waiting:
        eng.step()
    sync()
    t1 = time.time()
    while eng.running:
        eng.step()
    sync()
    t2 = time.time()
    ntok = sum(len(r.output_ids) for r in reqs)
    print(json.dumps({
        "test": "llm", "model": args.model, "batch": args.batch, "prompt": args.prompt, "gen": args.gen,
        "prefill_s": round(t1 - t0, 4), "prefill_tok_s": round(args.batch * args.prompt / (t1 - t0), 1),
        "decode_s": round(t2 - t1, 4), "decode_tok_s": round((ntok - args.batch) / (t2 - t1), 1),
        "ms_per_decode_step": round(1000 * (t2 - t1) / max(1, args.gen - 1), 3),
        "stats": eng.stats}), flush=True)


def bench_embed(args):
    from langstream_amd.engine.embedder import EmbeddingEngine
    from langstream_amd.models.bert import BertEncoder, PRESETS as BP
    from langstream_amd.tokenizers import WordPieceTokenizer, builtin_corpus
    enc = BertEncoder(BP["bge-small-en"], device="cuda")
    tok = WordPieceTokenizer.synthetic()
    eng = EmbeddingEngine(enc, tok)
    corpus = builtin_corpus()
    texts = [" ".join(corpus[i: i + 6]) for i in range(args.texts)]
    eng.embed(texts[:64])
    sync()
    t0 = time.time()
    for _ in range(args.iters):
        eng.embed(texts)
    sync()
    dt = (time.time() - t0) / args.iters
    ntok = sum(len(t) for t in tok.encode_batch(texts))
    # device-resident output (what the vector store consumes): no host list conversion
    eng.embed_tensor(texts[:64])
    sync()
    t0 = time.time()
    for _ in range(args.iters):
        for i in range(0, len(texts), 512):
            eng.embed_tensor(texts[i: i + 512])
    sync()
    dt_t = (time.time() - t0) / args.iters
    # encoder forward only (pre-tokenised, packed on the device)
    toks = tok.encode_batch(texts[:512])
    packed = [t.cuda() for t in enc.pack(toks)]
    enc.forward_packed(*packed)
    sync()
    t0 = time.time()
    for _ in range(args.iters * 4):
        enc.forward_packed(*packed)
    sync()
    dt_f = (time.time() - t0) / (args.iters * 4)
    print(json.dumps({"test": "embed", "fused": enc.fused_supported(), "texts": len(texts),
                      "avg_tokens": ntok / len(texts), "texts_per_s": round(len(texts) / dt, 1),
                      "tokens_per_s": round(ntok / dt, 1), "texts_per_s_device_out": round(len(texts) / dt_t, 1),
                      "encoder_forward_512_texts_ms": round(dt_f * 1000, 3),
                      "encoder_texts_per_s": round(512 / dt_f, 1)}), flush=True)


def bench_knn(args):
    from langstream_amd import ops
    X = torch.nn.functional.normalize(torch.randn(args.rows, 384, device="cuda"), dim=-1).bfloat16()
    for nq in str(args.queries).split(","):
        Q = torch.nn.functional.normalize(torch.randn(int(nq), 384, device="cuda"), dim=-1).bfloat16()
        for _ in range(3):
            ops.knn_topk(X, Q, 20, _ablate=args.knn_ablate)
        sync()
        t0 = time.time()
        for _ in range(20):
            ops.knn_topk(X, Q, 20, _ablate=args.knn_ablate)
        sync()
        dt = (time.time() - t0) / 20
        print(json.dumps({"test": "knn", "rows": args.rows, "queries": int(nq), "ms": round(dt * 1000, 3),
                          "GB_per_s": round(args.rows * 384 * 2 / dt / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="llm,embed,knn")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--prompt", type=int, default=512)
    ap.add_argument("--gen", type=int, default=128)
    ap.add_argument("--max-len", type=int, default=4096)
    ap.add_argument("--prefill-chunk", type=int, default=16384)
    ap.add_argument("--texts", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--queries", default="64", help="comma-separated query counts (knn)")
    ap.add_argument("--knn-ablate", type=int, default=0,
                    help="kNN main-pass timing ablation 1-3 (diagnosis only: WRONG results)")
    a = ap.parse_args()
    for w in a.what.split(","):
        {"llm": bench_llm, "embed": bench_embed, "knn": bench_knn}[w](a)
