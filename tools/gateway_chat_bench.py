"""End-to-end chat latency through the WebSocket gateway (BASELINE config "ai-chat-completions
agent, Llama-3-8B TP=1 bf16 on 1 MI355X, gateway chat").

Starts a chat application (chat gateway -> questions topic -> ai-chat-completions on the
in-process GPU engine, answers streamed back to the answers topic) plus the gateway server,
then C concurrent WebSocket sessions each ask Q questions in turn.  Per answer it records the
time to the first streamed chunk (TTFT) and to the last one, and reports p50 TTFT,
per-session decode tokens/s and the aggregate.  Weights are random-init (no checkpoints
offline), so generation runs to max-tokens (ignore-eos).

usage (GPU box): python tools/gateway_chat_bench.py [--sessions 1,4,16] [--questions 4] [--max-tokens 128]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PIPE = """
topics:
  - name: "questions"
    creation-mode: create-if-not-exists
  - name: "answers"
    creation-mode: create-if-not-exists
  - name: "log"
    creation-mode: create-if-not-exists
pipeline:
  - name: "chat"
    type: "ai-chat-completions"
    input: "questions"
    output: "log"
    configuration:
      model: "{model}"
      completion-field: "value"
      stream-to-topic: "answers"
      stream-response-completion-field: "value"
      min-chunks-per-message: {chunks}
      max-tokens: {max_tokens}
      ignore-eos: true
      messages:
        - role: user
          content: "{{{{ value }}}}"
"""

GATEWAYS = """
gateways:
  - id: chat
    type: chat
    parameters: [sessionId]
    chat-options:
      questions-topic: questions
      answers-topic: answers
      headers:
        - key: langstream-client-session-id
          value-from-parameters: sessionId
"""

CONFIG = """
configuration:
  resources:
    - type: "local-gpu-configuration"
      name: "local"
      configuration:
        chat-model: "{model}"
        max-batch: 256
        max-model-len: 4096
"""


async def session(base: str, sid: str, questions: int, out: list):
    import aiohttp
    async with aiohttp.ClientSession() as s:
        ws = await s.ws_connect(f"{base}/v1/chat/default/chatbench/chat?param:sessionId={sid}")
        await asyncio.sleep(0.2)
        for q in range(questions):
            t0 = time.perf_counter()
            await ws.send_str(json.dumps({"value": f"question {q} from {sid}: tell me about streaming pipelines"}))
            first = last = None
            chunks = 0
            while True:
                msg = await ws.receive(timeout=float(os.environ.get("CHAT_BENCH_TIMEOUT", "300")))
                if os.environ.get("CHAT_BENCH_DEBUG"):
                    print("recv", str(msg.data)[:200], flush=True)
                data = json.loads(msg.data)
                if "status" in data and "record" not in data:
                    continue   # produce ack
                rec = data.get("record") or {}
                chunks += 1
                now = time.perf_counter()
                if first is None:
                    first = now
                if str((rec.get("headers") or {}).get("stream-last-message")) == "true":
                    last = now
                    break
            out.append({"ttft": first - t0, "total": last - t0, "chunks": chunks})
        await ws.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", default="1,4,16")
    ap.add_argument("--questions", type=int, default=4)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--chunks", type=int, default=1, help="min-chunks-per-message")
    ap.add_argument("--model", default="llama-3-8b")
    args = ap.parse_args()
    import torch
    from langstream_amd.core.store import InMemoryApplicationStore, StoredApplication
    from langstream_amd.gateway.server import GatewayServer, GatewayService
    from langstream_amd.runtime.local import LocalApplicationRunner
    from langstream_amd.services import ServiceRegistry

    model = args.model if torch.cuda.is_available() else "llama-tiny"
    fmt = dict(model=model, max_tokens=args.max_tokens, chunks=args.chunks)
    files = {"pipeline.yaml": PIPE.format(**fmt), "gateways.yaml": GATEWAYS,
             "configuration.yaml": CONFIG.format(**fmt)}
    services = ServiceRegistry({"device": "cuda:0" if torch.cuda.is_available() else "cpu"})
    ServiceRegistry.set_default(services)
    engine = services.llm_engine(model, {"chat-model": model, "max-batch": 256, "max-model-len": 4096})   # load + graphs
    runner = LocalApplicationRunner.from_yaml(files, application_id="chatbench", services=services).start()
    store = InMemoryApplicationStore()
    store.put(StoredApplication("chatbench", "default", runner.application, files))
    gw = GatewayServer(GatewayService(store), port=0).start()
    base = gw.url.replace("http", "ws")
    try:
        loop = asyncio.new_event_loop()

        async def many(n, prefix, q, out):
            await asyncio.gather(*[session(base, f"{prefix}{i}", q, out) for i in range(n)])

        loop.run_until_complete(many(2, "warm", 1, []))
        for c in [int(v) for v in args.sessions.split(",")]:
            res: list = []
            engine.ttft_s.clear()
            t0 = time.perf_counter()
            loop.run_until_complete(many(c, f"s{c}-", args.questions, res))
            wall = time.perf_counter() - t0
            ttft = [r["ttft"] for r in res]
            decode = [(args.max_tokens - 1) / max(r["total"] - r["ttft"], 1e-9) for r in res]
            print(json.dumps({"sessions": c, "answers": len(res), "max_tokens": args.max_tokens, "model": model,
                              "ttft_p50_ms": round(1e3 * statistics.median(ttft), 1),
                              "ttft_max_ms": round(1e3 * max(ttft), 1),
                              "engine_ttft_p50_ms": round(1e3 * statistics.median(engine.ttft_s), 1)
                              if engine.ttft_s else None,
                              "answer_p50_s": round(statistics.median(r["total"] for r in res), 3),
                              "per_session_decode_tok_s": round(statistics.median(decode), 1),
                              "aggregate_tok_s": round(len(res) * args.max_tokens / wall, 1)}), flush=True)
    finally:
        gw.stop()
        runner.stop(10)
        services.shutdown()


if __name__ == "__main__":
    sys.exit(main())
