"""BASELINE configs 3 and 5: ai-chat-completions through the WebSocket chat gateway.

Config 3 = Llama-3-8B TP=1 on one MI355X (``bench.py --config chat``); config 5 =
Llama-3-70B TP=8 over xGMI (``bench.py --config chat --chat-model llama-3-70b --gpus 8 --tp
8``).  The chat application is the reference's chat-gateway shape
(GW/websocket/handlers/ChatHandler.java:29-190: chat gateway -> questions topic ->
ai-chat-completions streaming chunks to the answers topic, ChatCompletionsStep.java:
132-155): C concurrent WebSocket sessions ask Q questions each; per answer the client
records the time to the first streamed chunk (TTFT) and to the last one.

Tensor parallelism: the job is one TP group (torch.distributed over RCCL); rank 0 runs
the application, the gateway and the engine scheduler, ranks > 0 mirror every engine
step in the native worker loop (StepExecutor::worker_loop) until rank 0 stops.
Weights are random-init (no checkpoints offline): generation always runs to max-tokens.
"""
from __future__ import annotations

import asyncio
import json
import os
import statistics
import time

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
        max-batch: {max_batch}
        max-model-len: 4096
"""

METRIC = "chat tokens/s (whole job) + p50 TTFT through the websocket chat gateway"


async def _session(base: str, sid: str, questions: int, out: list, timeout: float):
    import aiohttp
    async with aiohttp.ClientSession() as s:
        ws = await s.ws_connect(f"{base}/v1/chat/default/chatbench/chat?param:sessionId={sid}")
        for q in range(questions):
            t0 = time.perf_counter()
            await ws.send_str(json.dumps({"value": f"question {q} from {sid}: tell me about streaming pipelines"}))
            first = last = None
            chunks = 0
            while True:
                msg = await ws.receive(timeout=timeout)
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


def run(args, rank: int, world: int, barrier) -> None:
    import torch
    from ..services import ServiceRegistry
    use_gpu = torch.cuda.is_available()
    tp = max(1, int(args.tp or world))
    if tp != world:
        raise SystemExit(f"--config chat: --tp {tp} must equal the number of ranks ({world}); one TP group per job")
    model = args.chat_model if use_gpu else "llama-tiny"
    services = ServiceRegistry({"device": f"cuda:{int(os.environ.get('LOCAL_RANK', '0') or 0)}" if use_gpu else "cpu"})
    ServiceRegistry.set_default(services)
    if world > 1:
        from ..parallel import init_tensor_parallel
        services.tp = init_tensor_parallel(world)
    sessions = max(1, args.batch if args.batch != 256 else 64)
    max_batch = max(sessions, 8)
    ecfg = {"chat-model": model, "max-batch": max_batch, "max-model-len": 4096}
    t_setup = time.time()
    engine = services.llm_engine(model, ecfg)   # weights + KV pool + graphs (every rank, lock-step)
    if rank != 0:
        engine.worker_loop()                    # until rank 0 stops the engine
        services.shutdown()
        return
    from ..core.store import InMemoryApplicationStore, StoredApplication
    from ..gateway.server import GatewayServer, GatewayService
    from ..runtime.local import LocalApplicationRunner
    fmt = dict(model=model, max_tokens=args.max_tokens, chunks=1, max_batch=max_batch)
    files = {"pipeline.yaml": PIPE.format(**fmt), "gateways.yaml": GATEWAYS, "configuration.yaml": CONFIG.format(**fmt)}
    runner = LocalApplicationRunner.from_yaml(files, application_id="chatbench", services=services).start()
    store = InMemoryApplicationStore()
    store.put(StoredApplication("chatbench", "default", runner.application, files))
    gw = GatewayServer(GatewayService(store), port=0).start()
    base = gw.url.replace("http", "ws")
    setup_s = time.time() - t_setup
    timeout = float(os.environ.get("CHAT_BENCH_TIMEOUT", "600"))
    try:
        loop = asyncio.new_event_loop()

        async def many(n, prefix, q, out):
            await asyncio.gather(*[_session(base, f"{prefix}{i}", q, out, timeout) for i in range(n)])

        for w in range(args.warmup):
            loop.run_until_complete(many(min(sessions, 4), f"warm{w}-", 1, []))
        engine.ttft_s.clear()
        res: list = []
        if use_gpu:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        loop.run_until_complete(many(sessions, "s", args.steps, res))
        if use_gpu:
            torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ttft = [r["ttft"] for r in res]
        decode = [(args.max_tokens - 1) / max(r["total"] - r["ttft"], 1e-9) for r in res]
        toks = len(res) * args.max_tokens
        print(json.dumps({
            "metric": METRIC, "value": round(toks / wall, 1), "unit": "tokens/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * wall / args.steps, 2),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "bf16" if use_gpu else "fp32", "data": "synthetic questions, random-init weights",
            "config": {"model": model, "tp": tp, "sessions": sessions, "questions_per_session": args.steps,
                       "max_new_tokens": args.max_tokens, "gateway": "websocket /v1/chat",
                       "parallelism": f"tp{tp}"},
            "ttft_p50_ms": round(1e3 * statistics.median(ttft), 1), "ttft_max_ms": round(1e3 * max(ttft), 1),
            "engine_ttft_p50_ms": round(1e3 * statistics.median(engine.ttft_s), 1) if engine.ttft_s else None,
            "answer_p50_s": round(statistics.median(r["total"] for r in res), 3),
            "per_session_decode_tok_s": round(statistics.median(decode), 1),
            "answers": len(res), "setup_s": round(setup_s, 1)}), flush=True)
    finally:
        gw.stop()
        runner.stop(10)
        services.shutdown()   # stops the engine: TP workers leave their loop
