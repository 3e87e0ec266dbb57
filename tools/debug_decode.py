"""Decode-step distributions vs prefill-only distributions of the same context (GPU).

For greedy generation from a 300-token prompt (whole and 100-token chunked prefill),
step k's top-5 (token, logprob) from the decode path is compared with a fresh prefill
of prompt + the first k generated tokens, and with the fp32 CPU model."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams  # noqa: E402
from langstream_amd.models.llama import LlamaModel, PRESETS  # noqa: E402


def tops(model, prompt, n_steps, chunk):
    events = []
    e = LLMEngine(model, None, num_blocks=64, max_model_len=1024, max_prefill_tokens=chunk)
    e.generate([prompt], SamplingParams(max_tokens=n_steps, temperature=0.0, ignore_eos=True, logprobs=5),
               callback=lambda ev: events.append(ev)) if hasattr(e, "generate_cb") else None
    r = e.submit(prompt, SamplingParams(max_tokens=n_steps, temperature=0.0, ignore_eos=True, logprobs=5),
                 callback=lambda ev: events.append(ev))
    while not r.finished:
        e.step()
    e._flush()
    return [(ev.token_id, [(t, round(lp, 3)) for t, lp in ev.top]) for ev in events]


cfg = PRESETS["llama-small"]
gpu = LlamaModel(cfg, device="cuda")
gpu.lm_head.mul_(30.0)
cpu = LlamaModel(cfg, device="cpu", dtype=torch.float32)
cpu.load_state_dict({k: v.float().cpu() for k, v in gpu.state_dict().items()})
prompt = list(range(10, 10 + 300))
for chunk in (4096, 100):
    dec = tops(gpu, prompt, 4, chunk)
    print(json.dumps({"chunk": chunk, "decode": dec}), flush=True)
    toks = [t for t, _ in dec]
    for k in range(1, 4):
        pf = tops(gpu, prompt + toks[:k], 1, 4096)[0]
        ref = tops(cpu, prompt + toks[:k], 1, 4096)[0]
        print(json.dumps({"chunk": chunk, "step": k, "decode_top": dec[k][1], "gpu_prefill_top": pf[1],
                          "cpu_fp32_top": ref[1]}), flush=True)
