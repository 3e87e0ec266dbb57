"""Chunked vs whole prefill on llama-small: greedy tokens and logprobs per step
(GPU debugging aid for tests/test_engine_gpu.py::test_llama_chunked_prefill_consistent)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from langstream_amd.engine.llm_engine import LLMEngine, SamplingParams  # noqa: E402
from langstream_amd.models.llama import LlamaModel, PRESETS  # noqa: E402

model = LlamaModel(PRESETS["llama-small"], device="cuda")
prompt = list(range(10, 10 + 300))
for lp in (0, 5):
    for chunk in (4096, 100):
        sp = SamplingParams(max_tokens=4, temperature=0.0, ignore_eos=True, logprobs=lp)
        eng = LLMEngine(model, None, num_blocks=64, max_model_len=1024, max_prefill_tokens=chunk)
        r = eng.generate([prompt], sp)[0]
        print(json.dumps({"logprobs": lp, "chunk": chunk, "tokens": r.output_ids,
                          "lps": [round(x, 4) for x in r.output_logprobs]}), flush=True)
