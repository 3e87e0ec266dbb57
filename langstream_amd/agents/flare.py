"""flare-controller (AIA/ai/langstream/ai/agents/flare/FlareControllerAgent.java:65-219).

Reads the text-completion tokens / logprobs; finds low-confidence spans
(exp(logprob) < min-prob (0.2), spans merged when closer than min-token-gap (5),
padded by num-pad-tokens (2)).  With spans: the record (plus the spans in
``retrieve-documents-field``) goes to ``loop-topic`` and nothing is emitted downstream;
without: the record passes through.  ``max-iterations`` (10) is read from
``num-iterations-field`` (value.flare_iterations).

Deliberate fixes of reference bugs (documented, behaviour otherwise identical):
``retrieve-documents-field`` is read from its own key (the reference reads
``loop-topic``: FlareControllerAgent.java:73-75), a token counts as a word when it
CONTAINS a word character (the reference's ``matches("\\w")`` requires a 1-char token),
span ends are clamped to the token count (the reference can overrun), and every pass
through the loop increments ``num-iterations-field`` (the reference reads the counter but
never writes it, so ``max-iterations`` could not stop a record whose answer keeps a
low-confidence span: with the word-token fix above, FlareControllerAgentRunnerIT's stubbed
completion is such an answer and now loops ``max-iterations`` + 1 times, then passes).
"""
from __future__ import annotations

import math
import re
from typing import Any, Dict, List

from ..api.agent import AgentProcessor
from ..api.record import SourceRecordAndResult
from ..runtime.registry import register_agent
from .genai.el import eval_expression
from .genai.mutable import MutableRecord

_WORD = re.compile(r"\w")


def low_confidence_spans(tokens: List[str], logprobs: List[float], min_prob: float, min_token_gap: int,
                         num_pad: int) -> List[str]:
    low = [i for i, lp in enumerate(logprobs)
           if lp is not None and math.exp(lp) < min_prob and i < len(tokens) and _WORD.search(tokens[i] or "")]
    if not low:
        return []
    spans = [[low[0], low[0] + num_pad + 1]]
    for prev, idx in zip(low, low[1:]):
        end = idx + num_pad + 1
        if idx - prev < min_token_gap:
            spans[-1][1] = end
        else:
            spans.append([idx, end])
    out = []
    for a, b in spans:
        s = "".join(tokens[a: min(b, len(tokens))])
        if s:
            out.append(s)
    return out


@register_agent("flare-controller")
class FlareControllerAgent(AgentProcessor):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.tokens_field = configuration.get("tokens-field", "")
        self.logprobs_field = configuration.get("logprobs-field", "")
        self.loop_topic = configuration.get("loop-topic", "")
        self.retrieve_field = configuration.get("retrieve-documents-field", "value.retrieve-documents")
        self.min_prob = float(configuration.get("min-prob", 0.2))
        self.min_gap = int(configuration.get("min-token-gap", 5))
        self.num_pad = int(configuration.get("num-pad-tokens", 2))
        self.max_iter = int(configuration.get("max-iterations", 10))
        self.iter_field = configuration.get("num-iterations-field", "value.flare_iterations")
        self.producer = None

    def start(self) -> None:
        prov = self.context.topic_connection_provider
        self.producer = prov.create_producer(self.context.global_agent_id, self.loop_topic)
        self.producer.start()

    def close(self) -> None:
        if self.producer is not None:
            self.producer.close()

    def process(self, records, sink) -> None:
        for r in records:
            try:
                mr = MutableRecord.from_record(r).copy()
                ctx = mr.el_context()
                it = eval_expression(self.iter_field, ctx) or 0
                if int(it) > self.max_iter:
                    sink(SourceRecordAndResult(r, [r], None))
                    continue
                tokens = eval_expression(self.tokens_field, ctx) or []
                lps = eval_expression(self.logprobs_field, ctx) or []
                spans = low_confidence_spans(list(tokens), [float(x) for x in lps], self.min_prob, self.min_gap,
                                             self.num_pad)
                if not spans:
                    sink(SourceRecordAndResult(r, [r], None))
                    continue
                mr.set_result_field(spans, self.retrieve_field)
                mr.set_result_field(int(it) + 1, self.iter_field)
                f = self.producer.write(mr.to_record())
                f.add_done_callback(lambda ff, r=r: sink(
                    SourceRecordAndResult(r, None, ff.exception()) if ff.exception() else
                    SourceRecordAndResult(r, [], None)))
            except Exception as e:  # noqa: BLE001
                sink(SourceRecordAndResult(r, None, e))
