"""GenAI toolkit agent (runtime type ``ai-tools``).

Parity: AIA/ai/langstream/ai/agents/GenAIToolKitAgent.java:53-233 -- one TransformStep
per agent built from ``steps[0]``; ``process()`` runs the step asynchronously for each
record and emits results as they complete (possibly out of order; the runner's
SourceRecordTracker keeps commits ordered).  Services (GPU engines, datasources) come
from the process-wide ServiceRegistry in the agent context.
"""
from __future__ import annotations

import logging
from concurrent.futures import Future
from typing import Any, Dict, List

from ...api.agent import AgentProcessor
from ...api.record import SimpleRecord, SourceRecordAndResult
from ...runtime.registry import register_agent
from . import steps as S
from .mutable import MutableRecord

log = logging.getLogger(__name__)


class _TopicStreamConsumer:
    """Writes streamed answer chunks to a topic (StreamingAnswersConsumer)."""

    def __init__(self, producer):
        self.producer = producer
        self.producer.start()

    def stream_answer_chunk(self, index: int, content: str, last: bool, rec: MutableRecord) -> None:
        r = rec.to_record()
        if r is not None:
            self.producer.write(r)

    def close(self) -> None:
        self.producer.close()


from ...core.catalog import GENAI_STEPS  # noqa: E402


@register_agent("ai-tools", *GENAI_STEPS)
class GenAIToolKitAgent(AgentProcessor):
    def __init__(self):
        super().__init__()
        self.config: Dict[str, Any] = {}
        self.step = None

    def init(self, configuration: Dict[str, Any]) -> None:
        self.config = dict(configuration)
        steps = self.config.get("steps")
        if not steps:
            # direct (un-planned) usage: the configuration is the step itself
            steps = [dict(self.config)]
        if len(steps) != 1:
            raise ValueError("ai-tools agents run exactly one step")
        self.step_cfg = dict(steps[0])
        if not self.step_cfg.get("type") and self._agent_type in GENAI_STEPS:
            self.step_cfg["type"] = self._agent_type

    def _services(self):
        svc = getattr(self.context, "services", None) if self.context is not None else None
        if svc is None:
            from ...services import ServiceRegistry
            svc = ServiceRegistry.default()
        return svc

    def _stream_factory(self, topic: str):
        prov = self.context.topic_connection_provider if self.context is not None else None
        if prov is None:
            raise ValueError("stream-to-topic requires a streaming cluster")
        return _TopicStreamConsumer(prov.create_producer(self.agent_id(), topic))

    def _build_step(self):
        cfg = self.step_cfg
        t = cfg.get("type")
        if t == "drop-fields":
            return S.DropFieldsStep(cfg)
        if t == "merge-key-value":
            return S.MergeKeyValueStep(cfg)
        if t == "unwrap-key-value":
            return S.UnwrapKeyValueStep(cfg)
        if t == "cast":
            return S.CastStep(cfg)
        if t == "flatten":
            return S.FlattenStep(cfg)
        if t == "drop":
            return S.DropStep(cfg)
        if t == "compute":
            return S.ComputeStep(cfg)
        if t == "compute-ai-embeddings":
            return S.ComputeAIEmbeddingsStep(cfg, self._services().embeddings_service(self.config,
                                                                                     cfg.get("model")))
        if t == "query":
            from ..vector.datasources import datasource_for
            return S.QueryStep(cfg, datasource_for(self.config.get("datasource") or cfg.get("datasource")))
        if t == "ai-chat-completions":
            return S.ChatCompletionsStep(cfg, self._services().completions_service(self.config, cfg.get("model")),
                                         self._stream_factory)
        if t == "ai-text-completions":
            return S.TextCompletionsStep(cfg, self._services().completions_service(self.config, cfg.get("model")),
                                         self._stream_factory)
        raise ValueError(f"Unknown step type {t}")

    def start(self) -> None:
        self.step = self._build_step()
        self.step.start()

    def close(self) -> None:
        if self.step is not None:
            self.step.close()

    def process(self, records, sink) -> None:
        if self.step is None:
            self.start()
        many = getattr(sink, "many", None)
        bulk = getattr(self.step, "process_bulk", None)
        if many is not None and bulk is not None and self.step.bulk_ok():
            self._process_bulk(records, many, bulk)
            return
        for r in records:
            self._process_one(r, sink)

    def _process_bulk(self, records, many, bulk) -> None:
        """The runner takes results in batches (``sink.many``) and the step completes
        records in batches (compute-ai-embeddings): one result batch per completed
        embedding batch instead of a future and a callback chain per record."""
        now, pend = [], []
        for r in records:
            try:
                mr = MutableRecord.from_record(r)
                if not self.step.applies(mr):
                    now.append(SourceRecordAndResult(r, [r], None))
                    continue
                pend.append((r, mr))
            except Exception as e:  # noqa: BLE001
                now.append(SourceRecordAndResult(r, None, e))
        if now:
            self.processed(len(now), sum(1 for x in now if x.error is None))
            many(now)
        if pend:
            bulk(pend, lambda done: self._emit_bulk(done, many))

    def _emit_bulk(self, done, many) -> None:
        out = []
        n_out = 0
        for r, mr, err in done:
            if err is not None:
                out.append(SourceRecordAndResult(r, None, err))
                continue
            try:
                rec = mr.to_record()
            except Exception as e:  # noqa: BLE001
                out.append(SourceRecordAndResult(r, None, e))
                continue
            if rec is not None:
                n_out += 1
            out.append(SourceRecordAndResult(r, [rec] if rec is not None else [], None))
        self.processed(len(done), n_out)
        many(out)

    def _process_one(self, r, sink) -> None:
        try:
            mr = MutableRecord.from_record(r)
            if not self.step.applies(mr):
                self.processed(1, 1)
                sink(SourceRecordAndResult(r, [r], None))
                return
            if not self.step.is_async:
                self.step.process(mr)
                out = mr.to_record()
                self.processed(1, 1 if out is not None else 0)
                sink(SourceRecordAndResult(r, [out] if out is not None else [], None))
                return
            fut = self.step.process_async(mr)
        except Exception as e:  # noqa: BLE001
            sink(SourceRecordAndResult(r, None, e))
            return

        def done(f: Future) -> None:
            err = f.exception()
            if err is not None:
                sink(SourceRecordAndResult(r, None, err))
                return
            out = mr.to_record()
            self.processed(1, 1 if out is not None else 0)
            sink(SourceRecordAndResult(r, [out] if out is not None else [], None))

        fut.add_done_callback(done)

    def build_additional_info(self) -> Dict[str, Any]:
        return {"step": self.step_cfg.get("type")}

    def get_agent_status(self):
        # the reference reports a toolkit agent under its declared type ("drop-fields",
        # "compute", ...: the NAR index maps every step type to GenAIToolKitAgent), not
        # the shared runtime type (GenIAgentsRunnerIT.testRunAIToolsComposite)
        st = super().get_agent_status()
        step = self.step_cfg.get("type") if getattr(self, "step_cfg", None) else None
        if step:
            for s in st:
                s.agent_type = step
        return st
