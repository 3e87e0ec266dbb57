"""CompositeAgentProcessor (RT/agent/CompositeAgentProcessor.java:51-251).

Runs a fused chain of processors in memory.  For each source record, processor i is
invoked on the records of step i-1; once every record of step i has emitted, the
results are concatenated and handed to step i+1.  The first error short-circuits to
a final error for that source record.  Processors may emit asynchronously from any
thread (GPU engines do), so the per-step join is lock-protected.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Any, Dict, List, Optional

from ..api.agent import AgentProcessor, AgentSink, AgentSource, AgentStatusResponse
from ..api.record import Record, RecordSink, SourceRecordAndResult

log = logging.getLogger(__name__)

# Optional stage tracer (benchmarks): when a list, every record entering processor i of a
# composite appends (source key, agent type of processor i, time.time()); the chain's end
# appends (key, "end", t).  Off (None) by default: one attribute test per step.
STAGE_TRACE: Optional[list] = None


class CompositeAgentProcessor(AgentProcessor):
    def __init__(self, factory=None):
        super().__init__()
        self.factory = factory  # callable(agent_type) -> AgentCode
        self.processors: List[AgentProcessor] = []
        self.source: Optional[AgentSource] = None
        self.sink: Optional[AgentSink] = None

    def init(self, configuration: Dict[str, Any]) -> None:
        from .registry import create_agent
        make = self.factory or create_agent
        src = configuration.get("source") or {}
        if src:
            self.source = make(src["agentType"])
            self.source.set_metadata(src["agentId"], src["agentType"], self._started_at)
            self.source.init(src.get("configuration") or {})
        for p in configuration.get("processors") or []:
            proc = make(p["agentType"])
            proc.set_metadata(p["agentId"], p["agentType"], self._started_at)
            proc.init(p.get("configuration") or {})
            self.processors.append(proc)
        snk = configuration.get("sink") or {}
        if snk:
            self.sink = make(snk["agentType"])
            self.sink.set_metadata(snk["agentId"], snk["agentType"], self._started_at)
            self.sink.init(snk.get("configuration") or {})

    def set_context(self, context) -> None:
        super().set_context(context)
        for p in self.processors:
            p.set_context(context)

    def start(self) -> None:
        for p in self.processors:
            p.start()

    def close(self) -> None:
        for p in self.processors:
            try:
                p.close()
            except Exception:  # noqa: BLE001
                log.exception("error closing processor")

    def restart(self) -> None:
        for p in self.processors:
            p.restart()

    def get_agent_status(self) -> List[AgentStatusResponse]:
        out: List[AgentStatusResponse] = []
        for p in self.processors:
            out.extend(p.get_agent_status())
        return out

    def process(self, records: List[Record], sink: RecordSink) -> None:
        if not records:
            raise ValueError("Records cannot be null or empty")
        self.processed(len(records), 0)
        if not self.processors:
            for r in records:
                sink(SourceRecordAndResult(r, [r], None))
            return
        for r in records:
            self._invoke(0, [r], r, sink)

    def _invoke(self, index: int, current: List[Record], initial: Record, final: RecordSink) -> None:
        proc = self.processors[index]
        tr = STAGE_TRACE
        if tr is not None:
            tr.append((initial.key(), f"{index}:{proc._agent_id}", time.time()))
        state = {"results": [], "failed": False}
        lock = threading.Lock()
        n = len(current)

        def on_result(res: SourceRecordAndResult) -> None:
            with lock:
                if state["failed"]:
                    return
                if res.error is not None:
                    state["failed"] = True
                    err = res.error
                else:
                    state["results"].append(res)
                    if len(state["results"]) != n:
                        return
                    err = None
                results = list(state["results"])
            if err is not None:
                final(SourceRecordAndResult(initial, None, err))
                return
            out: List[Record] = []
            for x in results:
                if x.result_records:
                    out.extend(x.result_records)
            if not out:
                self.processed(0, 0)
                final(SourceRecordAndResult(initial, [], None))
            elif index == len(self.processors) - 1:
                self.processed(0, len(out))
                if tr is not None:
                    tr.append((initial.key(), "end", time.time()))
                final(SourceRecordAndResult(initial, out, None))
            else:
                self._invoke(index + 1, out, initial, final)

        try:
            proc.process(current, on_result)
        except Exception as e:  # noqa: BLE001
            log.exception("Internal Error processing record")
            final(SourceRecordAndResult(initial, None, e))
