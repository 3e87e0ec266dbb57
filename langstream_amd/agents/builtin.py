"""Built-in agents: identity, noop, composite-agent (RT/agent/simple/*, CompositeAgentProcessorProvider.java)."""
from __future__ import annotations

from ..api.agent import AgentProcessor
from ..api.record import SourceRecordAndResult
from ..runtime.composite import CompositeAgentProcessor
from ..runtime.registry import register_agent


@register_agent("identity")
class IdentityAgent(AgentProcessor):
    def process(self, records, sink):
        self.processed(len(records), len(records))
        for r in records:
            sink(SourceRecordAndResult(r, [r], None))


@register_agent("noop")
class NoopAgent(AgentProcessor):
    """Drops every record (emits nothing, so the source record is committed)."""

    def process(self, records, sink):
        self.processed(len(records), 0)
        for r in records:
            sink(SourceRecordAndResult(r, [], None))


register_agent("composite-agent")(CompositeAgentProcessor)
