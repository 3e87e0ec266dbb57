"""Flow-control agents (FLOW/*): dispatch, trigger-event, timer-source, log-event.

* dispatch (DispatchAgent.java): ``routes: [{when, destination, action: dispatch|drop}]``;
  the first matching route writes the record to ``destination`` (not emitted
  downstream) or drops it; no match -> default output.
* trigger-event (TriggerEventProcessor.java): when ``when`` holds, a record built from
  ``fields`` (name/expression) is written to ``destination``; the source record then
  continues (``continue-processing`` true) or stops.
* timer-source (TimerSource.java): every ``period-seconds`` (60) emits one record built
  from ``fields``.
* log-event (LogEventProcessor.java): logs ``message`` / ``fields`` when ``when`` holds.
"""
from __future__ import annotations

import json
import logging
import threading
import time
from typing import Any, Dict, List

from ..api.agent import AgentProcessor, AgentSource
from ..api.record import Header, SimpleRecord, SourceRecordAndResult
from ..runtime.registry import register_agent
from .genai.el import eval_expression, eval_predicate
from .genai.mutable import MutableRecord

log = logging.getLogger(__name__)


def _producer(agent, topic):
    p = agent.context.topic_connection_provider.create_producer(agent.context.global_agent_id, topic)
    p.start()
    return p


@register_agent("dispatch")
class DispatchAgent(AgentProcessor):
    def init(self, configuration):
        self.routes = []
        for r in configuration.get("routes") or []:
            action = r.get("action", "dispatch")
            dest = r.get("destination", "") or ""
            if action not in ("dispatch", "drop"):
                raise ValueError(f"invalid action {action}")
            if action == "drop" and dest:
                raise ValueError("drop action cannot have a destination")
            self.routes.append((r.get("when", "true"), dest, action == "drop"))
        self.producers = {}

    def start(self):
        for _, dest, drop in self.routes:
            if dest and dest not in self.producers:
                self.producers[dest] = _producer(self, dest)

    def close(self):
        for p in self.producers.values():
            p.close()

    def process(self, records, sink):
        for r in records:
            try:
                ctx = MutableRecord.from_record(r).el_context()
                for when, dest, drop in self.routes:
                    if eval_predicate(when, ctx):
                        if drop:
                            sink(SourceRecordAndResult(r, [], None))
                        else:
                            f = self.producers[dest].write(r)
                            f.add_done_callback(lambda ff, r=r: sink(SourceRecordAndResult(
                                r, None, ff.exception()) if ff.exception() else SourceRecordAndResult(r, [], None)))
                        break
                else:
                    sink(SourceRecordAndResult(r, [r], None))
            except Exception as e:  # noqa: BLE001
                sink(SourceRecordAndResult(r, None, e))


def _build_fields(fields_cfg):
    return [(f.get("name", ""), f.get("expression", "")) for f in fields_cfg or []]


@register_agent("trigger-event")
class TriggerEventAgent(AgentProcessor):
    def init(self, configuration):
        self.destination = configuration.get("destination")
        if not self.destination:
            raise ValueError("destination is required")
        self.when = configuration.get("when", "true")
        self.continue_processing = str(configuration.get("continue-processing", "true")).lower() == "true"
        self.fields = _build_fields(configuration.get("fields"))

    def start(self):
        self.producer = _producer(self, self.destination)

    def close(self):
        self.producer.close()

    def process(self, records, sink):
        for r in records:
            try:
                mr = MutableRecord.from_record(r).copy()
                ctx = mr.el_context()
                if not eval_predicate(self.when, ctx):
                    sink(SourceRecordAndResult(r, [r], None))
                    continue
                vals = {n: eval_expression(e, ctx) for n, e in self.fields}
                for n, v in vals.items():
                    mr.set_result_field(v, n)
                f = self.producer.write(mr.to_record())
            except Exception as e:  # noqa: BLE001
                sink(SourceRecordAndResult(r, None, e))
                continue

            def done(ff, r=r):
                if ff.exception() is not None:
                    sink(SourceRecordAndResult(r, None, ff.exception()))
                else:
                    sink(SourceRecordAndResult(r, [r] if self.continue_processing else [], None))

            f.add_done_callback(done)


@register_agent("timer-source")
class TimerSource(AgentSource):
    def init(self, configuration):
        self.period = float(configuration.get("period-seconds", 60))
        self.fields = _build_fields(configuration.get("fields"))
        self._next = time.time()

    def read(self):
        now = time.time()
        if now < self._next:
            time.sleep(min(0.2, self._next - now))
            return []
        self._next = now + self.period
        mr = MutableRecord(None, None, {}, None, int(now * 1000))
        ctx = mr.el_context()
        for n, e in self.fields:
            mr.set_result_field(eval_expression(e, ctx), n)
        self.processed(0, 1)
        return [mr.to_record()]

    def commit(self, records):
        pass


@register_agent("log-event")
class LogEventAgent(AgentProcessor):
    def init(self, configuration):
        self.when = configuration.get("when", "true")
        self.message = configuration.get("message", "")
        self.fields = _build_fields(configuration.get("fields"))

    def process(self, records, sink):
        for r in records:
            try:
                ctx = MutableRecord.from_record(r).el_context()
                if eval_predicate(self.when, ctx):
                    from .genai.mustache import render
                    vals = {n: eval_expression(e, ctx) for n, e in self.fields}
                    msg = render(self.message, MutableRecord.from_record(r).json_context()) if self.message else ""
                    log.info("%s %s", msg, json.dumps(vals, default=str) if vals else "")
                sink(SourceRecordAndResult(r, [r], None))
            except Exception as e:  # noqa: BLE001
                sink(SourceRecordAndResult(r, None, e))
