"""AgentRunner: the per-agent record loop.

Parity: RT/agent/AgentRunner.java -- run/wiring :138-473, pending-record accounting
:475-625, bad-record handler :627-649, main loop :651-730, sink write + retries
:750-854, processor error handling :856-943, SimpleAgentContext :1024-1136;
RT/agent/TopicConsumerSource.java, TopicProducerSink.java.

Loop: source.read() -> processor.process(records, sink_cb) -> for each result:
  error    -> errors handler: RETRY (re-process that record) / SKIP (commit) / FAIL
              (permanent_failure; fatal unless on-failure is skip|dead-letter)
  []       -> commit the source record
  records  -> tracker.track; sink.write(each) -> on success tracker.commit (in-order
              source commit); on error -> errors handler (retry write / skip / fail)
A fatal error stops the loop (the pod would restart); records not committed are
redelivered by the topic runtime (at-least-once).
"""
from __future__ import annotations

import logging
import threading
import time
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..api.agent import (AgentCode, AgentContext, AgentProcessor, AgentService, AgentSink, AgentSource,
                         BadRecordHandler, ComponentType, completed)
from ..api.record import Record, SourceRecordAndResult
from ..api.topics import BatchWriteError, TopicConnectionProvider, TopicConnectionsRuntimeRegistry
from .composite import CompositeAgentProcessor
from .errors import Outcome, PermanentFailureException, StandardErrorsHandler
from .metrics import MetricsReporter
from .tracker import SourceRecordTracker

log = logging.getLogger(__name__)


class _ResultSink:
    """The callback a processor reports results through: ``sink(result)`` per record, or
    ``sink.many(results)`` for a batch completed together."""
    __slots__ = ("runner", "errors")

    def __init__(self, runner: "AgentRunner", errors: StandardErrorsHandler):
        self.runner, self.errors = runner, errors

    def __call__(self, res: SourceRecordAndResult) -> None:
        self.runner._on_processor_result(res, self.errors)

    def many(self, results: List[SourceRecordAndResult]) -> None:
        self.runner._on_processor_results(results, self.errors)


# ---------------------------------------------------------------- default adapters
class TopicConsumerSource(AgentSource):
    """Source reading from the agent's input topic; permanent failures go to the DLQ
    when one is configured, else are rethrown."""

    def __init__(self, consumer, dlq_producer=None):
        super().__init__()
        self.consumer = consumer
        self.dlq = dlq_producer

    def start(self) -> None:
        self.consumer.start()
        if self.dlq is not None:
            self.dlq.start()

    def close(self) -> None:
        self.consumer.close()
        if self.dlq is not None:
            self.dlq.close()

    def read(self) -> List[Record]:
        recs = self.consumer.read()
        self.processed(0, len(recs))
        return recs

    def commit(self, records: List[Record]) -> None:
        self.consumer.commit(records)

    def permanent_failure(self, record: Record, error: BaseException) -> None:
        if self.dlq is None:
            raise error
        from ..api.record import Header, SimpleRecord
        cause = error.__cause__ or error
        rec = SimpleRecord.with_headers(record, [Header("cause-msg", str(cause)),
                                                 Header("cause-class", type(cause).__name__)])
        self.dlq.write(rec).result(timeout=30)
        self.consumer.commit([record])

    def build_additional_info(self) -> Dict[str, Any]:
        return {"consumer": self.consumer.get_info()}


class TopicProducerSink(AgentSink):
    def __init__(self, producer):
        super().__init__()
        self.producer = producer

    def start(self) -> None:
        self.producer.start()

    def close(self) -> None:
        self.producer.close()

    def write(self, record: Record) -> Future:
        self.processed(1, 0)
        return self.producer.write(record)

    def write_many(self, records: List[Record]) -> Future:
        self.processed(len(records), 0)
        return self.producer.write_many(records)

    def build_additional_info(self) -> Dict[str, Any]:
        return {"producer": self.producer.get_info()}


class NoopSink(AgentSink):
    """Used when an agent has no output: records are dropped (and committed)."""

    def write(self, record: Record) -> Future:
        self.processed(1, 0)
        return completed(None)


class IdentityProcessor(AgentProcessor):
    def process(self, records, sink) -> None:
        self.processed(len(records), len(records))
        for r in records:
            sink(SourceRecordAndResult(r, [r], None))


# ---------------------------------------------------------------- pod configuration
@dataclass
class RuntimePodConfiguration:
    """RTAPI/agent/RuntimePodConfiguration.java: what a pod needs to run one agent."""
    agent_id: str
    agent_type: str
    component_type: str
    application_id: str
    tenant: str
    configuration: Dict[str, Any]
    input: Dict[str, Any] = field(default_factory=dict)      # {topic, deadLetterTopicProducer?}
    output: Dict[str, Any] = field(default_factory=dict)     # {topic}
    streaming_cluster: Any = None
    errors: Dict[str, Any] = field(default_factory=lambda: {"retries": 0, "onFailure": "fail"})
    code_directory: str = ""
    persistent_state_directory: Optional[str] = None
    replica: int = 0


class AgentRunner:
    def __init__(self, pod: RuntimePodConfiguration, services=None, metrics: Optional[MetricsReporter] = None):
        self.pod = pod
        self.services = services
        self.metrics = metrics or MetricsReporter.global_reporter()
        self._continue = threading.Event()
        self._continue.set()
        self._fatal: Optional[BaseException] = None
        self._fatal_lock = threading.Lock()
        self.source: Optional[AgentSource] = None
        self.processor: Optional[AgentProcessor] = None
        self.sink: Optional[AgentSink] = None
        self.service: Optional[AgentService] = None
        self.main_code: Optional[AgentCode] = None
        self.tracker: Optional[SourceRecordTracker] = None
        self.started = threading.Event()
        self.stopped = threading.Event()
        self.records_in = 0
        self.records_out = 0

    # ------------------------------------------------------------------ wiring
    def _make_context(self, topic_rt, consumer, producer, bad_record_handler) -> AgentContext:
        p = self.pod
        return AgentContext(
            agent_id=p.agent_id, global_agent_id=f"{p.application_id}-{p.agent_id}", tenant=p.tenant,
            consumer=consumer, producer=producer, topic_admin=None,
            topic_connection_provider=TopicConnectionProvider(topic_rt, p.streaming_cluster),
            metrics_reporter=self.metrics.with_agent(p.agent_id), bad_record_handler=bad_record_handler,
            critical_failure=self._critical_failure, code_directory=p.code_directory,
            persistent_state_directory=p.persistent_state_directory, services=self.services)

    def _critical_failure(self, error: BaseException) -> None:
        log.error("critical failure in agent %s: %r", self.pod.agent_id, error)
        self._set_fatal(error)
        self.stop()

    def _set_fatal(self, e: BaseException) -> None:
        with self._fatal_lock:
            if self._fatal is None:
                self._fatal = e

    def build(self) -> None:
        from .registry import create_agent
        p = self.pod
        topic_rt = TopicConnectionsRuntimeRegistry.get(p.streaming_cluster) if p.streaming_cluster else None
        consumer = producer = dlq = None
        if topic_rt is not None and p.input.get("topic"):
            consumer = topic_rt.create_consumer(p.agent_id, p.streaming_cluster, p.input)
            dlq = topic_rt.create_deadletter_topic_producer(p.agent_id, p.streaming_cluster, p.input)
        if topic_rt is not None and p.output.get("topic"):
            producer = topic_rt.create_producer(p.agent_id, p.streaming_cluster, p.output)
        on_failure = str(p.errors.get("onFailure", "fail"))

        def brh_fn(record, error, cleanup):
            if on_failure == "skip":
                log.warning("Skipping record %s: %r", record, error)
            elif on_failure == "dead-letter" and dlq is not None:
                dlq.write(record).result(timeout=30)
            else:
                cleanup()
                raise error

        ctx = self._make_context(topic_rt, consumer, producer, BadRecordHandler(brh_fn))
        self.context = ctx
        code = create_agent(p.agent_type)
        code.set_metadata(p.agent_id, p.agent_type, int(time.time() * 1000))
        code.init(p.configuration)
        self.main_code = code
        if isinstance(code, AgentService):
            self.service = code
        else:
            if isinstance(code, CompositeAgentProcessor):
                self.source = code.source
                self.sink = code.sink
                self.processor = code
            elif isinstance(code, AgentSource):
                self.source = code
            elif isinstance(code, AgentSink):
                self.sink = code
            elif isinstance(code, AgentProcessor):
                self.processor = code
            if self.source is None:
                if consumer is None:
                    raise ValueError(f"agent {p.agent_id} has no input topic and is not a source")
                self.source = TopicConsumerSource(consumer, dlq)
                self.source.set_metadata(p.agent_id, "topic-source", int(time.time() * 1000))
            if self.processor is None:
                self.processor = IdentityProcessor()
                self.processor.set_metadata(p.agent_id, "identity", int(time.time() * 1000))
            if self.sink is None:
                if producer is not None:
                    self.sink = TopicProducerSink(producer)
                    self.sink.set_metadata(p.agent_id, "topic-sink", int(time.time() * 1000))
                else:
                    self.sink = NoopSink()
                    self.sink.set_metadata(p.agent_id, "noop-sink", int(time.time() * 1000))
        self._topic_rt = topic_rt

    # ------------------------------------------------------------------ run
    @classmethod
    def run_main_loop(cls, source: AgentSource, processor: AgentProcessor, sink: AgentSink,
                      errors: Optional[Dict[str, Any]] = None, has_more=None, context: Optional[AgentContext] = None,
                      agent_id: str = "agent", max_loops: Optional[int] = None) -> "AgentRunner":
        """``AgentRunner.runMainLoop(source, processor, sink, context, errorsHandler,
        continueLoop)`` (RT/agent/AgentRunner.java:651-730) for already-built components:
        the loop runs while ``has_more()`` is true (then drains in-flight records) and
        raises the fatal error -- a ``PermanentFailureException`` under ``fail`` -- like
        the reference's static entry point.  Returns the runner (tracker, counters)."""
        pod = RuntimePodConfiguration(agent_id=agent_id, agent_type="custom", component_type="PROCESSOR",
                                      application_id="app", tenant="default", configuration={},
                                      errors=dict(errors or {"retries": 0, "onFailure": "fail"}))
        r = cls(pod)
        r.source, r.processor, r.sink = source, processor, sink
        r.main_code = processor
        r.context = context or r._make_context(None, None, None, BadRecordHandler(lambda rec, err, cleanup: None))
        try:
            r._main_loop(max_loops, has_more)
        finally:
            r._close()
            r.stopped.set()
        return r

    def stop(self) -> None:
        self._continue.clear()

    def run(self, max_loops: Optional[int] = None) -> None:
        """Blocking main loop; returns on stop() (or raises the fatal error)."""
        if self.main_code is None:
            self.build()
        try:
            if self.service is not None:
                self.service.set_context(self.context)
                self.service.start()
                self.started.set()
                while self._continue.is_set():
                    if getattr(self.service, "join_timeout", None):
                        if self.service.join_timeout(0.2):
                            break
                    else:
                        time.sleep(0.2)
                return
            self._main_loop(max_loops)
        finally:
            self._close()
            self.stopped.set()
        if self._fatal is not None:
            raise self._fatal

    def _close(self) -> None:
        for c in (self.source, self.processor, self.sink, self.service):
            if c is None:
                continue
            try:
                c.close()
            except Exception:  # noqa: BLE001
                log.exception("error closing %s", c)

    def _main_loop(self, max_loops: Optional[int], continue_fn: Optional[Callable[[], bool]] = None) -> None:
        source, processor, sink = self.source, self.processor, self.sink
        for c in (source, sink, processor):
            c.set_context(self.context)
        source.start()
        sink.start()
        processor.start()
        self.tracker = SourceRecordTracker(source)
        errors = StandardErrorsHandler(self.pod.errors)
        self.started.set()
        loops = 0
        while self._continue.is_set() and (continue_fn is None or continue_fn()):
            records = source.read()
            if records:
                self.records_in += len(records)
                self.metrics.counter("source_records_in", self.pod.agent_id).inc(len(records))
                self._run_processor(records, errors)
            self._check_fatal()
            if sink.handles_commit():
                sink.commit()
            loops += 1
            if max_loops is not None and loops >= max_loops:
                break
        self._drain(timeout=60.0)
        self._check_fatal()

    def _drain(self, timeout: float) -> None:
        """Wait (bounded) for in-flight records to reach the sink (E4).  A sink that
        handles its own commits (Kafka Connect) drains on close() instead."""
        if self.sink is not None and self.sink.handles_commit():
            return
        deadline = time.time() + timeout
        while self.tracker is not None and self.tracker.pending() > 0 and time.time() < deadline:
            if self._fatal is not None:
                return
            time.sleep(0.01)

    def _check_fatal(self) -> None:
        if self._fatal is not None:
            raise self._fatal

    # -- processor results
    def _run_processor(self, records: List[Record], errors: StandardErrorsHandler) -> None:
        self.processor.process(records, _ResultSink(self, errors))

    def _on_processor_results(self, results: List[SourceRecordAndResult], errors: StandardErrorsHandler) -> None:
        """A batch of results at once (a processor that completes records in batches,
        e.g. compute-ai-embeddings): one tracker update, ONE sink write of all the
        result records (``write_many``) and one commit pass when it is acknowledged.
        Errors and empty results take the per-record path; a failed batch write hands
        every record to the per-record write-error handling (retry / skip / DLQ)."""
        writer = getattr(self.sink, "write_many", None)
        if writer is None or self.sink.handles_commit():
            for r in results:
                self._on_processor_result(r, errors)
            return
        ok = []
        for r in results:
            if r.error is None and r.result_records:
                ok.append(r)
            else:
                self._on_processor_result(r, errors)
        if not ok:
            return
        try:
            self.tracker.track(ok)
            recs = [rec for r in ok for rec in r.result_records]
            fut = writer(recs)
        except BaseException as e:  # noqa: BLE001
            log.exception("Error while processing record")
            self._set_fatal(RuntimeError(f"Error while processing records: {e!r}"))
            return

        def done(f: Future) -> None:
            err = f.exception()
            if err is None:
                self.records_out += len(recs)
                self.metrics.counter("sink_records_out", self.pod.agent_id).inc(len(recs))
                self.tracker.commit(recs)
                return
            # a BatchWriteError names the records that failed: the delivered ones commit,
            # only the failed ones go to retry / skip / dead-letter
            per = err.errors if isinstance(err, BatchWriteError) and len(err.errors) == len(recs) else None
            i = 0
            delivered = []
            for r in ok:
                for rec in r.result_records:
                    e = err if per is None else per[i]
                    i += 1
                    if e is None:
                        delivered.append(rec)
                    else:
                        self._on_write_error(rec, r.source_record, e, errors)
            if delivered:
                self.records_out += len(delivered)
                self.metrics.counter("sink_records_out", self.pod.agent_id).inc(len(delivered))
                self.tracker.commit(delivered)

        fut.add_done_callback(done)

    def _on_processor_result(self, res: SourceRecordAndResult, errors: StandardErrorsHandler) -> None:
        src = res.source_record
        try:
            if res.error is not None:
                action = errors.handle_errors(src, res.error)
                if action == Outcome.SKIP:
                    log.error("Unrecoverable error while processing the records, skipping: %r", res.error)
                    self._on_final(SourceRecordAndResult(src, [], None), errors)
                elif action == Outcome.RETRY:
                    log.error("Retryable error while processing the records, retrying: %r", res.error)
                    self._run_processor([src], errors)
                else:
                    pfe = PermanentFailureException(res.error)
                    self.source.permanent_failure(src, pfe)
                    if errors.fail_processing_on_permanent_errors():
                        self._on_final(SourceRecordAndResult(src, [], pfe), errors)
                    else:
                        self._on_final(SourceRecordAndResult(src, [], None), errors)
            else:
                self._on_final(res, errors)
        except BaseException as e:  # noqa: BLE001
            log.exception("Error while processing record")
            self._set_fatal(e if isinstance(e, PermanentFailureException) else RuntimeError(
                f"Error while processing records: {e!r}"))

    def _on_final(self, res: SourceRecordAndResult, errors: StandardErrorsHandler) -> None:
        if res.error is not None:
            log.error("Fatal error: %r", res.error)
            self._set_fatal(res.error)
            return
        if not res.result_records:
            try:
                self.source.commit([res.source_record])
            except BaseException as e:  # noqa: BLE001
                self._set_fatal(e)
            return
        self.tracker.track([res])
        for rec in list(res.result_records):
            self._write(rec, res.source_record, errors)

    def _write(self, rec: Record, src: Record, errors: StandardErrorsHandler) -> None:
        fut = self.sink.write(rec)
        if self.sink.handles_commit():
            fut.add_done_callback(lambda f: f.exception() and self._set_fatal(f.exception()))
            return

        def done(f: Future) -> None:
            err = f.exception()
            if err is None:
                self.records_out += 1
                self.metrics.counter("sink_records_out", self.pod.agent_id).inc()
                self.tracker.commit([rec])
                return
            self._on_write_error(rec, src, err, errors)

        fut.add_done_callback(done)

    def _on_write_error(self, rec: Record, src: Record, err: BaseException, errors: StandardErrorsHandler) -> None:
        action = errors.handle_errors(src, err)
        if action == Outcome.SKIP:
            self.tracker.commit([rec])
        elif action == Outcome.RETRY:
            self._write(rec, src, errors)
        else:
            pfe = PermanentFailureException(err)
            try:
                self.source.permanent_failure(src, pfe)
            except BaseException as e2:  # noqa: BLE001
                self._set_fatal(e2)
                return
            if errors.fail_processing_on_permanent_errors():
                self._set_fatal(pfe)
            else:
                self.tracker.commit([rec])

    # ------------------------------------------------------------------ introspection
    def agent_info(self) -> List[Dict[str, Any]]:
        """/info payload: AgentStatusResponse of source + processor + sink (or service)."""
        out = []
        comps = [self.service] if self.service is not None else [self.source, self.processor, self.sink]
        for c in comps:
            if c is not None:
                out.extend(s.to_dict() for s in c.get_agent_status())
        return out

    def restart(self) -> None:
        for c in (self.source, self.processor, self.sink, self.service):
            if c is not None:
                c.restart()
