"""Ported reference runtime scenarios, part 1: the agent runner's record loop and error
policies.  Each test cites the Java method it mirrors under
``langstream-runtime/langstream-runtime-impl/src/test/java/ai/langstream/``; every
topic-level case runs on the memory streaming cluster and on the in-tree Kafka broker.
"""
from __future__ import annotations

import random
import threading

import pytest

from ref_runtime_harness import (AsyncProcessor, FailingSink, InjectedFailure, MockService, Run, uniq)
from langstream_amd.api.agent import AbstractAgentCode, AgentSink, AgentSource, SingleRecordAgentProcessor, completed
from langstream_amd.api.record import SimpleRecord
from langstream_amd.runtime.errors import PermanentFailureException
from langstream_amd.runtime.runner import AgentRunner
from langstream_amd.topics.kafka.broker import KafkaBroker


@pytest.fixture(scope="module")
def kafka():
    b = KafkaBroker(default_partitions=1).start()
    yield b
    b.stop()


@pytest.fixture(params=["memory", "kafka"])
def streaming(request, kafka):
    return request.param, (kafka.bootstrap if request.param == "kafka" else None)


# ---------------------------------------------------------------- runtime/agent/AgentRunnerTest.java
class _Sink(AgentSink):
    def write(self, record):
        return completed(None)


class _Source(AgentSource):
    def __init__(self, records, batch=1):
        super().__init__()
        self.records = list(records)
        self.batch = batch
        self.uncommitted = []
        self.lock = threading.Lock()

    def has_more(self):
        with self.lock:
            return bool(self.records)

    def read(self):
        with self.lock:
            out = self.records[: self.batch]
            del self.records[: self.batch]
            self.uncommitted += out
            return out

    def commit(self, records):
        with self.lock:
            for r in records:
                self.uncommitted.remove(r)


class _Processor(SingleRecordAgentProcessor):
    def __init__(self, fail_on):
        super().__init__()
        self.fail_on = set(fail_on)
        self.executions = 0

    def process_record(self, record):
        self.executions += 1
        if record.value() in self.fail_on:
            raise RuntimeError(f"Failed on {record.value()}")
        return [record]


def _loop(values, errors, batch=1):
    src = _Source([SimpleRecord.of("key", v) for v in values], batch)
    proc = _Processor({"fail-me"})
    err = None
    try:
        AgentRunner.run_main_loop(src, proc, _Sink(), errors=errors, has_more=src.has_more)
    except PermanentFailureException as e:
        err = e
    return src, proc, err


def test_agent_runner_skip():
    """AgentRunnerTest.skip"""
    src, proc, err = _loop(["fail-me"], {"retries": 0, "onFailure": "skip"})
    assert err is None and proc.executions == 1 and src.uncommitted == []


def test_agent_runner_fail_with_retries():
    """AgentRunnerTest.failWithRetries: 3 executions (the global counter), then the
    PermanentFailureException; the record stays uncommitted."""
    src, proc, err = _loop(["fail-me"], {"retries": 3, "onFailure": "fail"})
    assert isinstance(err, PermanentFailureException)
    assert proc.executions == 3 and len(src.uncommitted) == 1


def test_agent_runner_fail_no_retries():
    """AgentRunnerTest.failNoRetries"""
    src, proc, err = _loop(["fail-me"], {"retries": 0, "onFailure": "fail"})
    assert isinstance(err, PermanentFailureException)
    assert proc.executions == 1 and len(src.uncommitted) == 1


@pytest.mark.parametrize("values,batch", [
    (["fail-me", "process-me"], 1),   # someFailedSomeGoodWithSkip
    (["process-me", "fail-me"], 1),   # someGoodSomeFailedWithSkip
    (["process-me", "fail-me"], 2),   # someGoodSomeFailedWithSkipAndBatching
    (["fail-me", "process-me"], 2),   # someFailedSomeGoodWithSkipAndBatching
])
def test_agent_runner_some_failed_some_good_with_skip(values, batch):
    """AgentRunnerTest.{someFailedSomeGood,someGoodSomeFailed}WithSkip[AndBatching]"""
    src, proc, err = _loop(values, {"retries": 0, "onFailure": "skip"}, batch)
    assert err is None and proc.executions == 2 and src.uncommitted == []


# ---------------------------------------------------------------- kafka/ErrorHandlingTest.java
def _module(tin, tout, agent_type, step_errors="", module_errors="", extra_topic_opts="", output=True):
    out_topic = f"  - name: \"{tout}\"\n    creation-mode: create-if-not-exists\n" if output else ""
    out_line = f"    output: \"{tout}\"\n" if output else ""
    return {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
{extra_topic_opts}{out_topic}{module_errors}pipeline:
  - name: "some agent"
    id: "step"
    type: "{agent_type}"
    input: "{tin}"
{out_line}{step_errors}    configuration:
      fail-on-content: "fail-me"
"""}


POLL10 = "    options:\n      consumer.max.poll.records: 10\n"


def test_error_handling_discard_errors(streaming):
    """ErrorHandlingTest.testDiscardErrors: step-level skip (retries 3) overrides the
    module's fail (retries 5); only keep-me reaches the output."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _module(tin, tout, "mock-failing-processor",
                    step_errors="    errors:\n        on-failure: skip\n        retries: 3\n",
                    module_errors="errors:\n    on-failure: fail\n    retries: 5\n", extra_topic_opts=POLL10)
    with Run(*streaming, files) as r:
        r.produce(tin, "fail-me")
        r.produce(tin, "keep-me")
        r.wait_for(tout, ["keep-me"])
        assert not r.app.errors


def test_error_handling_dead_letter(streaming):
    """ErrorHandlingTest.testDeadLetter: failures go to <input>-deadletter, in order."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _module(tin, tout, "mock-failing-processor", step_errors="    errors:\n        on-failure: dead-letter\n")
    with Run(*streaming, files) as r:
        for i in range(10):
            r.produce(tin, f"fail-me-{i}")
            r.produce(tin, f"keep-me-{i}")
        r.wait_for(tin + "-deadletter", [f"fail-me-{i}" for i in range(10)])
        r.wait_for(tout, [f"keep-me-{i}" for i in range(10)])


def test_error_handling_fail_on_errors(streaming):
    """ErrorHandlingTest.testFailOnErrors: the runner fails with PermanentFailureException
    caused by the injected failure; running the pipeline again fails again on the same
    (uncommitted) first record."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _module(tin, tout, "mock-failing-processor", module_errors="errors:\n    on-failure: fail\n    retries: 5\n",
                    extra_topic_opts=POLL10)
    for attempt in range(2):
        with Run(*streaming, files) as r:
            if attempt == 0:
                r.produce(tin, "fail-me")
                r.produce(tin, "keep-me")
            e = r.wait_failure()
            assert isinstance(e, PermanentFailureException)
            assert isinstance(e.__cause__, InjectedFailure) and str(e.__cause__) == "Failing on content: fail-me"
            # (the second run fails on the same record: the failed one was never committed)


def test_error_handling_discard_errors_on_sink(streaming):
    """ErrorHandlingTest.testDiscardErrorsOnSink"""
    tin = uniq("input-topic")
    files = _module(tin, None, "mock-failing-sink", output=False,
                    step_errors="    errors:\n        on-failure: skip\n        retries: 3\n",
                    module_errors="errors:\n    on-failure: fail\n    retries: 5\n", extra_topic_opts=POLL10)
    with Run(*streaming, files) as r:
        r.produce(tin, "fail-me")
        r.produce(tin, "keep-me")
        _until(lambda: len(FailingSink.accepted) == 1)
        assert [x.value() for x in FailingSink.accepted] == ["keep-me"]


def test_error_handling_fail_on_errors_on_sink(streaming):
    """ErrorHandlingTest.testFailOnErrorsOnSink: step fail (retries 3) overrides module skip."""
    tin = uniq("input-topic")
    files = _module(tin, None, "mock-failing-sink", output=False,
                    step_errors="    errors:\n        on-failure: fail\n        retries: 3\n",
                    module_errors="errors:\n    on-failure: skip\n    retries: 5\n", extra_topic_opts=POLL10)
    for attempt in range(2):
        with Run(*streaming, files) as r:
            if attempt == 0:
                r.produce(tin, "fail-me")
                r.produce(tin, "keep-me")
            e = r.wait_failure()
            assert isinstance(e, PermanentFailureException) and str(e.__cause__) == "Failing on content: fail-me"


def test_error_handling_dead_letter_on_sink(streaming):
    """ErrorHandlingTest.testDeadLetterOnSink"""
    tin = uniq("input-topic")
    files = _module(tin, None, "mock-failing-sink", output=False,
                    step_errors="    errors:\n        on-failure: dead-letter\n        retries: 3\n")
    with Run(*streaming, files) as r:
        for i in range(10):
            r.produce(tin, f"fail-me-{i}")
            r.produce(tin, f"keep-me-{i}")
        r.wait_for(tin + "-deadletter", [f"fail-me-{i}" for i in range(10)])
        _until(lambda: len(FailingSink.accepted) == 10)
        assert sorted(x.value() for x in FailingSink.accepted) == sorted(f"keep-me-{i}" for i in range(10))


def _until(cond, timeout=30.0):
    import time
    deadline = time.time() + timeout
    while not cond():
        assert time.time() < deadline, "condition not reached"
        time.sleep(0.02)


# ---------------------------------------------------------------- kafka/AsyncProcessingIT.java
def _async_files(tin, tout, body, errors=""):
    return {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
{errors}topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
    partitions: 4
  - name: "{tout}"
    creation-mode: create-if-not-exists
    partitions: 2
pipeline:
{body.format(tin=tin, tout=tout)}"""}


def test_async_process_multi_thread_out_of_order(streaming):
    """AsyncProcessingIT.testProcessMultiThreadOutOfOrder: 100 records emitted out of
    order from 8 threads; all arrive, commits stay ordered."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    body = ('  - name: "async-process-records"\n    id: "step1"\n    type: "mock-async-processor"\n'
            '    input: "{tin}"\n    output: "{tout}"\n')
    with Run(*streaming, _async_files(tin, tout, body)) as r:
        want = [f"test message {i}" for i in range(100)]
        for v in want:
            r.produce(tin, v)
        r.wait_any_order(tout, want)


COMPOSITE = ('  - name: "async-process-records"\n    id: "step1"\n    type: "mock-async-processor"\n    input: "{tin}"\n'
             '  - name: "mock-failing-processor"\n    id: "step2"\n    type: "mock-failing-processor"\n'
             '  - name: "async-process-records"\n    id: "step3"\n    type: "mock-async-processor"\n'
             '  - name: "mock-failing-processor"\n    id: "step4"\n    type: "mock-failing-processor"\n'
             '    output: "{tout}"\n')


def test_async_composite_multi_step_out_of_order(streaming):
    """AsyncProcessingIT.testCompositeMultiStepProcessMultiThreadOutOfOrder: the four steps
    fuse into one composite agent; async steps interleave with sync ones."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run(*streaming, _async_files(tin, tout, COMPOSITE)) as r:
        assert [n.agent_type for n in r.plan.agents.values()] == ["composite-agent"]
        want = [f"test message {i}" for i in range(100)]
        for v in want:
            r.produce(tin, v)
        r.wait_any_order(tout, want)


FAILING_COMPOSITE = (
    '  - name: "mock-failing-processor"\n    type: "mock-failing-processor"\n    id: "step1"\n    input: "{tin}"\n'
    '    configuration:\n       fail-on-content: "fail-this-message-in-the-beginning"\n'
    '  - name: "async-process-records"\n    id: "step2"\n    type: "mock-async-processor"\n'
    '  - name: "mock-failing-processor"\n    id: "step3"\n    configuration:\n'
    '       fail-on-content: "fail-this-message-in-the-middle"\n    type: "mock-failing-processor"\n'
    '  - name: "async-process-records"\n    id: "step4"\n    type: "mock-async-processor"\n'
    '  - name: "mock-failing-processor"\n    id: "step5"\n    type: "mock-failing-processor"\n    output: "{tout}"\n'
    '    configuration:\n       fail-on-content: "fail-this-message-in-the-end"\n')


def _random_mix(dead_letter: bool, seed: int):
    rng = random.Random(seed)
    sent, ok, dlq = [], [], []
    for i in range(100):
        n = rng.randrange(5)
        if n < 3:
            v = ["fail-this-message-in-the-beginning", "fail-this-message-in-the-middle",
                 "fail-this-message-in-the-end"][n] + (f"-{i}" if dead_letter else "")
            dlq.append(v)
        else:
            v = f"test message {i}"
            ok.append(v)
        sent.append(v)
    return sent, ok, dlq


@pytest.mark.parametrize("retries", [0, 1, 2])
def test_async_composite_failure_and_skip(streaming, retries):
    """AsyncProcessingIT.testCompositeMultiStepProcessMultiThreadOutOfOrderWithFailureAndSkip"""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _async_files(tin, tout, FAILING_COMPOSITE, f"errors:\n   on-failure: skip\n   retries: {retries}\n")
    sent, ok, _ = _random_mix(False, retries)
    with Run(*streaming, files) as r:
        for v in sent:
            r.produce(tin, v)
        r.wait_any_order(tout, ok)


@pytest.mark.parametrize("retries", [0, 1, 2])
def test_async_composite_failure_and_dead_letter(streaming, retries):
    """AsyncProcessingIT.testCompositeMultiStepProcessMultiThreadOutOfOrderWithFailureAndDeadletter"""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _async_files(tin, tout, FAILING_COMPOSITE, f"errors:\n   on-failure: dead-letter\n   retries: {retries}\n")
    sent, ok, dlq = _random_mix(True, 10 + retries)
    with Run(*streaming, files) as r:
        for v in sent:
            r.produce(tin, v)
        r.wait_any_order(tout, ok)
        r.wait_any_order(tin + "-deadletter", dlq)


@pytest.mark.parametrize("content", ["fail-this-message-in-the-beginning", "fail-this-message-in-the-middle",
                                     "fail-this-message-in-the-end"])
@pytest.mark.parametrize("retries", [0, 1, 2])
def test_async_composite_with_fail(content, retries):
    """AsyncProcessingIT.testCompositeMultiStepProcessMultiThreadOutOfOrderWithFail: with
    on-failure: fail, the message that fails at the beginning, middle or end of the async
    composite stops the agent with the injected failure as cause (every retry count)."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = _async_files(tin, tout, FAILING_COMPOSITE, f"errors:\n   on-failure: fail\n   retries: {retries}\n")
    with Run("memory", None, files) as r:
        r.produce(tin, content)
        err = r.wait_failure()
        assert isinstance(err, PermanentFailureException)
        assert isinstance(err.__cause__, InjectedFailure), repr(err.__cause__)


# ---------------------------------------------------------------- state/StatefulAgentsTest.java
def test_single_stateful_agent(streaming, tmp_path):
    """StatefulAgentsTest.testSingleStatefulAgent: the agent's disk state survives a
    redeploy; reading the output from the beginning shows the whole sequence."""
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
  - name: "{tout}"
    creation-mode: create-if-not-exists
pipeline:
  - name: "some agent"
    id: "step"
    type: "mock-stateful-processor"
    input: "{tin}"
    output: "{tout}"
    resources:
       disk:
          enabled: true
"""}
    state = str(tmp_path / "state")
    with Run(*streaming, files, state_dir=state) as r:
        r.produce(tin, "a")
        r.produce(tin, "b")
        r.wait_for(tout, ["a", "ab"])
    with Run(*streaming, files, state_dir=state) as r:
        r.produce(tin, "c")
        r.produce(tin, "d")
        r.wait_for(tout, ["a", "ab", "abc", "abcd"])


# ---------------------------------------------------------------- services/ServiceAgentIT.java
def test_service_agent(tmp_path):
    """ServiceAgentIT.testService: a streaming-less app with one service agent: started,
    joined and closed exactly once."""
    MockService.reset()
    files = {"module.yaml": 'pipeline:\n  - name: "Service"\n    type: "mock-service"\n    id: step1\n'}
    r = Run("memory", None, files)
    with r:
        _until(lambda: MockService.joins >= 1)
    assert (MockService.starts, MockService.joins, MockService.closes) == (1, 1, 1)


# ---------------------------------------------------------------- kafka/KafkaRunnerDockerTest.java
def test_kafka_connect_to_topics(kafka):
    """KafkaRunnerDockerTest.testConnectToTopics: the topics exist on the broker after
    deploy; identity moves the record."""
    from langstream_amd.topics.kafka.client import KafkaClient
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
  - name: "{tout}"
    creation-mode: create-if-not-exists
pipeline:
  - id: "step1"
    type: "identity"
    input: "{tin}"
    output: "{tout}"
"""}
    with Run("kafka", kafka.bootstrap, files) as r:
        c = KafkaClient(kafka.bootstrap)
        assert tin in c.list_topics()
        c.close()
        r.produce(tin, "value")
        r.wait_for(tout, ["value"])


def test_kafka_apply_retention(kafka):
    """KafkaRunnerDockerTest.testApplyRetention: a topic's ``config`` reaches the broker
    (DescribeConfigs shows retention.ms = 300000)."""
    from langstream_amd.topics.kafka.client import KafkaClient
    tin = uniq("input-topic-with-retention")
    files = {"module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
    config:
      retention.ms: 300000
pipeline:
  - id: "step1"
    type: "identity"
    input: "{tin}"
"""}
    with Run("kafka", kafka.bootstrap, files):
        c = KafkaClient(kafka.bootstrap)
        assert tin in c.list_topics()
        assert c.describe_topic_configs(tin)["retention.ms"] == "300000"
        c.close()
