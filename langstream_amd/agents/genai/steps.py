"""GenAI toolkit steps (parity: AIA/com/datastax/oss/streaming/ai/*.java, step factory
util/TransformFunctionUtil.java:166-224, configuration defaults
CORE/agents/ai/steps/*Configuration.java).

Synchronous host steps: drop-fields, merge-key-value, unwrap-key-value, cast, flatten,
drop, compute.  Asynchronous steps (return a Future): compute-ai-embeddings (batched
through OrderedAsyncBatchExecutor onto the GPU encoder), query (datasource),
ai-chat-completions / ai-text-completions (GPU LLM engine; streamed chunks are written
to ``stream-to-topic`` with stream-id / stream-index / stream-last-message).
Every step honours ``when`` (JSTL predicate; false -> the record passes unchanged).
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
from concurrent.futures import Future
from typing import Any, Callable, Dict, List, Optional

from ...api.util import java_hash, OrderedAsyncBatchExecutor
from ...api import temporal as _temporal
from ...api.types import Float32, Int8, Int16, Int32
from .el import eval_expression, eval_predicate
from .mustache import compile_template
from ...api.avro import AvroRecord
from .mutable import MutableRecord

log = logging.getLogger(__name__)


def _done(v=None) -> Future:
    f: Future = Future()
    f.set_result(v)
    return f


class Step:
    is_async = False

    def __init__(self, cfg: Dict[str, Any]):
        self.cfg = cfg
        self.when = cfg.get("when")

    def applies(self, rec: MutableRecord) -> bool:
        return eval_predicate(self.when, rec.el_context()) if self.when else True

    def start(self) -> None:
        pass

    def close(self) -> None:
        pass

    def process(self, rec: MutableRecord) -> None:
        raise NotImplementedError

    def process_async(self, rec: MutableRecord) -> Future:
        try:
            self.process(rec)
            return _done()
        except Exception as e:  # noqa: BLE001
            f: Future = Future()
            f.set_exception(e)
            return f


# ---------------------------------------------------------------- host transforms
def _check_part(cfg) -> None:
    """``part``: absent / null, ``key`` or ``value`` (TransformFunctionUtil's step configs)."""
    if cfg.get("part") not in (None, "key", "value"):
        raise ValueError(f"Invalid part {cfg.get('part')!r}: expected key or value")


class DropFieldsStep(Step):
    def __init__(self, cfg):
        super().__init__(cfg)
        fields = cfg.get("fields")
        if not isinstance(fields, list) or not fields or not all(isinstance(f, str) and f for f in fields):
            raise ValueError("drop-fields needs a non-empty list of non-empty field names")
        _check_part(cfg)

    def process(self, rec):
        fields = self.cfg.get("fields") or []
        part = self.cfg.get("part")
        for target in (("value",) if part == "value" else ("key",) if part == "key" else ("key", "value")):
            obj = getattr(rec, target)
            if isinstance(obj, dict):
                for f in fields:
                    obj.pop(f, None)


class MergeKeyValueStep(Step):
    """MergeKeyValueStep.java: the key's fields are added to the value where the value has
    no field of that name (``putIfAbsent``: the value's fields first, in their order)."""

    def process(self, rec):
        if isinstance(rec.key, dict) and isinstance(rec.value, dict):
            merged = dict(rec.value)
            for k, v in rec.key.items():
                merged.setdefault(k, v)
            rec.value = merged


class UnwrapKeyValueStep(Step):
    """UnwrapKeyValueStep.java: a record with a key becomes its value (or, with
    ``unwrapKey``, its key) alone; a record without a key is untouched."""

    def process(self, rec):
        if rec.key is None:
            return
        if bool(self.cfg.get("unwrapKey", self.cfg.get("unwrap-key", False))):
            rec.value = rec.key
        rec.key = None


_CASTS: Dict[str, Callable[[Any], Any]] = {
    "string": lambda v: v if isinstance(v, str) else (json.dumps(v) if isinstance(v, (dict, list)) else (
        "true" if v is True else "false" if v is False else str(v))),
    "boolean": lambda v: v if isinstance(v, bool) else str(v).strip().lower() == "true",
    "int8": lambda v: Int8(int(float(v))), "int16": lambda v: Int16(int(float(v))),
    "int32": lambda v: Int32(int(float(v))),
    "int64": lambda v: int(float(v)), "float": lambda v: Float32(float(v)), "double": lambda v: float(v),
    "bytes": lambda v: v if isinstance(v, bytes) else str(v).encode(),
}


# cast's schema types (config-schema.yaml Cast.schema-type) -> JstlTypeConverter targets
_CAST_TYPES = ("bytes", "string", "int8", "int16", "int32", "int64", "float", "double", "boolean", "date",
               "timestamp", "time", "local_date_time", "local_date", "local_time", "instant")


def _cast_value(v, st: str):
    """CastStep.convertValue: JstlTypeConverter.coerceToType to the schema type's Java
    class (api/temporal.py); a struct value cast to STRING is its JSON text: an Avro
    record as GenericRecord.toString prints it (``{"a": 1, "b": 2}``, CastStepTest), a
    map as Jackson writes it (compact, TransformFunctionTest.testMixedPredicate)."""
    if st == "string" and isinstance(v, (dict, list)):
        if isinstance(v, AvroRecord):
            return json.dumps(v)
        return json.dumps(v, separators=(",", ":"), ensure_ascii=False)
    return _temporal.coerce(v, st)


class CastStep(Step):
    def __init__(self, cfg):
        super().__init__(cfg)
        st = cfg.get("schema-type", "string")
        if not isinstance(st, str) or st.strip().lower().replace("-", "_") not in _CAST_TYPES:
            raise ValueError(f"Unsupported schema-type {st!r}")
        _check_part(cfg)

    def process(self, rec):
        st = str(self.cfg.get("schema-type", "string")).strip().lower().replace("-", "_")
        if st not in _CAST_TYPES:
            raise ValueError(f"Unsupported schema-type {st}")

        def fn(v, st=st):
            return _cast_value(v, st)
        part = self.cfg.get("part")
        if part in (None, "key") and rec.key is not None:
            rec.key = fn(rec.key)
        if part in (None, "value") and rec.value is not None:
            rec.value = fn(rec.value)


def _flatten(d: dict, delim: str, prefix: str = "") -> dict:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{delim}{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(_flatten(v, delim, key))
        else:
            out[key] = v
    return out


class FlattenStep(Step):
    """FlattenStep.java: nested struct fields become top-level ``a<delim>b`` fields.  The
    reference flattens Avro records only; maps (JSON values) are flattened here too.  A
    value with no struct to flatten fails as there (``Unsupported schema type``)."""

    def __init__(self, cfg):
        super().__init__(cfg)
        if cfg.get("part") not in (None, "key", "value"):
            raise ValueError(f"Unsupported part for Flatten: {cfg.get('part')}")

    def process(self, rec):
        delim = self.cfg.get("delimiter", "_")
        part = self.cfg.get("part")
        if part not in (None, "key", "value"):
            raise ValueError(f"Unsupported part for Flatten: {part}")
        if part in (None, "key") and isinstance(rec.key, dict):
            rec.key = _flatten(rec.key, delim)
        if part in (None, "value"):
            if rec.value is None:
                raise ValueError("Flatten requires non-null schemas!")
            if not isinstance(rec.value, dict):
                raise ValueError(f"Unsupported schema type for Flatten: {type(rec.value).__name__}")
            rec.value = _flatten(rec.value, delim)


class DropStep(Step):
    def process(self, rec):
        rec.drop = True


# compute field type -> the Java class its expression is coerced to (ComputeField
# .getJavaType: DATE is a LocalDate, DATETIME an Instant) as a JstlTypeConverter target
_COMPUTE_TARGETS = {
    "STRING": "string", "INT8": "int8", "INT16": "int16", "INT32": "int32", "INT64": "int64", "FLOAT": "float",
    "DOUBLE": "double", "BOOLEAN": "boolean", "DATE": "local_date", "LOCAL_DATE": "local_date", "TIME": "time",
    "LOCAL_TIME": "local_time", "LOCAL_DATE_TIME": "local_date_time", "DATETIME": "instant", "INSTANT": "instant",
    "TIMESTAMP": "timestamp", "BYTES": "bytes", "DECIMAL": "big_decimal", "ARRAY": None, "MAP": None,
}
_COMPUTE_TYPES = _COMPUTE_TARGETS   # (the names a compute field may declare)


def _compute_value(v, t: Optional[str]):
    """The field's value as the JstlEvaluator typed by the field returns it."""
    if v is None or t is None:
        return v
    target = _COMPUTE_TARGETS[t]
    if target is None:
        return v
    if target == "string" and isinstance(v, (dict, list)):
        return json.dumps(v)
    return _temporal.coerce(v, target)


def _struct_value(v):
    """A computed field written into a struct (key.x / value.x): the value in its Avro
    form (ComputeStep.getAvroValue) -- Byte / Short as int, LocalDate / Date as epoch
    days (date), Time / LocalTime as millis of day (time-millis), Timestamp / Instant /
    LocalDateTime as epoch millis (timestamp-millis); other values as they are."""
    if isinstance(v, (Int8, Int16)):
        return int(v)
    if isinstance(v, _dt.date) and not isinstance(v, _dt.datetime):
        return Int32((v - _dt.date(1970, 1, 1)).days)
    if isinstance(v, _temporal.JDate):
        return Int32(v.millis // 86_400_000)
    if isinstance(v, (_temporal.Time, _temporal.LocalTime)):
        return _temporal.coerce(v, "int32")
    if isinstance(v, (_temporal.Timestamp, _temporal.Instant, _temporal.LocalDateTime, _temporal.OffsetDateTime)):
        return _temporal.coerce(v, "int64")
    return v


def compute_field_scope(scoped: str):
    """(name, scope) of a compute field (``ComputeField.java:96-121``): ``key`` / ``value``
    are the primitive scope, ``key.x`` / ``value.x`` a struct field, ``properties.x`` a
    header property, ``destinationTopic`` / ``messageKey`` (and this runtime's
    ``topicName``) a header."""
    if scoped in ("key", "value"):
        return scoped, "primitive"
    if scoped.startswith(("key.", "value.")):
        scope, name = scoped.split(".", 1)
        return name, scope
    if scoped.startswith("properties."):
        return scoped.split(".", 1)[1], "header.properties"
    if scoped in ("destinationTopic", "messageKey", "topicName"):
        return scoped, "header"
    raise ValueError(f"Invalid compute field name: {scoped}. It should be prefixed with 'key.' or 'value.' or "
                     f"'properties.' or be one of [key, value, destinationTopic, messageKey]")


class ComputeStep(Step):
    def __init__(self, cfg):
        super().__init__(cfg)
        self.fields = []
        if not cfg.get("fields"):
            raise ValueError("compute needs at least one field")
        seen = set()
        for f in cfg.get("fields"):
            name = f.get("name")
            if not name:
                raise ValueError("compute field name is required")
            compute_field_scope(name)
            if name in seen:
                raise ValueError(f"Duplicate compute field name {name}")
            seen.add(name)
            t = str(f.get("type") or "").upper() or None
            if t and t not in _COMPUTE_TYPES:
                raise ValueError(f"Unsupported compute type {t}")
            opt = f.get("optional", True)
            if not isinstance(opt, bool):
                raise ValueError(f"optional must be a boolean, got {opt!r}")
            self.fields.append((name, f.get("expression"), t, opt))

    def process(self, rec):
        ctx = rec.el_context()
        results = []
        for name, expr, t, optional in self.fields:
            v = eval_expression(expr, ctx) if expr is not None else None
            v = _compute_value(v, t)
            if v is None and not optional:
                raise ValueError(f"Field {name} is not optional but the expression evaluated to null")
            if name.startswith(("value.", "key.")):
                v = _struct_value(v)
            results.append((name, v))
        for name, v in results:
            if name in ("value", "key", "destinationTopic", "messageKey") or name.startswith(
                    ("value.", "key.", "properties.")):
                if name.startswith("value.") and not isinstance(rec.value, dict) and rec.value is not None:
                    rec.value = {}
                rec.set_result_field(v, name)
            elif name == "topicName":
                rec.input_topic = str(v)
            else:
                raise ValueError(f"Invalid compute field name {name}")


# ---------------------------------------------------------------- async AI / data steps
class _LoopOver:
    """Shared ``loop-over`` handling: process each element of a list field."""

    @staticmethod
    def items(rec: MutableRecord, field: Optional[str]):
        if not field:
            return None
        v = eval_expression(field, rec.el_context())
        if v is None:
            return []
        if not isinstance(v, list):
            raise ValueError(f"loop-over field {field} is not a list")
        return v


class ComputeAIEmbeddingsStep(Step):
    """Mustache text -> batched embeddings -> ``embeddings-field``
    (ComputeAIEmbeddingsStep.java:66-250).  Batches of ``batch-size`` are hashed by
    record key into ``concurrency`` ordered buckets; a bad record fails its batch."""
    is_async = True

    def __init__(self, cfg, service):
        super().__init__(cfg)
        self.service = service
        self.template = compile_template(cfg.get("text") or "")
        self.field = cfg.get("embeddings-field")
        if not self.field:
            raise ValueError("embeddings-field is required")
        self.loop_over = cfg.get("loop-over")
        self.executor = OrderedAsyncBatchExecutor(
            int(cfg.get("batch-size", 10)), self._process_batch, int(cfg.get("flush-interval", 0)),
            int(cfg.get("concurrency", 4)), lambda item: java_hash(item[0].key))

    def start(self):
        self.executor.start()

    def close(self):
        self.executor.stop()

    def process_async(self, rec: MutableRecord) -> Future:
        fut: Future = Future()
        try:
            items = _LoopOver.items(rec, self.loop_over)
            if items is not None:
                texts = []
                for it in items:
                    c = rec.json_context()
                    c["record"] = it
                    texts.append(self.template.render(c))
                if not texts:
                    fut.set_result(None)
                    return fut
                f2 = self.service.compute_embeddings(texts)

                def done(f):
                    try:
                        embs = f.result()
                        key = self.field.split(".")[-1] if self.field.startswith("record.") else self.field
                        # new item maps: nested objects are shared with the source record
                        new_items = [dict(it, **{key: e}) if isinstance(it, dict) else it
                                     for it, e in zip(items, embs)]
                        rec.set_result_field(new_items, self.loop_over)
                        fut.set_result(None)
                    except BaseException as ex:  # noqa: BLE001
                        fut.set_exception(ex)

                f2.add_done_callback(done)
                return fut
            text = self.template.render(rec.json_context())
        except Exception as e:  # noqa: BLE001
            fut.set_exception(e)
            return fut
        self.executor.add((rec, text, fut))
        return fut

    def bulk_ok(self) -> bool:
        return self.loop_over is None

    def process_bulk(self, pairs, emit) -> None:
        """(source record, MutableRecord) pairs -> ``emit([(source, mutable, error)])``
        once per completed embedding batch, for every pair of it that came through this
        call.  The same ordered batch executor (per-key order, batch-size, flush-interval,
        concurrency) as ``process_async``: only the completion is reported in bulk."""
        add = self.executor.add
        render = self.template.render
        for src, mr in pairs:
            try:
                text = render(mr.json_context())
            except Exception as e:  # noqa: BLE001
                emit([(src, mr, e)])
                continue
            add((mr, text, (src, emit)))

    @staticmethod
    def _complete(batch, err, set_field) -> None:
        """Resolve every item of a batch: per-record futures (process_async) and bulk
        tokens (process_bulk, one emit call per distinct emit)."""
        groups = {}
        for rec, _, tok in batch:
            e = err
            if e is None:
                try:
                    set_field(rec)
                except Exception as ex:  # noqa: BLE001
                    e = ex
            if isinstance(tok, Future):
                if e is None:
                    tok.set_result(None)
                else:
                    tok.set_exception(e)
            else:
                src, emit = tok
                g = groups.get(id(emit))
                if g is None:
                    g = groups[id(emit)] = (emit, [])
                g[1].append((src, rec, e))
        for emit, items in groups.values():
            emit(items)

    def _process_batch(self, batch, batch_fut: Future) -> None:
        texts = [t for _, t, _ in batch]
        try:
            f = self.service.compute_embeddings(texts)
        except Exception as e:  # noqa: BLE001
            self._complete(batch, e, None)
            batch_fut.set_exception(e)
            return

        def done(ff: Future):
            err = ff.exception()
            if err is not None:
                self._complete(batch, err, None)
                batch_fut.set_exception(err)
                return
            embs = iter(ff.result())
            field = self.field

            def set_field(rec):
                e = next(embs)
                rec.set_result_field(e if isinstance(e, list) else list(e), field)
            try:
                self._complete(batch, None, set_field)
            finally:
                batch_fut.set_result(None)

        f.add_done_callback(done)


class QueryStep(Step):
    """fields (JSTL) -> positional params -> datasource.fetch_data / execute_statement
    (QueryStep.java:54-222); ``loop-over``, ``only-first``, ``output-field``,
    ``mode: query|execute``, ``generated-keys``."""
    is_async = True

    def __init__(self, cfg, datasource):
        super().__init__(cfg)
        self.ds = datasource
        self.query = cfg.get("query")
        self.fields = cfg.get("fields") or []
        self.output_field = cfg.get("output-field")
        self.only_first = bool(cfg.get("only-first", False))
        self.loop_over = cfg.get("loop-over")
        self.mode = cfg.get("mode", "query")
        self.generated_keys = cfg.get("generated-keys") or []
        if self.mode not in ("query", "execute"):
            raise ValueError("mode must be query or execute")
        if not self.output_field and self.mode == "query":
            raise ValueError("output-field is required")
        self._batcher = None
        if self.mode == "query" and not self.loop_over and hasattr(self.ds, "fetch_data_batch"):
            from ...api.util import MicroBatcher
            self._batcher = MicroBatcher(lambda ps: self.ds.fetch_data_batch(self.query, ps), 64, "query-batcher")

    def _params(self, ctx) -> list:
        return [eval_expression(f, ctx) for f in self.fields]

    def _run_one(self, ctx):
        params = self._params(ctx)
        if self.mode == "execute":
            return self.ds.execute_statement(self.query, self.generated_keys, params)
        return self.ds.fetch_data(self.query, params) or []

    def _first(self, rows):
        # only-first: the first row, or an empty map when there is none (QueryStep.java:95-100)
        return (rows[0] if rows else {}) if self.only_first else rows

    def process_async(self, rec) -> Future:
        fut: Future = Future()
        if self._batcher is not None:
            try:
                inner = self._batcher.submit(self._params(rec.el_context()))
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)
                return fut

            def done(f):
                try:
                    r = self._first(f.result() or [])
                    rec.set_result_field(r, self.output_field)
                    fut.set_result(None)
                except BaseException as e:  # noqa: BLE001
                    fut.set_exception(e)

            inner.add_done_callback(done)
            return fut

        def run():
            try:
                items = _LoopOver.items(rec, self.loop_over)
                if items is not None:
                    # per item ("record" in the expressions): a query's rows are concatenated,
                    # an execute's results listed (QueryStep.processQuery / processExecute)
                    res = []
                    for it in items:
                        c = rec.el_context()
                        c["record"] = it
                        out = self._run_one(c)
                        if self.mode == "execute":
                            res.append(out)
                        else:
                            res.extend(out)
                    if self.mode != "execute":
                        res = self._first(res)
                    rec.set_result_field(res, self.output_field)
                else:
                    r = self._run_one(rec.el_context())
                    if self.mode != "execute":
                        r = self._first(r)
                    if self.output_field:
                        rec.set_result_field(r, self.output_field)
                fut.set_result(None)
            except BaseException as e:  # noqa: BLE001
                fut.set_exception(e)

        # on the agent thread, as the reference's QueryStep.process: results stay in input
        # order (JdbcDatabaseIT reads each written key back in sequence).  GPU vector
        # queries take the micro-batched path above instead.
        run()
        return fut


# The step configuration as the reference logs it (convertToMap of ChatCompletionsConfig /
# TextCompletionsConfig: every field in declaration order, unset ones as null, Integer /
# Double / boolean typed).  name -> (type, default)
CHAT_LOG_FIELDS = (("model", str, None), ("messages", list, None), ("stream-to-topic", str, None),
                   ("stream-response-completion-field", str, None), ("min-chunks-per-message", int, 20),
                   ("completion-field", str, None), ("stream", bool, True), ("log-field", str, None),
                   ("max-tokens", int, None), ("temperature", float, None), ("top-p", float, None),
                   ("logit-bias", dict, None), ("user", str, None), ("stop", list, None),
                   ("presence-penalty", float, None), ("frequency-penalty", float, None), ("options", dict, None))
TEXT_LOG_FIELDS = (("model", str, None), ("prompt", list, None), ("stream-to-topic", str, None),
                   ("stream-response-completion-field", str, None), ("min-chunks-per-message", int, 20),
                   ("completion-field", str, None), ("stream", bool, True), ("log-field", str, None),
                   ("logprobs-field", str, None), ("logprobs", float, None), ("max-tokens", int, None),
                   ("temperature", float, None), ("top-p", float, None), ("logit-bias", dict, None),
                   ("user", str, None), ("stop", list, None), ("presence-penalty", float, None),
                   ("frequency-penalty", float, None), ("options", dict, None))


def log_options(cfg: Dict[str, Any], fields, step_type: str) -> Dict[str, Any]:
    out: Dict[str, Any] = {"type": cfg.get("type", step_type), "when": cfg.get("when")}
    for name, typ, dflt in fields:
        v = cfg.get(name, dflt)
        if typ is bool and isinstance(v, str):
            v = v.strip().lower() == "true"
        elif v is not None and typ in (int, float, bool) and not isinstance(v, typ):
            v = typ(v)
        elif v is not None and typ is float:
            v = float(v)
        if name == "messages" and v is not None:
            v = [{"role": m.get("role"), "content": m.get("content")} for m in v]
        out[name] = v
    return out


class ChatCompletionsStep(Step):
    """ai-chat-completions (ChatCompletionsStep.java:77-196)."""
    is_async = True

    def __init__(self, cfg, service, stream_consumer_factory):
        super().__init__(cfg)
        self.service = service
        self.messages = [(m.get("role", "user"), compile_template(m.get("content") or ""))
                         for m in cfg.get("messages") or []]
        if not self.messages:
            raise ValueError("messages is required")
        self.field = cfg.get("completion-field")
        self.stream_field = cfg.get("stream-response-completion-field")
        self.log_field = cfg.get("log-field")
        self.stream_to = cfg.get("stream-to-topic")
        self.factory = stream_consumer_factory
        self.stream_consumer = None
        self.options = {k: cfg.get(k) for k in ("model", "max-tokens", "temperature", "top-p", "logit-bias", "user",
                                                 "stop", "presence-penalty", "frequency-penalty", "seed", "top-k",
                                                 "ignore-eos") if cfg.get(k) is not None}
        self.options.update(cfg.get("options") or {})
        self.options["min-chunks-per-message"] = int(cfg.get("min-chunks-per-message", 20))
        self.options["stream"] = bool(cfg.get("stream", True))
        self.log_options = log_options(cfg, CHAT_LOG_FIELDS, "ai-chat-completions")

    def start(self):
        if self.stream_to:
            self.stream_consumer = self.factory(self.stream_to)

    def close(self):
        if self.stream_consumer is not None:
            self.stream_consumer.close()

    def _apply(self, rec: MutableRecord, content: str, streaming: bool) -> None:
        field = self.field
        if streaming and self.stream_field:
            field = self.stream_field
        rec.set_result_field(content, field)

    def _chunk_consumer(self, rec):
        if self.stream_consumer is None:
            return None

        def consume(answer_id, index, content, last):
            c = rec.shallow_copy()
            c.properties["stream-id"] = answer_id
            c.properties["stream-index"] = str(index)
            c.properties["stream-last-message"] = "true" if last else "false"
            self._apply(c, content, True)
            self.stream_consumer.stream_answer_chunk(index, content, last, c)

        return consume

    def _render_messages(self, rec):
        from .services import ChatMessage
        ctx = rec.json_context()
        return [ChatMessage(role, t.render(ctx)) for role, t in self.messages]

    def process_async(self, rec) -> Future:
        fut: Future = Future()
        try:
            messages = self._render_messages(rec)
            inner = self.service.get_chat_completions(messages, self._chunk_consumer(rec), dict(self.options))
        except Exception as e:  # noqa: BLE001
            fut.set_exception(e)
            return fut

        def done(f):
            try:
                res = f.result()
                self._apply(rec, res.content, False)
                if self.log_field:
                    # ChatCompletionsStep.java:162-170: {options: the step config (every
                    # field, nulls included), messages: the rendered messages, model}
                    rec.set_result_field(json.dumps({"options": self.log_options, "messages": [m.to_dict() for m in messages],
                                                     "model": self.log_options.get("model")}, separators=(",", ":")),
                                         self.log_field)
                fut.set_result(None)
            except BaseException as e:  # noqa: BLE001
                fut.set_exception(e)

        inner.add_done_callback(done)
        return fut


class TextCompletionsStep(ChatCompletionsStep):
    """ai-text-completions (TextCompletionsStep.java:95-199): prompt[] templates,
    ``logprobs`` + ``logprobs-field = {tokens[], logprobs[]}`` (consumed by FLARE)."""

    def __init__(self, cfg, service, stream_consumer_factory):
        cfg = dict(cfg)
        cfg.setdefault("messages", [{"role": "user", "content": p} for p in (cfg.get("prompt") or [])])
        Step.__init__(self, cfg)
        self.service = service
        self.prompts = [compile_template(p) for p in cfg.get("prompt") or []]
        if not self.prompts:
            raise ValueError("prompt is required")
        self.field = cfg.get("completion-field")
        self.stream_field = cfg.get("stream-response-completion-field")
        self.log_field = cfg.get("log-field")
        self.stream_to = cfg.get("stream-to-topic")
        self.factory = stream_consumer_factory
        self.stream_consumer = None
        self.logprobs_field = cfg.get("logprobs-field")
        self.options = {k: cfg.get(k) for k in ("model", "max-tokens", "temperature", "top-p", "logit-bias", "user",
                                                 "stop", "presence-penalty", "frequency-penalty", "logprobs", "seed",
                                                 "top-k", "ignore-eos") if cfg.get(k) is not None}
        self.options.update(cfg.get("options") or {})
        self.options["min-chunks-per-message"] = int(cfg.get("min-chunks-per-message", 20))
        self.options["stream"] = bool(cfg.get("stream", True))
        self.log_options = log_options(cfg, TEXT_LOG_FIELDS, "ai-text-completions")

    def process_async(self, rec) -> Future:
        fut: Future = Future()
        try:
            ctx = rec.json_context()
            prompts = [t.render(ctx) for t in self.prompts]
            inner = self.service.get_text_completions(prompts, self._chunk_consumer(rec), dict(self.options))
        except Exception as e:  # noqa: BLE001
            fut.set_exception(e)
            return fut

        def done(f):
            try:
                res = f.result()
                self._apply(rec, res.content, False)
                if self.logprobs_field:
                    rec.set_result_field({"tokens": res.tokens, "logprobs": res.logprobs}, self.logprobs_field)
                if self.log_field:
                    rec.set_result_field(json.dumps({"options": self.log_options, "messages": prompts,
                                                     "model": self.log_options.get("model")}, separators=(",", ":")),
                                         self.log_field)
                fut.set_result(None)
            except BaseException as e:  # noqa: BLE001
                fut.set_exception(e)

        inner.add_done_callback(done)
        return fut
