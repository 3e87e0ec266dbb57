"""HTTP agents: ``http-request`` and ``langserve-invoke``.

Parity:
* http-request (``HttpRequestAgent.java:60-234``): required ``url`` and ``output-field``;
  ``method`` (GET), ``headers`` / ``query-string`` / ``body`` are Mustache templates over
  the JSON record, ``allow-redirects`` (true), ``handle-cookies`` (true).  Status >= 400
  is an error; the body is parsed as a JSON map when possible, else kept as text.
* langserve-invoke (``LangServeInvokeAgent.java:40-255``, ``LangServeClient.java``):
  body ``{"input": {<fields>}}`` where each field is an EL expression; URL ending in
  ``/invoke`` -> one POST, result ``output`` (or ``output[content-field]``); URL ending
  in ``/stream`` -> server-sent events, ``event: data`` lines carry chunks that are
  coalesced 1, 2, 4, ... up to ``min-chunks-per-message`` and written to
  ``stream-to-topic`` with ``stream-id`` / ``stream-index`` / ``stream-last-message``
  headers; ``event: end`` closes the answer.  Any other URL is rejected.

Requests run on a small thread pool so a slow endpoint never blocks the agent loop;
results are emitted asynchronously (the runner keeps commits ordered).
"""
from __future__ import annotations

import json
import logging
import urllib.parse
import uuid
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Callable, Dict, List, Optional

from ..api.agent import AgentProcessor
from ..api.record import SourceRecordAndResult
from ..api.util import get_boolean, get_int, get_map, get_string, required_non_empty_field
from ..runtime.registry import register_agent
from .genai.el import eval_expression
from .genai.mustache import compile_template
from .genai.mutable import MutableRecord

log = logging.getLogger(__name__)


def _session(allow_redirects: bool, handle_cookies: bool):
    import requests
    s = requests.Session()
    s.max_redirects = 30 if allow_redirects else 0
    if not handle_cookies:
        from http.cookiejar import DefaultCookiePolicy
        s.cookies.set_policy(DefaultCookiePolicy(allowed_domains=[]))
    return s


def _parse_body(text: str) -> Any:
    try:
        v = json.loads(text)
        if isinstance(v, dict):
            return v
    except ValueError:
        pass
    return text


@register_agent("http-request")
class HttpRequestAgent(AgentProcessor):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.url = required_non_empty_field(configuration, "url", "http-request agent")
        self.output_field = required_non_empty_field(configuration, "output-field", "http-request agent")
        self.method = get_string("method", "GET", configuration).upper()
        body = get_string("body", None, configuration)
        self.body_t = compile_template(body) if body is not None else None
        self.header_t = {k: compile_template(str(v)) for k, v in get_map("headers", {}, configuration).items()}
        self.query_t = {k: compile_template(str(v)) for k, v in get_map("query-string", {}, configuration).items()}
        self.allow_redirects = get_boolean("allow-redirects", True, configuration)
        self.handle_cookies = get_boolean("handle-cookies", True, configuration)
        self.pool: Optional[ThreadPoolExecutor] = None
        self.http = None

    def start(self) -> None:
        self.pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix=f"agent-{self.agent_id()}-http")
        self.http = _session(self.allow_redirects, self.handle_cookies)

    def close(self) -> None:
        if self.pool is not None:
            self.pool.shutdown(wait=False, cancel_futures=True)

    def process(self, records, sink) -> None:
        if self.pool is None:
            self.start()
        for r in records:
            self._one(r, sink)

    def _one(self, record, sink) -> None:
        try:
            mr = MutableRecord.from_record(record)
            ctx = mr.json_context()
            url = self.url
            if self.query_t:
                url += "?" + "&".join(f"{k}={urllib.parse.quote_plus(t.render(ctx))}" for k, t in self.query_t.items())
            headers = {k: t.render(ctx) for k, t in self.header_t.items()}
            data = self.body_t.render(ctx).encode() if self.body_t is not None else None
        except Exception as e:  # noqa: BLE001
            sink(SourceRecordAndResult(record, None, e))
            return

        def call():
            try:
                resp = self.http.request(self.method, url, headers=headers, data=data,
                                         allow_redirects=self.allow_redirects, timeout=120)
                if resp.status_code >= 400:
                    raise RuntimeError(f"Error processing record: {record} with response: {resp.status_code} "
                                       f"{resp.text[:200]}")
                mr.set_result_field(_parse_body(resp.text), self.output_field)
                out = mr.to_record()
                self.processed(1, 1 if out is not None else 0)
                sink(SourceRecordAndResult(record, [out] if out is not None else [], None))
            except Exception as e:  # noqa: BLE001
                log.error("http-request failed for %s: %s", record, e)
                sink(SourceRecordAndResult(record, None, e))

        self.pool.submit(call)


class _ChunkWriter:
    """Coalesce streamed chunks 1, 2, 4, ... up to ``min_chunks`` per message."""

    def __init__(self, min_chunks: int, emit: Callable[[str, int, str, bool], None]):
        self.min_chunks = max(1, min_chunks)
        self.emit = emit
        self.current = 1
        self.buf: List[str] = []
        self.total: List[str] = []
        self.index = 0
        self.answer_id = str(uuid.uuid4())

    def add(self, content: str, last: bool) -> None:
        if content:
            self.buf.append(content)
            self.total.append(content)
        if len(self.buf) >= self.current or last:
            self.current = min(self.current * 2, self.min_chunks)
            self.index += 1
            self.emit(self.answer_id, self.index, "".join(self.buf), last)
            self.buf.clear()

    @property
    def answer(self) -> str:
        return "".join(self.total)


@register_agent("langserve-invoke")
class LangServeInvokeAgent(AgentProcessor):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.url = required_non_empty_field(configuration, "url", "langserve-invoke agent")
        self.output_field = required_non_empty_field(configuration, "output-field", "langserve-invoke agent")
        self.stream_to_topic = get_string("stream-to-topic", "", configuration)
        self.stream_field = get_string("stream-response-field", self.output_field, configuration)
        self.min_chunks = get_int("min-chunks-per-message", 20, configuration)
        self.content_field = get_string("content-field", "content", configuration)
        self.debug = get_boolean("debug", False, configuration)
        self.method = get_string("method", "POST", configuration).upper()
        self.fields = [(get_string("name", "", f), get_string("expression", "", f))
                       for f in configuration.get("fields") or []]
        self.header_t = {k: compile_template(str(v)) for k, v in get_map("headers", {}, configuration).items()}
        self.allow_redirects = get_boolean("allow-redirects", True, configuration)
        self.handle_cookies = get_boolean("handle-cookies", True, configuration)
        if not (self.url.endswith("/invoke") or self.url.endswith("/stream")):
            log.warning("langserve-invoke url %s ends neither in /invoke nor /stream", self.url)
        self.pool = None
        self.http = None
        self.producer = None

    def start(self) -> None:
        self.pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix=f"agent-{self.agent_id()}-langserve")
        self.http = _session(self.allow_redirects, self.handle_cookies)
        if self.stream_to_topic:
            prov = self.context.topic_connection_provider
            self.producer = prov.create_producer(self.context.global_agent_id, self.stream_to_topic)
            self.producer.start()

    def close(self) -> None:
        if self.producer is not None:
            self.producer.close()
            self.producer = None
        if self.pool is not None:
            self.pool.shutdown(wait=False, cancel_futures=True)

    def process(self, records, sink) -> None:
        if self.pool is None:
            self.start()
        for r in records:
            self._one(r, sink)

    def _content(self, body: str, streaming: bool) -> Any:
        if body is None:
            return ""
        try:
            if body.startswith("{"):
                m = json.loads(body)
                if not streaming:
                    out = m.get("output")
                    if out is None or isinstance(out, str):
                        return out
                    if isinstance(out, dict):
                        m = out
                return m if not self.content_field else m.get(self.content_field)
            if body.startswith('"'):
                return json.loads(body)
        except ValueError:
            log.info("Not able to parse response to json: %s", body)
        return body

    def _one(self, record, sink) -> None:
        try:
            mr = MutableRecord.from_record(record)
            el = mr.el_context()
            body = json.dumps({"input": {n: eval_expression(e, el) for n, e in self.fields}}, separators=(",", ":"),
                              ensure_ascii=False, default=str)
            jctx = mr.json_context()
            headers = {"Content-Type": "application/json"}
            headers.update({k: t.render(jctx) for k, t in self.header_t.items()})
            if not (self.url.endswith("/invoke") or self.url.endswith("/stream")):
                raise ValueError(f"Unsupported url: {self.url}")
        except Exception as e:  # noqa: BLE001
            sink(SourceRecordAndResult(record, None, e))
            return

        def emit_chunk(answer_id, index, chunk, last):
            if self.producer is None:
                return
            c = mr.shallow_copy()
            c.set_result_field(chunk, self.stream_field)
            c.properties["stream-id"] = answer_id
            c.properties["stream-index"] = str(index)
            c.properties["stream-last-message"] = "true" if last else "false"
            r = c.to_record()
            if r is not None:
                self.producer.write(r)

        def call():
            try:
                if self.url.endswith("/invoke"):
                    resp = self.http.request(self.method, self.url, data=body, headers=headers, timeout=300)
                    if resp.status_code >= 400:
                        raise RuntimeError(f"Error processing, http response: {resp.status_code}")
                    result = self._content(resp.text, False)
                    result = "" if result is None else str(result)
                else:
                    w = _ChunkWriter(self.min_chunks, emit_chunk)
                    done = False
                    with self.http.request(self.method, self.url, data=body, headers=headers, stream=True,
                                           timeout=300) as resp:
                        if resp.status_code >= 400:
                            raise RuntimeError(f"Error processing, http response: {resp.status_code}")
                        for line in resp.iter_lines(decode_unicode=True):
                            if line is None:
                                continue
                            if line.startswith("event: end"):
                                w.add("", True)
                                done = True
                                break
                            if line.startswith("data: "):
                                c = self._content(line[len("data: "):], True)
                                w.add("" if c is None else str(c), False)
                    if not done:
                        w.add("", True)
                    result = w.answer
                out_rec = mr.shallow_copy()
                out_rec.set_result_field(result, self.output_field)
                out = out_rec.to_record()
                self.processed(1, 1)
                sink(SourceRecordAndResult(record, [out] if out is not None else [], None))
            except Exception as e:  # noqa: BLE001
                log.error("langserve-invoke failed: %s", e)
                sink(SourceRecordAndResult(record, None, e))

        self.pool.submit(call)
