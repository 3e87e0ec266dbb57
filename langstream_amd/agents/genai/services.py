"""AI service providers for the GenAI toolkit.

Parity: AIA/ai/langstream/ai/agents/services/ServiceProviderRegistry.java:49-67 (dispatch on
the config key), OpenAICompletionService.java:122-498 (chat/text completions, streaming
chunk coalescing :256-306, embeddings), OllamaProvider.java:165-328, HuggingFaceProvider.java,
VertexAIProvider.java, BedrockServiceProvider.java.

MI355X-native: the ``local`` key (``local-gpu-configuration`` resource) binds the
in-process GPU engines (``engine/llm_engine.py``, ``engine/embedder.py``); remote
providers stay available over HTTP for parity (they need network access).
"""
from __future__ import annotations

import json
import logging
import threading
import urllib.parse
import uuid
from concurrent.futures import Future
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

log = logging.getLogger(__name__)

ChunkConsumer = Callable[[str, int, str, bool], None]  # (answer_id, index, content, last)


@dataclass
class ChatMessage:
    role: str
    content: str

    def to_dict(self) -> dict:
        return {"role": self.role, "content": self.content}


@dataclass
class CompletionResult:
    content: str
    answer_id: str = ""
    finish_reason: Optional[str] = None
    tokens: List[str] = field(default_factory=list)
    logprobs: List[float] = field(default_factory=list)
    prompt_tokens: int = 0
    completion_tokens: int = 0


class ChunkCoalescer:
    """Start at 1 chunk per message, double up to ``min_chunks_per_message``: low latency
    for the first message, fewer topic messages afterwards (OpenAICompletionService.java:256-306)."""

    def __init__(self, consumer: Optional[ChunkConsumer], min_chunks_per_message: int, answer_id: str):
        self.consumer = consumer
        self.min_chunks = max(1, int(min_chunks_per_message or 1))
        self.answer_id = answer_id
        self.current = 1
        self.buffer: List[str] = []
        self.n = 0
        self.index = 0
        self.lock = threading.Lock()

    def accept(self, delta: str, last: bool) -> None:
        with self.lock:
            if delta:
                self.buffer.append(delta)
                self.n += 1
            if self.n >= self.current or last:
                self.current = min(self.current * 2, self.min_chunks)
                text = "".join(self.buffer)
                self.buffer.clear()
                self.n = 0
                self.index += 1
                idx = self.index
            else:
                return
        if self.consumer is not None:
            self.consumer(self.answer_id, idx, text, last)


class CompletionsService:
    def get_chat_completions(self, messages: List[ChatMessage], consumer: Optional[ChunkConsumer],
                             options: Dict[str, Any]) -> Future:
        raise NotImplementedError

    def get_text_completions(self, prompts: List[str], consumer: Optional[ChunkConsumer],
                             options: Dict[str, Any]) -> Future:
        raise NotImplementedError


class EmbeddingsService:
    def compute_embeddings(self, texts: List[str]) -> Future:
        raise NotImplementedError


# ---------------------------------------------------------------- local GPU
def llama3_chat_prompt(messages: List[ChatMessage]) -> str:
    out = ["<|begin_of_text|>"]
    for m in messages:
        out.append(f"<|start_header_id|>{m.role}<|end_header_id|>\n\n{m.content}<|eot_id|>")
    out.append("<|start_header_id|>assistant<|end_header_id|>\n\n")
    return "".join(out)


def _sampling_from_options(options: Dict[str, Any], tok):
    from ...engine.llm_engine import SamplingParams
    stop = options.get("stop") or []
    if isinstance(stop, str):
        stop = [stop]
    lb = options.get("logit-bias") or options.get("logit_bias")
    temperature = options.get("temperature")
    return SamplingParams(
        max_tokens=int(options.get("max-tokens") or options.get("max_tokens") or 256),
        temperature=1.0 if temperature is None else float(temperature),
        top_p=float(options.get("top-p") or options.get("top_p") or 1.0),
        top_k=int(options.get("top-k") or options.get("top_k") or 0),
        seed=options.get("seed"),
        stop=list(stop),
        presence_penalty=float(options.get("presence-penalty") or 0.0),
        frequency_penalty=float(options.get("frequency-penalty") or 0.0),
        logit_bias={int(k): float(v) for k, v in lb.items()} if isinstance(lb, dict) else None,
        logprobs=int(options.get("logprobs") or 0) if options.get("logprobs") not in (True, False) else (
            1 if options.get("logprobs") else 0),
        ignore_eos=bool(options.get("ignore-eos", False)),
    )


class LocalCompletionsService(CompletionsService):
    """Chat / text completions on the in-process continuous-batching GPU engine."""

    def __init__(self, engine, tokenizer, model_name: str = "local"):
        self.engine = engine
        self.tok = tokenizer
        self.model_name = model_name

    def _submit(self, prompt_text: str, consumer, options, want_logprobs: bool) -> Future:
        fut: Future = Future()
        answer_id = f"chatcmpl-{uuid.uuid4().hex[:24]}"
        coalescer = ChunkCoalescer(consumer, int(options.get("min-chunks-per-message", 20)), answer_id)
        stream = bool(options.get("stream", True)) and consumer is not None
        params = _sampling_from_options(options, self.tok)
        if want_logprobs and params.logprobs == 0:
            params.logprobs = 1
        ids = self.tok.encode(prompt_text, add_bos=False)
        toks: List[str] = []
        lps: List[float] = []

        def on_token(ev) -> None:
            if ev.token_id >= 0:
                if want_logprobs:
                    toks.append(self.tok.decode([ev.token_id]))
                    lps.append(ev.logprob)
                if stream:
                    coalescer.accept(ev.text, ev.finished)
            elif stream and ev.finished:
                coalescer.accept("", True)
            if ev.finished:
                req = holder.get("req")
                text = req.text if req is not None else ""
                if ev.finish_reason == "error":
                    fut.set_exception(RuntimeError("generation failed"))
                else:
                    fut.set_result(CompletionResult(text, answer_id, ev.finish_reason, toks, lps,
                                                    len(ids), len(req.output_ids) if req else 0))

        holder: Dict[str, Any] = {}
        holder["req"] = self.engine.submit(ids, params, on_token)
        return fut

    def get_chat_completions(self, messages, consumer, options) -> Future:
        return self._submit(llama3_chat_prompt(messages), consumer, options, False)

    def get_text_completions(self, prompts, consumer, options) -> Future:
        return self._submit("\n".join(prompts), consumer, options, bool(options.get("logprobs")))


class LocalEmbeddingsService(EmbeddingsService):
    def __init__(self, engine):
        self.engine = engine

    def compute_embeddings(self, texts: List[str]) -> Future:
        return self.engine.embed_async(texts)


# ---------------------------------------------------------------- remote (HTTP) providers
def _http_json(url: str, payload: dict, headers: Dict[str, str], timeout: float = 120.0) -> dict:
    import requests
    r = requests.post(url, json=payload, headers=headers, timeout=timeout)
    r.raise_for_status()
    return r.json()


def _run_async(fn) -> Future:
    fut: Future = Future()

    def run():
        try:
            fut.set_result(fn())
        except BaseException as e:  # noqa: BLE001
            fut.set_exception(e)

    threading.Thread(target=run, daemon=True).start()
    return fut


class OpenAIService(CompletionsService, EmbeddingsService):
    """OpenAI / Azure OpenAI REST with the reference client's wire behaviour
    (``TransformFunctionUtil.java:95-135`` builds the Azure OpenAI SDK client;
    ``OpenAICompletionService.java:122-498`` streams):

    * with a ``url`` the deployment route ``{url}/openai/deployments/{model}/{op}
      ?api-version=2023-08-01-preview`` is used whatever the provider (``azure`` sends the
      key as ``api-key``, ``openai`` as a bearer token) and the body carries no model;
      without one, ``https://api.openai.com/v1/{op}`` with ``model`` in the body;
    * request bodies list only the options that are set, in the SDK's field order;
    * streamed chat: role-only deltas are not chunks, chunks coalesce 1, 2, 4 ... up to
      ``min-chunks-per-message`` and carry the stream's own completion id;
    * streamed text completions: a blank first chunk is dropped (some models open with
      line breaks), every other chunk -- empty ones included -- counts, and the logprobs
      of the kept chunks are collected ({tokens[], logprobs[]}).
    """

    API_VERSION = "2023-08-01-preview"

    def __init__(self, cfg: Dict[str, Any], model: Optional[str] = None):
        self.cfg = cfg
        self.model = model
        self.url = (cfg.get("url") or "").rstrip("/")
        self.key = cfg.get("access-key")
        self.provider = cfg.get("provider", "openai")

    def _headers(self):
        if self.provider == "azure":
            return {"api-key": self.key or ""}
        return {"Authorization": f"Bearer {self.key}"}

    def _endpoint(self, kind: str, model: str) -> str:
        if self.url:
            return f"{self.url}/openai/deployments/{model}/{kind}?api-version={self.API_VERSION}"
        return f"https://api.openai.com/v1/{kind}"

    def _body(self, first: Dict[str, Any], options: Dict[str, Any], fields, model: str, stream: bool):
        body = dict(first)
        conv = {"max-tokens": int, "temperature": float, "top-p": float, "presence-penalty": float,
                "frequency-penalty": float, "logprobs": int}
        for k in fields:
            v = options.get(k)
            if v is None:
                continue
            body[k.replace("-", "_")] = conv[k](v) if k in conv else v
        if stream:
            body["stream"] = True
        if not self.url:
            body["model"] = model
        return body

    def _post(self, url: str, body: Dict[str, Any], stream: bool):
        import requests
        data = json.dumps(body, separators=(",", ":"))
        r = requests.post(url, data=data.encode(), headers={**self._headers(), "Content-Type": "application/json"},
                          stream=stream, timeout=300)
        r.raise_for_status()
        return r

    @staticmethod
    def _events(r):
        for line in r.iter_lines():
            if not line or not line.startswith(b"data:"):
                continue
            data = line[5:].strip()
            if data == b"[DONE]":
                return
            yield json.loads(data)

    def compute_embeddings(self, texts):
        model = self.model or "text-embedding-ada-002"
        # the SDK keeps the response's list order (it does not re-sort by "index")
        return _run_async(lambda: [d["embedding"] for d in self._post(
            self._endpoint("embeddings", model), self._body({"input": list(texts)}, {}, (), model, False),
            False).json()["data"]])

    CHAT_FIELDS = ("max-tokens", "temperature", "top-p", "logit-bias", "user", "stop", "presence-penalty",
                   "frequency-penalty")
    TEXT_FIELDS = ("max-tokens", "temperature", "top-p", "logit-bias", "user", "logprobs", "stop",
                   "presence-penalty", "frequency-penalty")

    def get_chat_completions(self, messages, consumer, options):
        model = options.get("model") or self.model
        stream = bool(options.get("stream", True))

        def run():
            body = self._body({"messages": [m.to_dict() for m in messages]}, options, self.CHAT_FIELDS, model, stream)
            r = self._post(self._endpoint("chat/completions", model), body, stream)
            if not stream:
                res = r.json()
                ch = res["choices"][0]
                return CompletionResult((ch.get("message") or {}).get("content") or "", res.get("id", ""),
                                        ch.get("finish_reason"))
            co, parts, aid, reason = None, [], "", None
            with r:
                for ev in self._events(r):
                    choices = ev.get("choices") or []
                    if not choices:
                        continue
                    aid = ev.get("id") or aid
                    if co is None:
                        co = ChunkCoalescer(consumer, int(options.get("min-chunks-per-message", 20)), aid)
                    ch = choices[0]
                    d = (ch.get("delta") or {}).get("content") or ""
                    parts.append(d)
                    reason = ch.get("finish_reason") or reason
                    co.accept(d, ch.get("finish_reason") is not None)
            return CompletionResult("".join(parts), aid, reason)

        return _run_async(run)

    def get_text_completions(self, prompts, consumer, options):
        model = options.get("model") or self.model
        stream = bool(options.get("stream", True))

        def run():
            body = self._body({"prompt": list(prompts)}, options, self.TEXT_FIELDS, model, stream)
            r = self._post(self._endpoint("completions", model), body, stream)
            if not stream:
                res = r.json()
                ch = res["choices"][0]
                lp = ch.get("logprobs") or {}
                return CompletionResult(ch.get("text", ""), res.get("id", ""), ch.get("finish_reason"),
                                        lp.get("tokens") or [], lp.get("token_logprobs") or [])
            minc = max(1, int(options.get("min-chunks-per-message", 20)))
            state = {"first": True, "cur": 1, "n": 0, "idx": 0, "buf": [], "total": [], "toks": [], "lps": []}
            aid, reason = "", None
            with r:
                for ev in self._events(r):
                    choices = ev.get("choices") or []
                    if not choices:
                        continue
                    aid = ev.get("id") or aid
                    ch = choices[0]
                    last = ch.get("finish_reason") is not None
                    reason = ch.get("finish_reason") or reason
                    content = ch.get("text")
                    if content is None:
                        continue
                    if state["first"]:
                        state["first"] = False
                        if not content.strip():
                            continue
                    state["buf"].append(content)
                    state["total"].append(content)
                    lp = ch.get("logprobs") or {}
                    state["toks"] += lp.get("tokens") or []
                    state["lps"] += lp.get("token_logprobs") or []
                    state["n"] += 1
                    if state["n"] >= state["cur"] or last:
                        state["cur"] = min(state["cur"] * 2, minc)
                        state["idx"] += 1
                        text = "".join(state["buf"])
                        state["buf"].clear()
                        state["n"] = 0
                        if consumer is not None:
                            consumer(aid, state["idx"], text, last)
            return CompletionResult("".join(state["total"]), aid, reason, state["toks"], state["lps"])

        return _run_async(run)


class OllamaService(CompletionsService, EmbeddingsService):
    """Ollama: /api/generate line-JSON stream (messages joined into one prompt),
    /api/embeddings one request per text (OllamaProvider.java:165-328)."""

    def __init__(self, cfg: Dict[str, Any], model: Optional[str] = None):
        self.url = cfg.get("url", "http://localhost:11434").rstrip("/")
        self.model = model

    def compute_embeddings(self, texts):
        return _run_async(lambda: [_http_json(f"{self.url}/api/embeddings", {"model": self.model, "prompt": t},
                                              {})["embedding"] for t in texts])

    def _generate(self, prompt, consumer, options):
        def run():
            import requests
            aid = f"ollama-{uuid.uuid4().hex[:16]}"
            co = ChunkCoalescer(consumer, int(options.get("min-chunks-per-message", 20)), aid)
            parts = []
            with requests.post(f"{self.url}/api/generate", json={"model": options.get("model") or self.model,
                                                                  "prompt": prompt, "stream": True},
                               stream=True, timeout=300) as r:
                r.raise_for_status()
                for line in r.iter_lines():
                    if not line:
                        continue
                    ev = json.loads(line)
                    parts.append(ev.get("response", ""))
                    co.accept(ev.get("response", ""), bool(ev.get("done")))
            return CompletionResult("".join(parts), aid)

        return _run_async(run)

    def get_chat_completions(self, messages, consumer, options):
        return self._generate("\n".join(m.content for m in messages), consumer, options)

    def get_text_completions(self, prompts, consumer, options):
        return self._generate("\n".join(prompts), consumer, options)


class HuggingFaceAPIService(EmbeddingsService, CompletionsService):
    """HF inference REST (``provider: api``); ``provider: local`` maps to the GPU encoder.

    Embeddings (HuggingFaceRestEmbeddingService.java:42-190): POST
    ``{api-url}{model}`` (default ``https://api-inference.huggingface.co/pipeline/
    feature-extraction/``) with ``{"inputs": texts, "options": options}`` (options default
    ``{"wait_for_model": "true"}``, HuggingFaceProvider.java:135-139), Bearer
    ``access-key``; a non-200 answer fails the batch.
    Completions (HuggingFaceProvider.java:157-199): POST ``{inference-url}/models/{model}``
    (default ``https://api-inference.huggingface.co``) with the JSON array of the message
    contents / prompts; the answer is a list of ``{score, token_str, sequence}``.  Text
    completions return ``[0].sequence``; chat completions return one choice per answer
    bean, the first of which is the completion.  The API is not streamed: the chunk
    consumer gets the whole answer as the last chunk."""

    EMBED_URL = "https://api-inference.huggingface.co/pipeline/feature-extraction/"
    INFER_URL = "https://api-inference.huggingface.co"

    def __init__(self, cfg: Dict[str, Any], model: Optional[str] = None, options: Optional[Dict[str, Any]] = None):
        self.cfg = cfg
        self.model = model
        self.embed_url = cfg.get("api-url") or self.EMBED_URL
        self.infer_url = (cfg.get("inference-url") or self.INFER_URL).rstrip("/")
        self.options = options or {"wait_for_model": "true"}

    def _headers(self) -> Dict[str, str]:
        return {"Authorization": f"Bearer {self.cfg.get('access-key', '')}", "Content-Type": "application/json"}

    def compute_embeddings(self, texts):
        if not self.model:
            raise ValueError("huggingface api embeddings: model name is required")
        url = self.embed_url + self.model
        return _run_async(lambda: _http_json(url, {"inputs": list(texts), "options": self.options}, self._headers()))

    def _infer(self, contents: List[str], options: Dict[str, Any]) -> List[dict]:
        model = (options or {}).get("model") or self.model
        if not model:
            raise ValueError("huggingface completions: model is required")
        import requests
        r = requests.post(f"{self.infer_url}/models/{model}", data=json.dumps(list(contents)),
                          headers=self._headers(), timeout=120)
        r.raise_for_status()
        beans = r.json()
        if not isinstance(beans, list):
            raise ValueError(f"huggingface completions: unexpected answer {str(beans)[:200]}")
        return beans

    def get_text_completions(self, prompts, consumer, options):
        def run():
            beans = self._infer(prompts, options)
            text = (beans[0] or {}).get("sequence", "") if beans else ""
            if consumer is not None:
                ChunkCoalescer(consumer, 1, "").accept(text, True)
            return CompletionResult(text)
        return _run_async(run)

    def get_chat_completions(self, messages, consumer, options):
        def run():
            beans = self._infer([m.content for m in messages], options)
            choices = [(b or {}).get("sequence", "") for b in beans]
            text = choices[0] if choices else ""
            if consumer is not None:
                ChunkCoalescer(consumer, 1, "").accept(text, True)
            res = CompletionResult(text)
            res.choices = choices
            return res
        return _run_async(run)


class VertexAIService(CompletionsService, EmbeddingsService):
    """Vertex AI ``:predict`` REST (VertexAIProvider.java:59-500): chat = instances
    [{context, examples, messages[{author, content}]}] -> predictions[0].candidates[0];
    text = instances[{prompt}] (one prompt) -> predictions[0].content; embeddings =
    instances[{content}] -> predictions[i].embeddings.values.  Parameters temperature,
    max-tokens -> maxOutputTokens, topP, topK.  Auth: static ``token`` or an OAuth2 token
    minted from ``serviceAccountJson``."""

    def __init__(self, cfg: Dict[str, Any], model: Optional[str] = None):
        self.cfg = cfg
        self.model = model
        self.project = cfg.get("project")
        self.region = cfg.get("region") or "us-central1"
        self.url = (cfg.get("url") or f"https://{self.region}-aiplatform.googleapis.com").rstrip("/")
        tok = (cfg.get("token") or "").strip()
        sa = (cfg.get("serviceAccountJson") or "").strip()
        self._static = tok or None
        self._sa = None
        if not tok and sa:
            from ...utils.cloudauth import GoogleServiceAccount
            self._sa = GoogleServiceAccount(sa)
        if not tok and not sa:
            raise ValueError("vertex: either token or serviceAccountJson is required")

    def _headers(self):
        return {"Authorization": f"Bearer {self._static or self._sa.token()}"}

    def _predict(self, model: str, body: dict) -> dict:
        url = f"{self.url}/v1/projects/{self.project}/locations/{self.region}/publishers/google/models/{model}:predict"
        return _http_json(url, body, self._headers())

    @staticmethod
    def _params(options: Dict[str, Any]) -> Dict[str, Any]:
        out = {}
        for src, dst, cast in (("temperature", "temperature", float), ("max-tokens", "maxOutputTokens", int),
                               ("topP", "topP", float), ("topK", "topK", int)):
            if options.get(src) is not None:
                out[dst] = cast(options[src])
        return out

    def compute_embeddings(self, texts):
        model = self.model or "textembedding-gecko"
        return _run_async(lambda: [p["embeddings"]["values"] for p in self._predict(
            model, {"instances": [{"content": t} for t in texts]})["predictions"]])

    def get_chat_completions(self, messages, consumer, options):
        model = options.get("model") or self.model

        def run():
            body = {"instances": [{"context": "", "examples": [],
                                   "messages": [{"author": m.role, "content": m.content} for m in messages]}],
                    "parameters": self._params(options)}
            preds = self._predict(model, body)["predictions"]
            cands = preds[0].get("candidates") or [] if preds else []
            text = cands[0].get("content", "") if cands else ""
            aid = f"vertex-{uuid.uuid4().hex[:16]}"
            if consumer is not None:
                consumer(aid, 0, text, True)
            return CompletionResult(text, aid)

        return _run_async(run)

    def get_text_completions(self, prompts, consumer, options):
        if len(prompts) != 1:
            raise ValueError("Vertex AI only supports a single prompt for text completions.")
        model = options.get("model") or self.model

        def run():
            body = {"instances": [{"prompt": prompts[0]}], "parameters": self._params(options)}
            text = self._predict(model, body)["predictions"][0].get("content", "")
            aid = f"vertex-{uuid.uuid4().hex[:16]}"
            if consumer is not None:
                consumer(aid, 0, text, True)
            return CompletionResult(text, aid)

        return _run_async(run)


class BedrockService(CompletionsService, EmbeddingsService):
    """AWS Bedrock runtime ``/model/{modelId}/invoke`` with SigV4 (BedrockServiceProvider.java,
    bedrock/BedrockClient.java): embeddings = one Titan call per text ({"inputText"} ->
    {"embedding"}); completions = one prompt, body {request-prompt-property: prompt,
    **request-parameters} from ``options``, the answer = the EL expression
    ``response-completions-expression`` evaluated over the JSON response (a leading
    newline stripped); chat joins the message contents as the prompt list."""

    def __init__(self, cfg: Dict[str, Any], model: Optional[str] = None):
        self.cfg = cfg
        self.model = model
        self.region = cfg.get("region") or "us-east-1"
        self.ak, self.sk = cfg.get("access-key"), cfg.get("secret-key")
        if not self.ak or not self.sk:
            raise ValueError("bedrock: access-key and secret-key are required")
        self.url = (cfg.get("endpoint-override") or cfg.get("url")
                    or f"https://bedrock-runtime.{self.region}.amazonaws.com").rstrip("/")

    def _invoke(self, model: str, body: dict) -> dict:
        import requests
        url = f"{self.url}/model/{urllib.parse.quote(model, safe='')}/invoke"
        data = json.dumps(body).encode()
        from ...utils.cloudauth import sigv4_headers
        headers = sigv4_headers("POST", url, self.region, "bedrock", self.ak, self.sk, data,
                                {"content-type": "application/json", "accept": "application/json"},
                                session_token=self.cfg.get("session-token"))
        r = requests.post(url, data=data, headers=headers, timeout=120)
        if r.status_code != 200:
            raise RuntimeError(f"bedrock invoke {model}: HTTP {r.status_code} {r.text[:300]}")
        return r.json()

    def compute_embeddings(self, texts):
        model = self.model or "amazon.titan-embed-text-v1"
        return _run_async(lambda: [self._invoke(model, {"inputText": t})["embedding"] for t in texts])

    def get_text_completions(self, prompts, consumer, options):
        if len(prompts) != 1:
            raise ValueError("Bedrock models only support a single prompt for completions.")
        model = options.get("model") or self.model
        bo = options.get("options") or {}
        expr = bo.get("response-completions-expression")
        if not expr:
            raise ValueError("bedrock: options.response-completions-expression is required")

        def run():
            from .el import eval_expression
            body = {bo.get("request-prompt-property", "prompt"): prompts[0]}
            body.update(bo.get("request-parameters") or {})
            resp = self._invoke(model, body)
            val = eval_expression(expr, dict(resp))
            if val is None:
                raise RuntimeError(f"No result found in response (tried with expression {expr}, response was: {resp})")
            text = str(val)
            if text.startswith("\n"):
                text = text[1:]
            aid = f"bedrock-{uuid.uuid4().hex[:16]}"
            if consumer is not None:
                consumer(aid, 0, text, True)
            return CompletionResult(text, aid)

        return _run_async(run)

    def get_chat_completions(self, messages, consumer, options):
        return self.get_text_completions(["\n".join(m.content for m in messages)], consumer, options)


class UnavailableService(CompletionsService, EmbeddingsService):
    def __init__(self, name: str, why: str):
        self.name, self.why = name, why

    def _fail(self, *a, **k):
        f: Future = Future()
        f.set_exception(RuntimeError(f"{self.name} service unavailable: {self.why}"))
        return f

    compute_embeddings = _fail
    get_chat_completions = _fail
    get_text_completions = _fail
