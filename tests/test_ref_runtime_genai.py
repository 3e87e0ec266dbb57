"""Ported reference runtime scenarios, part 2: the GenAI toolkit agents against stub AI
services (the reference's @WireMockTest cases: the same request paths, bodies and
streamed responses), on the memory streaming cluster and the in-tree Kafka broker.

* kafka/ChatCompletionsIT.testChatCompletionWithStreaming (legacy / mustache prompt)
* kafka/TextCompletionsIT.testTextCompletionsWithLogProbs
* kafka/ComputeEmbeddingsIT.testComputeEmbeddings (vertex, open-ai, hugging-face api,
  bedrock; the DJL-local golden vector needs the real multilingual-e5-small weights, which
  do not ship offline: parity unpinned), testComputeBatchEmbeddings (same / different
  keys), testLegacySyntax
"""
from __future__ import annotations

import datetime as _dt
import json

import pytest

from ref_runtime_harness import FakeHTTP, Run, as_json, header, uniq
from langstream_amd.topics.kafka.broker import KafkaBroker


@pytest.fixture(scope="module")
def kafka():
    b = KafkaBroker(default_partitions=1).start()
    yield b
    b.stop()


@pytest.fixture(params=["memory", "kafka"])
def streaming(request, kafka):
    return request.param, (kafka.bootstrap if request.param == "kafka" else None)


@pytest.fixture(scope="module")
def wiremock():
    w = FakeHTTP()
    yield w
    w.close()


@pytest.fixture(autouse=True)
def _reset(wiremock):
    wiremock.reset()


def _globals():
    return {"input-topic": uniq("input-topic"), "output-topic": uniq("output-topic"),
            "stream-topic": uniq("stream-topic")}


MODULE_TOPICS = """module: "module-1"
id: "pipeline-1"
topics:
  - name: "${globals.input-topic}"
    creation-mode: create-if-not-exists
  - name: "${globals.output-topic}"
    creation-mode: create-if-not-exists
  - name: "${globals.stream-topic}"
    creation-mode: create-if-not-exists
"""


# ---------------------------------------------------------------- ChatCompletionsIT
CHAT_SSE = "".join(
    "data: " + json.dumps({"id": "chatcmpl-7tEPYbaK1YcjxwbmkuDqv22vE5w7u", "object": "chat.completion.chunk",
                           "created": 1693397792, "model": "gpt-35-turbo",
                           "choices": [{"index": 0, "finish_reason": fr, "delta": d}], "usage": None}) + "\n\n"
    for d, fr in [({"role": "assistant"}, None), ({"content": "A"}, None), ({"content": " car"}, None),
                  ({"content": " is"}, None), ({"content": " a"}, None), ({"content": " vehicle"}, None),
                  ({}, "stop")]) + "data: [DONE]\n"


@pytest.mark.parametrize("legacy", [True, False])
def test_chat_completion_with_streaming(streaming, wiremock, legacy):
    """ChatCompletionsIT.testChatCompletionWithStreaming: the Azure deployment route and
    body, the completion into value.answer, the log-field (the step config + rendered
    messages + model), the session header kept, and the stream topic's chunks 'A',
    ' car is', ' a vehicle' (1, 2, then the rest) with stream-id / -index / -last-message."""
    wiremock.stub("POST", "/openai/deployments/gpt-35-turbo/chat/completions?api-version=2023-08-01-preview",
                  body='{"messages":[{"role":"user","content":"What can you tell me about the car ?"}],"stream":true}',
                  text=CHAT_SSE)
    prompt = ("What can you tell me about {{% value.question }} ?" if legacy
              else "What can you tell me about {{{ value.question }}} ?")
    g = _globals()
    files = {"configuration.yaml": f"""
configuration:
  resources:
    - type: "open-ai-configuration"
      name: "OpenAI Azure configuration"
      configuration:
        url: "{wiremock.url}"
        access-key: "xxx"
        provider: "azure"
""", "module.yaml": MODULE_TOPICS + f"""pipeline:
  - name: "convert-to-json"
    id: "step1"
    type: "document-to-json"
    input: "${{globals.input-topic}}"
    configuration:
      text-field: "question"
  - name: "chat-completions"
    type: "ai-chat-completions"
    output: "${{globals.output-topic}}"
    configuration:
      model: "gpt-35-turbo"
      stream-to-topic: "${{globals.stream-topic}}"
      stream-response-completion-field: "value"
      completion-field: "value.answer"
      log-field: "value.prompt"
      min-chunks-per-message: 3
      stream: true
      messages:
        - role: user
          content: "{prompt}"
"""}
    with Run(*streaming, files, globals_=g) as r:
        r.produce(g["input-topic"], "the car", headers={"session-id": "2139847128764192"})
        recs, _ = r.read_all(g["output-topic"], 1, 30)
        assert len(recs) == 1
        v = as_json(recs[0].value())
        log_field = json.loads(v.pop("prompt"))
        assert v == {"question": "the car", "session-id": "2139847128764192", "answer": "A car is a vehicle"}
        assert log_field == {
            "options": {"type": "ai-chat-completions", "when": None, "model": "gpt-35-turbo",
                        "messages": [{"role": "user", "content": prompt}], "stream-to-topic": g["stream-topic"],
                        "stream-response-completion-field": "value", "min-chunks-per-message": 3,
                        "completion-field": "value.answer", "stream": True, "log-field": "value.prompt",
                        "max-tokens": None, "temperature": None, "top-p": None, "logit-bias": None, "user": None,
                        "stop": None, "presence-penalty": None, "frequency-penalty": None, "options": None},
            "messages": [{"role": "user", "content": "What can you tell me about the car ?"}],
            "model": "gpt-35-turbo"}
        assert header(recs[0], "stream-id") is None and header(recs[0], "stream-index") is None
        assert header(recs[0], "session-id") == "2139847128764192"
        chunks = r.wait_for(g["stream-topic"], ["A", " car is", " a vehicle"])
        for i, c in enumerate(chunks):
            assert header(c, "stream-id") == "chatcmpl-7tEPYbaK1YcjxwbmkuDqv22vE5w7u"
            assert header(c, "stream-index") == str(i + 1)
            assert header(c, "stream-last-message") == ("true" if i == 2 else "false")
            assert header(c, "session-id") == "2139847128764192"


# ---------------------------------------------------------------- TextCompletionsIT
_TOKENS = [("\n\n", -0.16865084, None), ("I", -0.50947005, None), (" am", -0.81064594, None),
           (" an", -0.0639758, None), (" AI", -0.007819127, None), (" language", -4.2176867, None),
           (" model", -0.00009771052, None), (" and", -0.38906613, None), (" I", -1.1028589, None),
           (" do", -0.18535662, None), (" not", -0.00009115311, None), (" have", -0.0122308275, None),
           (" personal", -0.9290634, None), (" experiences", -0.2772571, None), (" or", -0.06607247, None),
           (" the", -2.1178281, "length")]
TEXT_SSE = "".join(
    "data: " + json.dumps({"id": "cmpl-85xN9HjW7xxICcseHdvb5k5fXL04G", "object": "text_completion",
                           "created": 1696430559, "model": "gpt-3.5-turbo-instruct",
                           "choices": [{"text": t, "index": 0, "logprobs": {"tokens": [t], "token_logprobs": [lp],
                                                                            "top_logprobs": [{t: lp}],
                                                                            "text_offset": [36]},
                                        "finish_reason": fr}]}) + "\n\n"
    for t, lp, fr in _TOKENS) + "data: " + json.dumps(
    {"id": "cmpl-85xN9HjW7xxICcseHdvb5k5fXL04G", "object": "text_completion", "created": 1696430559,
     "model": "gpt-3.5-turbo-instruct", "choices": [{"text": "", "index": 0, "logprobs": {
         "tokens": [], "token_logprobs": [], "top_logprobs": [], "text_offset": []}, "finish_reason": "length"}]}) + \
    "\n\ndata: [DONE]\n"


def test_text_completions_with_logprobs(streaming, wiremock):
    """TextCompletionsIT.testTextCompletionsWithLogProbs: provider openai with a url still
    takes the deployment route; body {prompt, logprobs: 5, stream}; the blank first chunk
    is dropped from the answer and from the logprobs field."""
    wiremock.stub("POST", "/openai/deployments/gpt-3.5-turbo-instruct/completions?api-version=2023-08-01-preview",
                  body='{"prompt":["What can you tell me about the car ?"],"logprobs":5,"stream":true}', text=TEXT_SSE)
    prompt = "What can you tell me about {{{ value.question }}} ?"
    g = _globals()
    files = {"configuration.yaml": f"""
configuration:
  resources:
    - type: "open-ai-configuration"
      name: "OpenAI Azure configuration"
      configuration:
        access-key: "xxx"
        provider: "openai"
        url: "{wiremock.url}"
""", "module.yaml": MODULE_TOPICS + f"""pipeline:
  - name: "convert-to-json"
    id: "step1"
    type: "document-to-json"
    input: "${{globals.input-topic}}"
    configuration:
      text-field: "question"
  - name: "text-completions"
    type: "ai-text-completions"
    output: "${{globals.output-topic}}"
    configuration:
      model: "gpt-3.5-turbo-instruct"
      completion-field: "value.answer"
      log-field: "value.prompt"
      logprobs: 5
      logprobs-field: "value.logprobs"
      min-chunks-per-message: 3
      stream: true
      prompt:
        - "{prompt}"
"""}
    with Run(*streaming, files, globals_=g) as r:
        r.produce(g["input-topic"], "the car")
        recs, _ = r.read_all(g["output-topic"], 1, 30)
        assert len(recs) == 1
        v = as_json(recs[0].value())
        log_field = json.loads(v.pop("prompt"))
        kept = _TOKENS[1:]
        assert v == {"question": "the car",
                     "answer": "I am an AI language model and I do not have personal experiences or the",
                     "logprobs": {"tokens": [t for t, _, _ in kept], "logprobs": [lp for _, lp, _ in kept]}}
        assert log_field == {
            "options": {"type": "ai-text-completions", "when": None, "model": "gpt-3.5-turbo-instruct",
                        "prompt": [prompt], "stream-to-topic": None, "stream-response-completion-field": None,
                        "min-chunks-per-message": 3, "completion-field": "value.answer", "stream": True,
                        "log-field": "value.prompt", "logprobs-field": "value.logprobs", "logprobs": 5.0,
                        "max-tokens": None, "temperature": None, "top-p": None, "logit-bias": None, "user": None,
                        "stop": None, "presence-penalty": None, "frequency-penalty": None, "options": None},
            "messages": ["What can you tell me about the car ?"], "model": "gpt-3.5-turbo-instruct"}
        assert isinstance(log_field["options"]["logprobs"], float)


# ---------------------------------------------------------------- ComputeEmbeddingsIT
def _providers(url):
    amz_date = _dt.datetime.utcnow().strftime("%Y%m%d")
    return {
        "vertex": ("textembedding-gecko", f"""
configuration:
    resources:
       - type: "vertex-configuration"
         name: "Vertex configuration"
         configuration:
           url: "{url}"
           region: "us-east1"
           project: "the-project"
           token: "some-token"
""", [("POST", "/v1/projects/the-project/locations/us-east1/publishers/google/models/textembedding-gecko:predict",
       {"predictions": [{"embeddings": {"statistics": {"truncated": False, "token_count": 6},
                                         "values": [1.0, 5.4, 8.7]}}]})], None),
        "open-ai": ("text-embedding-ada-002", f"""
configuration:
    resources:
      - type: "open-ai-configuration"
        name: "OpenAI Azure configuration"
        configuration:
          url: "{url}"
          access-key: "xxx"
          provider: "azure"
""", [("POST", "/openai/deployments/text-embedding-ada-002/embeddings?api-version=2023-08-01-preview",
       {"data": [{"embedding": [1.0, 5.4, 8.7], "index": 0, "object": "embedding"}],
        "model": "text-embedding-ada-002", "object": "list", "usage": {"prompt_tokens": 5, "total_tokens": 5}})],
            None),
        "hugging-face-api": ("some-model", f"""
configuration:
    resources:
       - type: "hugging-face-configuration"
         name: "Hugging Face API configuration"
         configuration:
           api-url: "{url}/embeddings/"
           model-check-url: "{url}/modelcheck/"
           access-key: "some-token"
           provider: "api"
""", [("GET", "/modelcheck/some-model", {"modelId": "some-model", "tags": ["sentence-transformers"]}),
      ("POST", "/embeddings/some-model", [[1.0, 5.4, 8.7]])], None),
        "bedrock": ("amazon.titan-embed-text-v1", f"""
configuration:
  resources:
   - type: "bedrock-configuration"
     name: "bedrock configuration"
     configuration:
       endpoint-override: "{url}"
       access-key: "xx"
       secret-key: "yy"
""", [("POST", "/model/amazon.titan-embed-text-v1/invoke", {"embedding": [1.0, 5.4, 8.7]})],
            ("Authorization", f"AWS4-HMAC-SHA256 Credential=xx/{amz_date}/us-east-1/bedrock/aws4_request",
             '"inputText"')),
    }


@pytest.mark.parametrize("provider", ["vertex", "open-ai", "hugging-face-api", "bedrock"])
def test_compute_embeddings(streaming, wiremock, provider):
    """ComputeEmbeddingsIT.testComputeEmbeddings[provider]"""
    model, conf, stubs, check = _providers(wiremock.url)[provider]
    for method, path, body in stubs:
        wiremock.stub(method, path, json_body=body)
    tin, tout = uniq("input-topic"), uniq("output-topic")
    files = {"configuration.yaml": conf, "module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
  - name: "{tout}"
    creation-mode: create-if-not-exists
pipeline:
  - name: "compute-embeddings"
    id: "step1"
    type: "compute-ai-embeddings"
    input: "{tin}"
    output: "{tout}"
    configuration:
      model: "{model}"
      model-url: "null"
      embeddings-field: "value.embeddings"
      text: "something to embed"
      concurrency: 1
      flush-interval: 0
"""}
    with Run(*streaming, files) as r:
        r.produce(tin, '{"name": "some name", "description": "some description"}')
        recs, _ = r.read_all(tout, 1, 30)
        assert [as_json(x.value()) for x in recs] == [
            {"name": "some name", "description": "some description", "embeddings": [1.0, 5.4, 8.7]}]
    if check is not None:
        hdr, must_contain, body_part = check
        req = next(q for q in wiremock.requests if q[0] == "POST")
        assert must_contain in req[3].get(hdr, "") and body_part in req[2]


def _batch_files(url, tin, tout, text="something to embed"):
    return {"configuration.yaml": f"""
configuration:
  resources:
    - type: "open-ai-configuration"
      name: "OpenAI Azure configuration"
      configuration:
        url: "{url}"
        access-key: "sdòflkjsòlfkj"
        provider: "azure"
""", "module.yaml": f"""
module: "module-1"
id: "pipeline-1"
topics:
  - name: "{tin}"
    creation-mode: create-if-not-exists
    options:
      consumer.max.poll.records: 100
  - name: "{tout}"
    creation-mode: create-if-not-exists
pipeline:
  - name: "compute-embeddings"
    id: "step1"
    type: "compute-ai-embeddings"
    input: "{tin}"
    output: "{tout}"
    configuration:
      model: "text-embedding-ada-002"
      embeddings-field: "value.embeddings"
      text: "{text}"
      batch-size: 3
      concurrency: 4
      flush-interval: 10000
"""}


EMB = [[1.0, 5.4, 8.7], [2.0, 5.4, 8.7], [3.0, 5.4, 8.7]]


@pytest.mark.parametrize("same_key", [True, False])
def test_compute_batch_embeddings(streaming, wiremock, same_key):
    """ComputeEmbeddingsIT.testComputeBatchEmbeddings: batches of 3 per key bucket (the
    stub answers every batch with the same three vectors, in list order): one key -> the
    messages keep their order; three keys -> three buckets, message i gets vector i // 3."""
    wiremock.stub("POST", "/openai/deployments/text-embedding-ada-002/embeddings?api-version=2023-08-01-preview",
                  json_body={"data": [{"embedding": e, "index": 0, "object": "embedding"} for e in EMB],
                             "model": "text-embedding-ada-002", "object": "list",
                             "usage": {"prompt_tokens": 5, "total_tokens": 5}})
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run(*streaming, _batch_files(wiremock.url, tin, tout)) as r:
        want = []
        for i in range(9):
            key = "key" if same_key else f"key_{i % 3}"
            r.produce(tin, '{"name": " name_%d", "description": "some description"}' % i, key=key)
            e = EMB[i % 3] if same_key else EMB[i // 3]
            want.append({"name": f" name_{i}", "description": "some description", "embeddings": e})
        recs, _ = r.read_all(tout, 9, 30)
        got = [as_json(x.value()) for x in recs]
        if same_key:
            assert got == want
        else:
            assert sorted(map(json.dumps, got)) == sorted(map(json.dumps, want))


def test_compute_embeddings_legacy_syntax(streaming, wiremock):
    """ComputeEmbeddingsIT.testLegacySyntax: ``{{% value.name}}`` renders; the request body
    is exactly {"input":["something to embed foo"]}; the lone record flushes after the
    10 s flush-interval."""
    wiremock.stub("POST", "/openai/deployments/text-embedding-ada-002/embeddings?api-version=2023-08-01-preview",
                  body='{"input":["something to embed foo"]}',
                  json_body={"data": [{"embedding": EMB[0], "index": 0, "object": "embedding"}],
                             "model": "text-embedding-ada-002", "object": "list",
                             "usage": {"prompt_tokens": 5, "total_tokens": 5}})
    tin, tout = uniq("input-topic"), uniq("output-topic")
    with Run(*streaming, _batch_files(wiremock.url, tin, tout, "something to embed {{% value.name}}")) as r:
        r.produce(tin, '{"name": "foo"}')
        recs, _ = r.read_all(tout, 1, 30)
        assert [as_json(x.value()) for x in recs] == [{"name": "foo", "embeddings": EMB[0]}]
