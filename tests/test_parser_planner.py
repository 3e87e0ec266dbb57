"""Application model: YAML parsing, placeholders, planning and agent fusion.

Mirrors the reference's parser/planner unit tests (SURVEY §4:
ModelBuilderTest, PlaceholderTest, ComposableAgentExecutionPlanOptimiserTest,
KafkaClusterRuntimeDockerTest topic-creation expectations)."""
import pytest

from langstream_amd.api.model import DEFAULT_MODULE
from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.parser import build_application_instance
from langstream_amd.core.placeholders import resolve_in_string, resolve_placeholders
from langstream_amd.core.planner import Planner

PIPE = """
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
  - name: "output-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "step1"
    type: "drop-fields"
    input: "input-topic"
    configuration:
      fields: ["a"]
  - name: "step2"
    type: "compute"
    configuration:
      fields:
        - name: "value.x"
          expression: "value.b + 1"
  - name: "step3"
    type: "compute"
    output: "output-topic"
    configuration:
      fields:
        - name: "value.y"
          expression: "value.x * 2"
"""


def _plan(files, instance=None, secrets=None):
    app = build_application_instance(files, instance, secrets).application
    app = resolve_placeholders(app)
    return Planner().build_execution_plan("app", app)


def test_auto_ids_and_implicit_chaining():
    app = build_application_instance({"pipeline.yaml": PIPE}).application
    pipe = app.modules[DEFAULT_MODULE].pipelines["pipeline"]
    ids = [a.id for a in pipe.agents]
    assert ids == ["pipeline-drop-fields-1", "pipeline-compute-2", "pipeline-compute-3"]
    assert pipe.agents[1].input.connection_type == "AGENT"
    assert pipe.agents[0].output.connection_type == "AGENT"


def test_composable_agents_fuse_into_one_composite():
    plan = _plan({"pipeline.yaml": PIPE})
    assert len(plan.agents) == 1
    node = next(iter(plan.agents.values()))
    assert node.agent_type == "composite-agent"
    assert [p["agentId"] for p in node.configuration["processors"]] == [
        "pipeline-drop-fields-1", "pipeline-compute-2", "pipeline-compute-3"]
    assert node.input.name == "input-topic" and node.output.name == "output-topic"
    # intermediate implicit topics are discarded by the fusion
    assert sorted(plan.topics) == ["input-topic", "output-topic"]


def test_different_parallelism_prevents_fusion_and_creates_implicit_topic():
    pipe = PIPE.replace('  - name: "step3"\n', '  - name: "step3"\n    resources:\n      parallelism: 2\n')
    plan = _plan({"pipeline.yaml": pipe})
    assert len(plan.agents) == 2
    assert "agent-pipeline-compute-3-input" in plan.topics
    t = plan.topics["agent-pipeline-compute-3-input"]
    assert t.implicit and t.partitions == 1


def test_dead_letter_topic_created():
    pipe = PIPE.replace('    input: "input-topic"\n', '    input: "input-topic"\n    errors:\n'
                        '      on-failure: dead-letter\n')
    plan = _plan({"pipeline.yaml": pipe})
    assert "input-topic-deadletter" in plan.topics


def test_errors_validation():
    bad = PIPE.replace('    input: "input-topic"\n', '    input: "input-topic"\n    errors:\n'
                       '      on-failure: explode\n')
    with pytest.raises(ValueError, match="on-failure"):
        build_application_instance({"pipeline.yaml": bad})


def test_missing_agent_type_rejected():
    with pytest.raises(ValueError, match="type is always required"):
        build_application_instance({"p.yaml": "pipeline:\n  - name: x\n"})


def test_instance_and_secrets_not_allowed_in_app():
    with pytest.raises(ValueError):
        build_application_instance({"instance.yaml": "instance: {}"})


def test_gateway_validation():
    gw = """
gateways:
  - id: chat
    type: chat
    chat-options:
      questions-topic: q
"""
    with pytest.raises(ValueError, match="answers-topic"):
        build_application_instance({"gateways.yaml": gw, "pipeline.yaml": PIPE})
    ok = gw + "      answers-topic: a\n"
    app = build_application_instance({"gateways.yaml": ok, "pipeline.yaml": PIPE}).application
    assert app.gateways[0].chat_options.answers_topic == "a"


def test_placeholders_resolve_globals_and_secrets():
    conf = """
configuration:
  resources:
    - type: "open-ai-configuration"
      name: "OpenAI"
      configuration:
        access-key: "${secrets.openai.key}"
        url: "{{ secrets.openai.url }}"
"""
    pipe = PIPE.replace('          expression: "value.b + 1"', '          expression: "\'${globals.suffix}\'"')
    instance = "instance:\n  globals:\n    suffix: hello\n  streamingCluster:\n    type: memory\n"
    secrets = "secrets:\n  - id: openai\n    data:\n      key: k123\n      url: http://x\n"
    app = build_application_instance({"configuration.yaml": conf, "pipeline.yaml": pipe}, instance,
                                     secrets).application
    app = resolve_placeholders(app)
    res = next(iter(app.resources.values()))
    assert res.configuration["access-key"] == "k123"
    assert res.configuration["url"] == "http://x"
    agent = app.modules[DEFAULT_MODULE].pipelines["pipeline"].agents[1]
    assert agent.configuration["fields"][0]["expression"] == "'hello'"


def test_resolve_in_string():
    ctx = {"globals": {"a": "1", "n": {"b": 2}}, "secrets": {}}
    assert resolve_in_string("x-${globals.a}-${globals.n.b}", ctx) == "x-1-2"
    assert resolve_in_string("x-{{globals.a}}-{{ globals.n.b }}", ctx) == "x-1-2"
    # mustache templates meant for the agent (not globals/secrets) are left alone
    assert resolve_in_string("hi {{ value.question }}", ctx) == "hi {{ value.question }}"


def test_deployer_plan_dict_roundtrip():
    app = build_application_instance({"pipeline.yaml": PIPE}).application
    plan = ApplicationDeployer().create_implementation("app", app)
    d = plan.to_dict()
    assert d["application-id"] == "app"
    assert len(d["agents"]) == 1


def test_service_agent_cannot_have_input():
    pipe = """
topics:
  - name: t
pipeline:
  - name: svc
    type: python-service
    input: t
    configuration:
      className: x.Y
"""
    with pytest.raises(ValueError, match="Service agents"):
        _plan({"pipeline.yaml": pipe})


# ---------------------------------------------------------------- configuration models
def _one(agent_type, cfg, extra=""):
    import yaml
    body = yaml.safe_dump({"pipeline": [{"name": "a1", "type": agent_type, "input": "in", "configuration": cfg}],
                           "topics": [{"name": "in", "creation-mode": "create-if-not-exists"}]})
    return _plan({"pipeline.yaml": body, **({"configuration.yaml": extra} if extra else {})})


def test_config_validator_unknown_required_types_and_el():
    with pytest.raises(ValueError, match=r"Found error on agent configuration \(agent: 'a1', type: 'drop-fields'\). "
                                         r"Property 'bogus' is unknown"):
        _one("drop-fields", {"fields": ["a"], "bogus": 1})
    with pytest.raises(ValueError, match="Property 'fields' is required"):
        _one("drop-fields", {})
    with pytest.raises(ValueError, match=r"Property 'fields\[0\]' has a wrong data type"):
        _one("drop-fields", {"fields": [{"x": 1}]})
    with pytest.raises(ValueError, match="Property 'fields.expression' is required"):
        _one("compute", {"fields": [{"name": "value.x"}]})
    with pytest.raises(ValueError, match="Property 'fields.expression' has an invalid EL expression"):
        _one("compute", {"fields": [{"name": "value.x", "expression": "value.a +* 2"}]})
    with pytest.raises(ValueError, match="Property 'max' has a wrong data type. Expected type: int"):
        _one("re-rank", {"field": "f", "output-field": "o", "max": "many"})
    # coercion as in the reference (numbers / booleans given as strings)
    plan = _one("re-rank", {"field": "f", "output-field": "o", "max": "7", "lambda": "0.3"})
    node = next(iter(plan.agents.values()))
    assert node.configuration["max"] == 7 and node.configuration["lambda"] == 0.3
    # python agents accept any extra keys
    _one("python-processor", {"className": "x.Y", "anything": {"goes": True}})
    with pytest.raises(ValueError, match="Property 'className' is required"):
        _one("python-processor", {})


def test_vector_sink_model_follows_datasource_service():
    res = """
configuration:
  resources:
    - type: datasource
      name: ks
      configuration:
        service: cassandra
        contact-points: 127.0.0.1
        loadBalancing-localDc: dc1
"""
    _one("vector-db-sink", {"datasource": "ks", "table-name": "t", "mapping": "a=value.a"}, res)
    with pytest.raises(ValueError, match="Property 'fields' is unknown"):
        _one("vector-db-sink", {"datasource": "ks", "table-name": "t", "mapping": "a=value.a", "fields": []}, res)
    with pytest.raises(ValueError, match=r"resource configuration \(resource: 'ks', type: 'datasource'\). "
                                         r"Property 'loadBalancing-localDc' is required"):
        _one("vector-db-sink", {"datasource": "ks", "table-name": "t", "mapping": "a=value.a"},
             res.replace("        loadBalancing-localDc: dc1\n", ""))


def test_asset_model_and_docs():
    from langstream_amd.api.model import AssetDefinition
    from langstream_amd.core.config_model import docs_markdown, generate_docs, validate_asset
    with pytest.raises(ValueError, match=r"asset configuration \(asset: 'c', type: 'astra-collection'\). "
                                         r"Property 'vector-dimension' is required"):
        validate_asset("c", "astra-collection", {"datasource": "d", "collection-name": "c"})
    assert validate_asset("c", "astra-collection", {"datasource": "d", "collection-name": "c",
                                                     "vector-dimension": "8"})["vector-dimension"] == 8
    docs = generate_docs("1.0")
    assert docs["version"] == "1.0" and set(docs) == {"version", "agents", "resources", "assets"}
    ce = docs["agents"]["compute-ai-embeddings"]
    assert ce["properties"]["batch-size"] == {"description": "Records per embedding batch.", "required": False,
                                              "type": "integer", "defaultValue": 10}
    assert docs["agents"]["compute"]["properties"]["fields"]["items"]["properties"]["expression"][
        "extendedValidationType"] == "EL_EXPRESSION"
    assert "vector-db-sink_cassandra" in docs["agents"] and "datasource_milvus" in docs["resources"]
    assert "milvus-collection" in docs["assets"]
    md = docs_markdown(docs)
    assert "### `text-splitter`" in md and "| `chunk_size` | integer |" in md
    from langstream_amd.cli.main import main
    assert main(["docs", "--format", "markdown", "-o", "/dev/null"]) == 0
