"""The reference's ``ApplicationServiceValidateUpdateTest`` (``langstream-webservice/src/test/
java/ai/langstream/webservice/application/ApplicationServiceValidateUpdateTest.java``):
which application updates the control plane accepts.  Topics may not be added, removed,
renamed or redefined (creation mode, schema, partitions); agents keep their ids, types and
connections while names, ``when``, ``composable`` and resources may change.

The Java ``testAgents`` cases pass every agent pair through ``validateTopicsUpdate`` and
swallow the expected failures, so they pin nothing for agents; here each case is checked
against ``validate_agents_update`` (``ApplicationService.validateAgentsUpdate``) for real."""
import pytest
import yaml

from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.parser import build_application_instance
from langstream_amd.webservice.server import validate_agents_update, validate_topics_update

CONFIGURATION = """
configuration:
  resources:
    - name: open-ai
      type: open-ai-configuration
      configuration:
        url: "http://something"
        access-key: "xxcxcxc"
        provider: "azure"
"""
INSTANCE = """
instance:
  streamingCluster:
    type: "noop"
  computeCluster:
    type: "none"
"""
IO = [{"name": "input-topic"}, {"name": "output-topic"}]


def _plan(topics, agents=()):
    module = {"id": "pi", "module": "mod", "topics": topics}
    if agents:
        module["pipeline"] = list(agents)
    info = build_application_instance({"configuration.yaml": CONFIGURATION, "module.yaml": yaml.safe_dump(module)},
                                      INSTANCE, None)
    return ApplicationDeployer().create_implementation("app", info.application)


def _valid(check, a, b) -> bool:
    try:
        check(a, b)
        return True
    except ValueError:
        return False


def T(name="input-topic", creation=None, schema=None, partitions=0):
    t = {"name": name, "partitions": partitions}
    if creation:
        t["creation-mode"] = creation
    if schema:
        t["schema"] = {"type": schema[0], "schema": schema[1]}
    return t


@pytest.mark.parametrize("old,new,ok", [
    ([T()], [T()], True),
    ([T()], [T("input-topic1")], False),
    ([T()], [T(), T("input-topic1")], False),
    ([T(), T("input-topic1")], [T()], False),
    ([T(creation="create-if-not-exists")], [T(creation="create-if-not-exists")], True),
    ([T(creation="none")], [T()], True),
    ([T(schema=("avro", "{}"))], [T()], False),
    ([T(schema=("avro", "{}"))], [T(schema=("json", "{}"))], False),
    ([T(schema=("avro", "{}"))], [T(schema=("avro", "{schema:true}"))], False),
    ([T(partitions=1)], [T(partitions=0)], False),
    ([T(partitions=1)], [T(partitions=2)], False),
])
def test_topics(old, new, ok):
    """ApplicationServiceValidateUpdateTest.testTopics"""
    assert _valid(validate_topics_update, _plan(old), _plan(new)) is ok


def A(id="agent", name="My Agent", type="drop", inp="input-topic", out="output-topic", conf=None, res=None):
    a = {"id": id, "name": name, "type": type, "input": inp, "output": out, "configuration": conf or {}}
    if res:
        a["resources"] = {"parallelism": res[0], "size": res[1]}
    return a


@pytest.mark.parametrize("old,new,ok", [
    ([A()], [A()], True),
    ([A()], [A("agent1")], False),
    ([A("agent1")], [A()], False),
    ([A()], [A(), A("agent2")], False),
    ([A("agent1"), A("agent2")], [A("agent1")], False),
    ([A()], [A(name="My Agent - another name")], True),
    ([A()], [A(type="drop-fields", conf={"fields": ["f"]})], False),
    ([A()], [A(inp="output-topic", out="input-topic")], False),
    ([A(conf={"when": "true"})], [A(conf={"when": "false"})], True),
    ([A(conf={"when": "true"})], [A(conf={"composable": "false"})], True),
    ([A(res=(1, 1))], [A(res=(1, 1))], True),
    ([A(res=(1, 1))], [A(res=(2, 1))], True),
    ([A(res=(1, 1))], [A(res=(1, 2))], True),
    ([A(res=(1, 1))], [A(res=(2, 2))], True),
    ([A(res=(2, 2))], [A(res=(1, 1))], True),
])
def test_agents(old, new, ok):
    """ApplicationServiceValidateUpdateTest.testAgents"""
    a, b = _plan(IO, old), _plan(IO, new)
    assert _valid(validate_topics_update, a, b)
    assert _valid(validate_agents_update, a, b) is ok
