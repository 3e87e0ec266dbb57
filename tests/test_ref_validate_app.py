"""The reference's ``ApplicationServiceValidateAppTest`` (``langstream-webservice/src/test/java/
ai/langstream/webservice/application/ApplicationServiceValidateAppTest.java``): on a
kubernetes compute cluster the application id and every agent id (given or computed)
must make valid resource names."""
import pytest

from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.parser import build_application_instance

INSTANCE = """
instance:
  streamingCluster:
    type: "noop"
  computeCluster:
    type: "kubernetes"
"""


def files_with_one_agent(module=None, pipeline=None, agent_id=None):
    pipeline = pipeline or "pipeline"
    return {f"{pipeline}.yaml": f"""
module: {module if module is not None else 'null'}
id: {pipeline}
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
  - name: "output-topic"
    creation-mode: create-if-not-exists
pipeline:
  - id: {agent_id if agent_id is not None else 'null'}
    type: "drop"
    input: "input-topic"
    output: "output-topic"
"""}


def valid(app_id, files) -> bool:
    app = build_application_instance(files, INSTANCE, None).application
    try:
        ApplicationDeployer().create_implementation(app_id, app)
        return True
    except ValueError:
        return False


@pytest.mark.parametrize("app_id,ok", [
    (None, False), ("", False), ("myapp", True), ("all-chars09", True), ("myapp with spaces", False),
    ("myapp_", False), ("9myapp", False), ("Umyapp", False), ("a" * 20, True), ("a" * 21, False)])
def test_application_id(app_id, ok):
    """testApplicationId"""
    assert valid(app_id, files_with_one_agent(agent_id="s")) is ok


@pytest.mark.parametrize("agent_id,ok", [
    ("agent", True), ("agent01-", True), ("a" * 37, True), ("a" * 38, False), ("with spaces", False),
    ("Upper", False), ("0agent", True), ("0", True)])
def test_agent_with_fixed_id(agent_id, ok):
    """testAgentWithFixedId"""
    assert valid("app", files_with_one_agent(agent_id=agent_id)) is ok


@pytest.mark.parametrize("module,ok", [
    (None, True), ("m" * 21, True), ("m" * 24, False), ("with spaces", False), ("withUpper", False)])
def test_agent_with_computed_id(module, ok):
    """testAgentWithComputedId"""
    assert valid("app", files_with_one_agent(module=module)) is ok


def test_other_compute_clusters_take_any_id():
    app = build_application_instance(files_with_one_agent(agent_id="Upper"),
                                     INSTANCE.replace("kubernetes", "none"), None).application
    ApplicationDeployer().create_implementation("My_App", app)
