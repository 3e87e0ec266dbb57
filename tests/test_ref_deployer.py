"""The reference's ``ApplicationDeployerTest.testDeploy`` (``langstream-core/src/test/java/ai/
langstream/impl/deploy/ApplicationDeployerTest.java``): the compute cluster receives the
plan of the application with its placeholders resolved from the secrets; a resource no
agent uses is not validated, whatever its type."""
from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.parser import build_application_instance


def test_deploy():
    seen = []

    class MockCompute:
        def deploy(self, tenant, plan, code_archive_id=None):
            seen.append((tenant, plan, code_archive_id))

    app = build_application_instance(
        {"configuration.yaml": """
configuration:
    resources:
        - type: "openai-azure-config"
          name: "OpenAI Azure configuration"
          id: "openai-azure"
          configuration:
            credentials: "${secrets.openai-credentials.accessKey}"
"""},
        """
instance:
    streamingCluster:
        type: memory
    computeCluster:
        type: none
""",
        """
secrets:
    - name: "OpenAI Azure credentials"
      id: "openai-credentials"
      data:
        accessKey: "my-access-key"
""").application
    deployer = ApplicationDeployer(compute_cluster=MockCompute())
    plan = deployer.create_implementation("app", app)
    deployer.deploy("tenant", plan, None)
    assert len(seen) == 1 and seen[0][0] == "tenant"
    assert seen[0][1].application.resources["openai-azure"].configuration["credentials"] == "my-access-key"
