"""The reference's ``ApplicationServiceResourceLimitTest`` (``langstream-webservice/src/test/java/
ai/langstream/webservice/application/ApplicationServiceResourceLimitTest.java``): an
application's units (size x parallelism of every agent after consecutive composable agents
merge) plus the tenant's other applications' must fit the tenant's limit, or the default
limit when the tenant sets none; 0 means unlimited."""
import pytest

from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.parser import build_application_instance
from langstream_amd.webservice.server import ControlPlane

INSTANCE = """
instance:
  streamingCluster:
    type: "noop"
  computeCluster:
    type: "kubernetes"
"""


def files_with_two_agents(size, parallelism):
    return {"pip.yaml": f"""
module: mod
id: pip
resources:
  size: {size}
  parallelism: {parallelism}
topics:
  - name: "input-topic"
    creation-mode: create-if-not-exists
  - name: "output-topic"
    creation-mode: create-if-not-exists
pipeline:
  - id: step1
    type: "drop"
    input: "input-topic"
  - id: step2
    type: "drop"
    output: "output-topic"
"""}


CASES = [  # (tenant limit, app, (size, parallelism), current usage, default limit, ok)
    (0, "app1", (100, 100), {}, 0, True),
    (0, "app1", (1, 2), {}, 1, False), (0, "app1", (1, 2), {}, 2, True), (0, "app1", (1, 2), {}, 3, True),
    (0, "app1", (2, 1), {}, 1, False), (0, "app1", (2, 1), {}, 2, True), (0, "app1", (2, 1), {}, 3, True),
    (0, "app1", (1, 2), {"app1": 1}, 1, False), (0, "app1", (1, 2), {"app1": 2}, 2, True),
    (0, "app1", (1, 2), {"app1": 2, "app2": 2}, 4, True), (0, "app3", (1, 2), {"app1": 2, "app2": 2}, 4, False),
    (6, "app3", (1, 2), {"app1": 2, "app2": 2}, 4, True), (4, "app3", (1, 2), {"app1": 2, "app2": 2}, 4, False),
    (0, "app3", (1, 2), {"app1": 2, "app2": 2}, 4, False),
]


@pytest.mark.parametrize("tenant_limit,app_id,res,usage,default,ok", CASES)
def test_resource_limit(tenant_limit, app_id, res, usage, default, ok):
    cp = ControlPlane(max_units_per_tenant=default)
    cp.store.put_tenant("tenant", {"maxTotalResourceUnits": tenant_limit})
    app = build_application_instance(files_with_two_agents(*res), INSTANCE, None).application
    plan = ApplicationDeployer().create_implementation(app_id, app)
    assert len(plan.agents) == 1    # the two drop agents run as one
    if ok:
        cp.check_resource_usage("tenant", app_id, plan, usage)
    else:
        with pytest.raises(PermissionError) as e:
            cp.check_resource_usage("tenant", app_id, plan, usage)
        assert str(e.value) == f"Not enough resources to deploy application {app_id}"
