"""Control plane (webservice REST + admin client), CLI helpers, k8s manifests and the
agent HTTP API.

Mirrors the reference's ApplicationResourceTest / TenantResourceTest / CLI
AppsCmdTest (mock server) with the real in-process servers."""
import json
import os
import textwrap
import time

import pytest
import yaml

from langstream_amd.cli.client import AdminClient, AdminClientError
from langstream_amd.cli.main import main as cli_main, mermaid
from langstream_amd.core.deployer import ApplicationDeployer
from langstream_amd.core.k8s import render_manifests
from langstream_amd.core.parser import build_application_instance
from langstream_amd.topics.memory import reset_memlogs
from langstream_amd.webservice.server import ControlPlane, WebServiceServer

PIPE = """
topics:
  - name: "in-topic"
    creation-mode: create-if-not-exists
  - name: "out-topic"
    creation-mode: create-if-not-exists
pipeline:
  - name: "upper"
    type: "python-processor"
    input: "in-topic"
    output: "out-topic"
    resources:
      parallelism: 2
      size: 2
    configuration:
      className: "upper.Upper"
"""

CODE = """
import logging
from langstream import SimpleRecord

class Upper:
    def process(self, record):
        logging.getLogger("upper").info("processing %s", record.value())
        return [SimpleRecord(str(record.value()).upper())]
"""


@pytest.fixture()
def app_dir(tmp_path):
    d = tmp_path / "app"
    (d / "python").mkdir(parents=True)
    (d / "pipeline.yaml").write_text(PIPE)
    (d / "python" / "upper.py").write_text(textwrap.dedent(CODE))
    return str(d)


@pytest.fixture()
def server(tmp_path):
    reset_memlogs()
    cp = ControlPlane(code_dir=str(tmp_path / "code"), max_units_per_tenant=10)
    srv = WebServiceServer(cp, port=0).start()
    yield cp, srv
    for t in list(cp.store.list_tenants()):
        for a in cp.store.list(t):
            cp.delete(t, a.application_id, force=True)
    srv.stop()
    reset_memlogs()


def test_tenants_and_app_lifecycle(server, app_dir):
    import logging
    logging.getLogger("upper").setLevel(logging.INFO)
    cp, srv = server
    cl = AdminClient(srv.url, "t1")
    with pytest.raises(AdminClientError) as ei:
        cl.deploy("app", app_dir)
    assert ei.value.status == 404  # tenant missing
    cl.tenant_put("t1")
    assert "t1" in cl.tenants()
    plan = cl.deploy("app", app_dir, dry_run=True)
    assert "in-topic" in [t["name"] for m in plan["modules"] for t in m.get("topics") or []]
    assert cl.list() == []
    res = cl.deploy("app", app_dir)
    assert res["status"]["status"]["status"] == "DEPLOYED"
    with pytest.raises(AdminClientError) as ei:
        cl.deploy("app", app_dir)
    assert ei.value.status == 409
    sa = cp.store.get("t1", "app")
    sa.runner.produce("in-topic", "hello")
    out = sa.runner.consume("out-topic", 1, timeout=20)
    assert out[0].value() == "HELLO"
    info = cl.get("app", stats=True)
    assert len(info["status"]["agents"]) == 2  # two replicas
    logs = list(cl.logs("app", follow=False))
    assert any("processing hello" in r["message"] for r in logs)
    zipped = cl.download("app")
    assert zipped[:2] == b"PK"
    old_archive = sa.code_archive_id
    cl.update("app", app_dir)  # same python code -> same code archive
    assert cp.store.get("t1", "app").code_archive_id == old_archive
    cl.delete("app")
    assert cl.list() == []
    import requests
    docs = requests.get(f"{srv.url}/api/docs", timeout=10).json()
    assert "ai-chat-completions" in docs["agents"] and "open-ai-configuration" in docs["resources"]


def test_tenant_resource_limit(server, app_dir, tmp_path):
    cp, srv = server
    cl = AdminClient(srv.url, "t2")
    cl.tenant_put("t2")
    cl.deploy("a1", app_dir)  # 2 replicas x size 2 = 4 units
    cl.deploy("a2", app_dir)  # 8 units
    with pytest.raises(AdminClientError) as ei:
        cl.deploy("a3", app_dir)  # 12 > 10
    assert ei.value.status == 403


def test_mermaid_and_manifests(app_dir):
    m = mermaid(app_dir)
    assert m.startswith("flowchart LR") and "in-topic" in m and "python-processor" in m
    app = build_application_instance({"pipeline.yaml": PIPE}).application
    plan = ApplicationDeployer().create_implementation("app", app)
    ms = render_manifests(plan, "t1", "abc")
    kinds = [x["kind"] for x in ms]
    assert kinds == ["Secret", "Agent", "StatefulSet", "Service"]
    sts = ms[2]
    assert sts["spec"]["replicas"] == 2 and sts["spec"]["podManagementPolicy"] == "Parallel"
    c = sts["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["cpu"] == "1" and c["resources"]["limits"]["memory"] == "1024M"
    assert "amd.com/gpu" not in c["resources"]["limits"]  # CPU agent
    assert yaml.safe_load_all(__import__("langstream_amd.core.k8s", fromlist=["to_yaml"]).to_yaml(ms))


def test_cli_profiles_and_diagram(tmp_path, app_dir, monkeypatch, capsys):
    monkeypatch.setattr("langstream_amd.cli.main.CONFIG", str(tmp_path / "cfg.yaml"))
    assert cli_main(["profiles", "create", "p1", "--web-service-url", "http://x:1", "--tenant", "tt",
                     "--set-current"]) == 0
    capsys.readouterr()
    assert cli_main(["profiles", "list", "-o", "json"]) == 0     # ListProfileCmd: the whole config
    out = json.loads(capsys.readouterr().out)
    assert out["currentProfile"] == "p1" and out["profiles"]["p1"]["tenant"] == "tt"
    assert cli_main(["apps", "diagram", "-app", app_dir]) == 0
    assert "flowchart" in capsys.readouterr().out


def test_agent_http_api():
    import requests
    from langstream_amd.runtime.local import LocalApplicationRunner
    from langstream_amd.runtime.pod import AgentAPIServer
    reset_memlogs()
    pipe = PIPE.replace('type: "python-processor"', 'type: "compute"').replace(
        'className: "upper.Upper"', 'fields:\n        - name: "value"\n          expression: "fn:uppercase(value)"')
    with LocalApplicationRunner.from_yaml({"pipeline.yaml": pipe}) as app:
        api = AgentAPIServer(app.runners, host="127.0.0.1", port=0).start()
        try:
            app.produce("in-topic", "x")
            app.consume("out-topic", 1, timeout=10)
            info = requests.get(f"http://127.0.0.1:{api.port}/info", timeout=5).json()
            assert info and info[0]["agent-id"]
            m = requests.get(f"http://127.0.0.1:{api.port}/metrics", timeout=5).text
            assert "langstream" in m
            assert requests.post(f"http://127.0.0.1:{api.port}/commands/restart", timeout=5).status_code == 200
        finally:
            api.stop()
    reset_memlogs()
