"""The reference's ``ArchetypeResourceTest`` (``langstream-webservice/src/test/java/ai/langstream/
webservice/archetype/ArchetypeResourceTest.java``) against this control plane's HTTP API,
on the reference's own test archetype (``langstream-webservice/src/test/archetypes/simple``,
read in place; skipped without the reference checkout).  The Java test deploys into a k3s
test server; here the control plane's start step is a stub that marks the application
deployed, since the archetype's Kafka cluster is a placeholder address."""
import os

import pytest
import requests

from langstream_amd.webservice.server import ControlPlane, WebServiceServer

ARCHETYPES = "/root/reference/langstream-webservice/src/test/archetypes"
pytestmark = pytest.mark.skipif(not os.path.isdir(ARCHETYPES), reason="reference checkout absent")


@pytest.fixture()
def srv(monkeypatch, tmp_path):
    cp = ControlPlane(code_dir=str(tmp_path / "code"))
    cp.archetypes_dir = ARCHETYPES

    def start(sa, plan):
        sa.status = "DEPLOYED"
        cp.store.put(sa)
    monkeypatch.setattr(cp, "_start", start)
    s = WebServiceServer(cp, port=0).start()
    yield cp, s.url
    s.stop()


def test_archetypes_metadata(srv):
    """testArchetypesMetadata"""
    cp, url = srv
    assert requests.put(f"{url}/api/tenants/my-tenant").status_code == 200
    r = requests.get(f"{url}/api/archetypes/my-tenant")
    assert r.status_code == 200
    lst = r.json()
    assert len(lst) == 1 and lst[0]["id"] == "simple"
    assert requests.get(f"{url}/api/archetypes/my-tenant/not-exists").status_code == 404
    r = requests.get(f"{url}/api/archetypes/my-tenant/simple")
    assert r.status_code == 200

    def par(name, binding):
        return {"default": None, "name": name, "label": None, "description": None, "type": None,
                "subtype": None, "binding": binding, "required": False}
    assert r.json() == {"archetype": {
        "id": "simple", "title": "Simple", "labels": None, "description": None, "icon": None,
        "sections": [
            {"title": "Section 1", "description": "Xxxxx", "parameters": [
                par("s1", "globals.string-value"), par("i1", "globals.input-value"), par("r1", "globals.int-value"),
                par("m1", "globals.map-value"), par("l1", "globals.list-value"),
                par("m2", "globals.nested-map.key2.key2-1")]},
            {"title": "Section 2", "description": "Xxxxx", "parameters": [
                par("s2", "secrets.open-ai.foo"), par("i2", "secrets.open-ai.foo-int"),
                par("k2", "secrets.kafka.bootstrap-servers")]}]}}


def test_deploy_from_archetype(srv):
    """testDeployFromArchetype"""
    cp, url = srv
    assert requests.put(f"{url}/api/tenants/my-tenant").status_code == 200
    params = {"s1": "value 1", "i1": 50, "r1": 89, "m1": {"key1": "value 1", "key2": {"key2-1": "value 2-1"}},
              "m2": "a", "l1": ["value 1", "value 2"], "s2": "value secret 2", "i2": 100, "k2": "value 3"}
    r = requests.post(f"{url}/api/archetypes/my-tenant/simple/applications/app-id", json=params)
    assert r.status_code == 200, r.text
    g = r.json()["instance"]["globals"]
    assert g["input-value"] == 50 and g["int-value"] == 89
    assert g["list-value"] == ["value 1", "value 2"]
    assert g["map-value"] == {"key1": "value 1", "key2": {"key2-1": "value 2-1"}}
    assert g["nested-map"] == {"key1": {"key1-1": "nested-map-value-1-1", "key1-2": "nested-map-value-1-2"},
                               "key2": {"key2-1": "a", "key2-2": "nested-map-value-2-2"}}
    assert r.json()["instance"]["streamingCluster"]["type"] == "kafka"
    sa = cp.store.get("my-tenant", "app-id")
    sec = sa.application.secrets.secrets
    assert sec["open-ai"].data["foo"] == "value secret 2"
    assert sec["open-ai"].data["foo-int"] == 100
    assert sec["kafka"].data["bootstrap-servers"] == "value 3"
    code = requests.get(f"{url}/api/applications/my-tenant/app-id/code")
    assert code.status_code == 200 and code.content[:2] == b"PK"
