"""The reference's ``DefaultTenantTest`` / ``DefaultTenantDisabledTest`` (``langstream-webservice/
src/test/java/ai/langstream/webservice/``) and ``GlobalMetadataService``'s unit cap
(``maxTotalResourceUnitsLimit``, GlobalMetadataService.java:66-75)."""
import pytest
import requests

from langstream_amd.webservice.server import ControlPlane, WebServiceServer


def test_default_tenant():
    cp = ControlPlane(default_tenant="default")
    assert list(cp.store.list_tenants()) == ["default"]
    assert cp.store.get_tenant("default") is not None


def test_default_tenant_disabled():
    assert len(ControlPlane(default_tenant=None).store.list_tenants()) == 0


def test_max_total_resource_units_limit(tmp_path):
    cp = ControlPlane(code_dir=str(tmp_path), max_units_limit=10)
    srv = WebServiceServer(cp, port=0).start()
    try:
        r = requests.put(f"{srv.url}/api/tenants/t", json={"maxTotalResourceUnits": 11})
        assert r.status_code == 400 and r.text == "Max total resource units limit is 10"
        assert requests.put(f"{srv.url}/api/tenants/t", json={"maxTotalResourceUnits": 10}).status_code == 200
        assert requests.patch(f"{srv.url}/api/tenants/t", json={"maxTotalResourceUnits": 12}).status_code == 400
        assert requests.patch(f"{srv.url}/api/tenants/t", json={"maxTotalResourceUnits": 0}).status_code == 200
    finally:
        srv.stop()
