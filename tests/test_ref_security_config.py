"""The reference's ``SecurityConfigurationTest`` (``langstream-webservice/src/test/java/ai/
langstream/webservice/security/infrastructure/primary/SecurityConfigurationTest.java``)
with its own HS256 secret key and its two pre-signed tokens (``iss`` = ``testrole`` /
``notadmin``), ``auth-claim: iss`` and ``admin-roles: testrole``."""
import pytest
import requests

from langstream_amd.webservice.server import ControlPlane, WebServiceServer

SECURITY = {"secret-key": "jDdra78Vo1+RVMGY2easnWe0sAFrEa2581ra5YMotbE=", "auth-claim": "iss",
            "admin-roles": "testrole"}
ROLE_NOTADMIN = "eyJhbGciOiJIUzI1NiJ9.eyJpc3MiOiJub3RhZG1pbiJ9.SMRG0RwT4O9XzOOIPhOV2K7TdwDJI4EDNNFruN_3qtc"
ROLE_TESTROLE = "eyJhbGciOiJIUzI1NiJ9.eyJpc3MiOiJ0ZXN0cm9sZSJ9.Y6VOsE3vw4zOuRnG_WtVGWn25lgwNGkY5VrRpXR9SVI"


@pytest.fixture()
def url(tmp_path):
    cp = ControlPlane(code_dir=str(tmp_path / "code"))
    s = WebServiceServer(cp, port=0, security=SECURITY).start()
    yield s.url
    s.stop()


def _call(url, method, path, token):
    return requests.request(method, url + path, headers={"Authorization": f"Bearer {token}"}, timeout=30)


def test_should_be_authorized(url):
    assert _call(url, "PUT", "/api/tenants/security-configuration-resource", ROLE_TESTROLE).status_code == 200


def test_should_be_forbidden_if_token_is_invalid(url):
    assert _call(url, "PUT", "/api/tenants/security-configuration-resource", "invalid").status_code == 403


def test_should_be_forbidden_if_not_in_admin_role(url):
    assert _call(url, "PUT", "/api/tenants/security-configuration-resource", ROLE_NOTADMIN).status_code == 403


@pytest.mark.parametrize("method,path", [
    ("GET", "/api/applications/{tenant}"), ("GET", "/api/applications/{tenant}/app"),
    ("GET", "/api/applications/{tenant}/app/logs"), ("GET", "/api/applications/{tenant}/app/code"),
    ("GET", "/api/applications/{tenant}/app/code/code-id-1"), ("DELETE", "/api/applications/{tenant}/app")])
def test_should_be_forbidden_if_not_same_tenant(url, method, path):
    """A tenant's principal reaches its own tenant's routes (any status but 403), not
    another tenant's; an admin reaches every tenant's."""
    assert _call(url, method, path.replace("{tenant}", "notadmin"), ROLE_NOTADMIN).status_code != 403
    assert _call(url, method, path.replace("{tenant}", "another-tenant"), ROLE_NOTADMIN).status_code == 403
    assert _call(url, method, path.replace("{tenant}", "notadmin"), ROLE_TESTROLE).status_code != 403
