"""Admin client for the control plane REST API (SURVEY §2.7 G7,
``langstream-admin-client/.../AdminClient.java``): tenants, applications (multipart
deploy / update with app zip + instance + secrets), logs, code download, archetypes.
Retries idempotent calls on connection errors / 5xx with backoff."""
from __future__ import annotations

import io
import json
import os
import time
import zipfile
from typing import Any, Dict, Iterator, Optional


def zip_directory(path: str) -> bytes:
    """The application directory as a zip, minus ``.langstreamignore`` matches (ignored
    directories are not descended into; ``ApplicationPackager.java:44-80``)."""
    from .ignore import load_ignore
    ign = load_ignore(path)
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_DEFLATED) as z:
        for root, dirs, files in os.walk(path):
            dirs[:] = sorted(d for d in dirs if d not in ("__pycache__", ".git")
                             and not (ign and ign.matches(os.path.join(root, d), True)))
            for fn in sorted(files):
                full = os.path.join(root, fn)
                if ign and ign.matches(full, False):
                    continue
                z.write(full, os.path.relpath(full, path))
    return buf.getvalue()


class AdminClientError(Exception):
    def __init__(self, status: int, text: str):
        super().__init__(f"HTTP {status}: {text}")
        self.status = status


class AdminClient:
    def __init__(self, web_service_url: str, tenant: str = "default", token: Optional[str] = None,
                 retries: int = 3, timeout: float = 120.0):
        import requests
        self.url = web_service_url.rstrip("/")
        self.tenant = tenant
        self.retries = retries
        self.timeout = timeout
        self.http = requests.Session()
        if token:
            self.http.headers["Authorization"] = f"Bearer {token}"

    def _call(self, method: str, path: str, idempotent: bool = True, **kw):
        import requests
        last = None
        for i in range(self.retries if idempotent else 1):
            try:
                r = self.http.request(method, self.url + path, timeout=self.timeout, **kw)
            except requests.ConnectionError as e:
                last = e
                time.sleep(0.5 * (2 ** i))
                continue
            if r.status_code >= 500 and idempotent and i + 1 < self.retries:
                time.sleep(0.5 * (2 ** i))
                continue
            if r.status_code >= 400:
                raise AdminClientError(r.status_code, r.text)
            return r
        raise last  # type: ignore[misc]

    def raw(self, method: str, path: str, **kw) -> str:
        """The response body as text (the reference CLI prints some bodies as sent)."""
        return self._call(method, path, idempotent=method in ("GET", "PUT", "DELETE"), **kw).text

    @staticmethod
    def _json(r) -> Any:
        return r.json() if r.content and r.content.strip() else {}

    # tenants
    def tenants(self) -> Dict[str, Any]:
        return self._call("GET", "/api/tenants").json()

    def tenant_put(self, name: str, config: Optional[dict] = None) -> Dict[str, Any]:
        return self._call("PUT", f"/api/tenants/{name}", json=config or {}).json()

    def tenant_create(self, name: str, max_units: Optional[int] = None) -> Dict[str, Any]:
        """POST: fails with 409 when the tenant exists (CreateTenantCmd.java)."""
        return self._json(self._call("POST", f"/api/tenants/{name}", json={"maxTotalResourceUnits": max_units}))

    def tenant_update(self, name: str, max_units: Optional[int] = None) -> Dict[str, Any]:
        """PATCH: fails with 404 when the tenant does not exist (UpdateTenantCmd.java)."""
        return self._json(self._call("PATCH", f"/api/tenants/{name}", json={"maxTotalResourceUnits": max_units}))

    def tenant_get(self, name: str) -> Dict[str, Any]:
        return self._call("GET", f"/api/tenants/{name}").json()

    def tenant_delete(self, name: str) -> None:
        self._call("DELETE", f"/api/tenants/{name}")

    # applications
    def _files(self, app: Optional[str], instance: Optional[str], secrets: Optional[str]):
        files = {}
        if app:
            data = zip_directory(app) if os.path.isdir(app) else open(app, "rb").read()
            files["app"] = ("app.zip", data, "application/zip")
        for name, p in (("instance", instance), ("secrets", secrets)):
            if p:
                if os.path.exists(p):   # ${ENV:-default} / <file:...> (LocalFileReferenceResolver.java)
                    from ..core.file_refs import read_yaml_with_references
                    content = read_yaml_with_references(p)
                else:
                    content = p
                files[name] = (name + ".yaml", content, "text/yaml")
        return files

    def deploy(self, app_id: str, app: Optional[str], instance: Optional[str] = None, secrets: Optional[str] = None,
               dry_run: bool = False, auto_upgrade: bool = False) -> Dict[str, Any]:
        return self._json(self.deploy_raw(app_id, app, instance, secrets, dry_run, auto_upgrade))

    def deploy_raw(self, app_id, app, instance=None, secrets=None, dry_run=False, auto_upgrade=False):
        return self._call("POST", f"/api/applications/{self.tenant}/{app_id}", idempotent=False,
                          params={"dry-run": str(dry_run).lower(), "auto-upgrade": str(auto_upgrade).lower()},
                          files=self._files(app, instance, secrets))

    def update(self, app_id: str, app: Optional[str], instance: Optional[str] = None,
               secrets: Optional[str] = None, auto_upgrade: bool = False,
               force_restart: bool = False) -> Dict[str, Any]:
        return self._json(self._call("PATCH", f"/api/applications/{self.tenant}/{app_id}", idempotent=False,
                                     params={"auto-upgrade": str(auto_upgrade).lower(),
                                             "force-restart": str(force_restart).lower()},
                                     files=self._files(app, instance, secrets)))

    def get(self, app_id: str, stats: bool = False) -> Dict[str, Any]:
        return self._call("GET", f"/api/applications/{self.tenant}/{app_id}",
                          params={"stats": str(stats).lower()}).json()

    def list(self):
        return self._call("GET", f"/api/applications/{self.tenant}").json()

    def delete(self, app_id: str, force: bool = False) -> None:
        self._call("DELETE", f"/api/applications/{self.tenant}/{app_id}", params={"force": str(force).lower()})

    def logs(self, app_id: str, follow: bool = False) -> Iterator[Dict[str, Any]]:
        """The application's log records (NDJSON: timestamp, replica, message)."""
        r = self._call("GET", f"/api/applications/{self.tenant}/{app_id}/logs",
                       params={"follow": str(follow).lower(), "format": "json"}, stream=True)
        for line in r.iter_lines():
            if line:
                rec = json.loads(line)
                if not rec.get("heartbeat"):
                    yield rec

    def log_lines(self, app_id: str, fmt: str = "text", filters=None, follow: bool = True) -> Iterator[str]:
        """GetApplicationLogsCmd: the raw lines in ``text`` or ``json`` format."""
        params = [("format", fmt), ("follow", str(follow).lower())] + [("filter", f) for f in filters or []]
        r = self._call("GET", f"/api/applications/{self.tenant}/{app_id}/logs", params=params, stream=True)
        for line in r.iter_lines(decode_unicode=True):
            if line is not None:
                yield line

    def download_response(self, app_id: str):
        return self._call("GET", f"/api/applications/{self.tenant}/{app_id}/code")

    def download(self, app_id: str) -> bytes:
        return self._call("GET", f"/api/applications/{self.tenant}/{app_id}/code").content

    def archetypes(self):
        return self._call("GET", f"/api/archetypes/{self.tenant}").json()

    def archetype_deploy(self, archetype: str, app_id: str, params: Dict[str, Any]) -> Dict[str, Any]:
        return self._call("POST", f"/api/archetypes/{self.tenant}/{archetype}/applications/{app_id}",
                          idempotent=False, json=params).json()
