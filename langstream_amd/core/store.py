"""Application stores (``API/storage/ApplicationStore.java:26-91``,
``TESTER/InMemoryApplicationStore.java``, ``CORE/storage/LocalStore.java``).

``ApplicationStore``: put / get / get_specs / get_secrets / delete / list per tenant,
plus a tenant registry (``GlobalMetadataStore`` analogue).  Two implementations:
``InMemoryApplicationStore`` (docker-run mode, tests) and ``LocalDiskApplicationStore``
(JSON + the app's YAML files under a directory, survives restarts of the control plane).
The gateway and the webservice resolve applications through the same store.
"""
from __future__ import annotations

import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

from ..api.model import Application


@dataclass
class StoredApplication:
    application_id: str
    tenant: str
    application: Application
    files: Dict[str, str] = field(default_factory=dict)     # app YAML files (for redeploy / download)
    instance: Optional[str] = None
    secrets: Optional[str] = None
    code_archive_id: Optional[str] = None
    status: str = "CREATED"
    created_at: float = field(default_factory=time.time)
    updated_at: float = field(default_factory=time.time)
    runner: Any = None                                       # live LocalApplicationRunner (not persisted)

    def summary(self) -> Dict[str, Any]:
        return {"application-id": self.application_id, "tenant": self.tenant,
                "status": {"status": {"status": self.status}}, "code-archive-id": self.code_archive_id,
                "created-at": self.created_at, "updated-at": self.updated_at}


class ApplicationStore:
    def put(self, app: StoredApplication) -> None: raise NotImplementedError
    def get(self, tenant: str, application_id: str) -> Optional[StoredApplication]: raise NotImplementedError
    def delete(self, tenant: str, application_id: str) -> bool: raise NotImplementedError
    def list(self, tenant: str) -> List[StoredApplication]: raise NotImplementedError

    # tenants
    def put_tenant(self, tenant: str, config: Optional[dict] = None) -> None: raise NotImplementedError
    def get_tenant(self, tenant: str) -> Optional[dict]: raise NotImplementedError
    def delete_tenant(self, tenant: str) -> bool: raise NotImplementedError
    def list_tenants(self) -> Dict[str, dict]: raise NotImplementedError

    def get_specs(self, tenant: str, application_id: str) -> Optional[Application]:
        a = self.get(tenant, application_id)
        return a.application if a else None


class InMemoryApplicationStore(ApplicationStore):
    def __init__(self, default_tenant: Optional[str] = "default"):
        self._apps: Dict[tuple, StoredApplication] = {}
        self._tenants: Dict[str, dict] = {default_tenant: {"name": default_tenant}} if default_tenant else {}
        self._lock = threading.RLock()

    def put(self, app: StoredApplication) -> None:
        with self._lock:
            app.updated_at = time.time()
            self._apps[(app.tenant, app.application_id)] = app

    def get(self, tenant, application_id):
        with self._lock:
            return self._apps.get((tenant, application_id))

    def delete(self, tenant, application_id) -> bool:
        with self._lock:
            return self._apps.pop((tenant, application_id), None) is not None

    def list(self, tenant):
        with self._lock:
            return [a for (t, _), a in sorted(self._apps.items()) if t == tenant]

    def put_tenant(self, tenant, config=None):
        with self._lock:
            self._tenants[tenant] = dict(config or {}, name=tenant)

    def get_tenant(self, tenant):
        with self._lock:
            return self._tenants.get(tenant)

    def delete_tenant(self, tenant) -> bool:
        with self._lock:
            for k in [k for k in self._apps if k[0] == tenant]:
                del self._apps[k]
            return self._tenants.pop(tenant, None) is not None

    def list_tenants(self):
        with self._lock:
            return dict(self._tenants)


class LocalDiskApplicationStore(InMemoryApplicationStore):
    """In-memory store mirrored to ``<root>/<tenant>/<app>/`` (app.json + YAML files)."""

    def __init__(self, root: str):
        super().__init__()
        self.root = root
        os.makedirs(root, exist_ok=True)
        self._load()

    def _dir(self, tenant, app_id):
        return os.path.join(self.root, tenant, app_id)

    def _load(self) -> None:
        from .parser import build_application_instance
        tf = os.path.join(self.root, "tenants.json")
        if os.path.exists(tf):
            with open(tf) as f:
                self._tenants = json.load(f)
        for tenant in sorted(os.listdir(self.root)):
            td = os.path.join(self.root, tenant)
            if not os.path.isdir(td):
                continue
            for app_id in sorted(os.listdir(td)):
                meta = os.path.join(td, app_id, "app.json")
                if not os.path.exists(meta):
                    continue
                with open(meta) as f:
                    m = json.load(f)
                try:
                    app = build_application_instance(m["files"], m.get("instance"), m.get("secrets")).application
                except Exception:  # noqa: BLE001
                    continue
                self._apps[(tenant, app_id)] = StoredApplication(
                    app_id, tenant, app, m["files"], m.get("instance"), m.get("secrets"), m.get("code-archive-id"),
                    m.get("status", "CREATED"), m.get("created-at", time.time()), m.get("updated-at", time.time()))

    def _save_tenants(self) -> None:
        with open(os.path.join(self.root, "tenants.json"), "w") as f:
            json.dump(self._tenants, f)

    def put(self, app):
        super().put(app)
        d = self._dir(app.tenant, app.application_id)
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "app.json"), "w") as f:
            json.dump({"files": app.files, "instance": app.instance, "secrets": app.secrets,
                       "code-archive-id": app.code_archive_id, "status": app.status, "created-at": app.created_at,
                       "updated-at": app.updated_at}, f)

    def delete(self, tenant, application_id):
        ok = super().delete(tenant, application_id)
        p = os.path.join(self._dir(tenant, application_id), "app.json")
        if os.path.exists(p):
            os.remove(p)
        return ok

    def put_tenant(self, tenant, config=None):
        super().put_tenant(tenant, config)
        self._save_tenants()

    def delete_tenant(self, tenant):
        ok = super().delete_tenant(tenant)
        self._save_tenants()
        return ok
