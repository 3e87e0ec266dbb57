"""Kubernetes application store (reference
``langstream-k8s-storage/.../KubernetesApplicationStore.java:89-574``).

Applications live as ``Application`` custom resources in the tenant namespace
``langstream-<tenant>`` (spec: tenant, codeArchiveId, application = JSON of the app's YAML
files + instance, options), their secrets in a ``<app>-secrets`` Secret; the operator
(``operator/__init__.py``) reconciles them.  Tenants are Namespaces plus an entry in
the ``langstream-tenants`` ConfigMap of the system namespace.  Status comes from the CR's
status written by the operator.
"""
from __future__ import annotations

import base64
import json
import time
from typing import Dict, List, Optional

from ..core.parser import build_application_instance
from ..core.store import ApplicationStore, StoredApplication
from .kube import CR_API, KubeClient

TENANTS_CONFIGMAP = "langstream-tenants"


def tenant_namespace(tenant: str, prefix: str = "langstream-") -> str:
    return f"{prefix}{tenant}"


def secrets_name(app_id: str) -> str:
    return f"{app_id}-secrets"


def read_app_secrets(kube: KubeClient, namespace: str, app_id: str) -> Optional[str]:
    s = kube.get("v1", "Secret", namespace, secrets_name(app_id))
    data = (s or {}).get("data") or {}
    return base64.b64decode(data["secrets"]).decode() if data.get("secrets") else None


class KubernetesApplicationStore(ApplicationStore):
    def __init__(self, kube: KubeClient, system_namespace: str = "langstream", namespace_prefix: str = "langstream-"):
        self.kube = kube
        self.system_namespace = system_namespace
        self.prefix = namespace_prefix

    # ------------------------------------------------------------------ apps
    def put(self, app: StoredApplication) -> None:
        ns = tenant_namespace(app.tenant, self.prefix)
        if app.secrets:
            self.kube.apply({"apiVersion": "v1", "kind": "Secret",
                             "metadata": {"name": secrets_name(app.application_id), "namespace": ns},
                             "data": {"secrets": base64.b64encode(app.secrets.encode()).decode()}})
        self.kube.apply({"apiVersion": CR_API, "kind": "Application",
                         "metadata": {"name": app.application_id, "namespace": ns},
                         "spec": {"tenant": app.tenant, "codeArchiveId": app.code_archive_id,
                                  "application": json.dumps({"files": app.files, "instance": app.instance}),
                                  "options": json.dumps({"deleteMode": "CLEANUP_REQUIRED"})}})

    def _to_stored(self, cr) -> StoredApplication:
        md, spec = cr["metadata"], cr["spec"]
        payload = json.loads(spec.get("application") or "{}")
        secrets = read_app_secrets(self.kube, md["namespace"], md["name"])
        built = build_application_instance(payload.get("files") or {}, payload.get("instance"), secrets)
        application = getattr(built, "application", built)
        status = ((cr.get("status") or {}).get("status") or {}).get("status") or "CREATED"
        return StoredApplication(application_id=md["name"], tenant=spec.get("tenant") or "default",
                                 application=application, files=payload.get("files") or {},
                                 instance=payload.get("instance"), secrets=secrets,
                                 code_archive_id=spec.get("codeArchiveId"), status=status)

    def get(self, tenant: str, application_id: str) -> Optional[StoredApplication]:
        cr = self.kube.get(CR_API, "Application", tenant_namespace(tenant, self.prefix), application_id)
        return self._to_stored(cr) if cr else None

    def delete(self, tenant: str, application_id: str) -> bool:
        # the operator's finalizer runs the cleanup (agents, then topics/assets) before the CR goes
        return self.kube.delete(CR_API, "Application", tenant_namespace(tenant, self.prefix), application_id)

    def list(self, tenant: str) -> List[StoredApplication]:
        return [self._to_stored(cr) for cr in
                self.kube.list(CR_API, "Application", tenant_namespace(tenant, self.prefix))]

    # ------------------------------------------------------------------ tenants
    def _tenants_cm(self) -> Dict[str, str]:
        cm = self.kube.get("v1", "ConfigMap", self.system_namespace, TENANTS_CONFIGMAP)
        return dict((cm or {}).get("data") or {})

    def put_tenant(self, tenant: str, config: Optional[dict] = None) -> None:
        self.kube.apply({"apiVersion": "v1", "kind": "Namespace",
                         "metadata": {"name": tenant_namespace(tenant, self.prefix),
                                      "labels": {"langstream.ai/tenant": tenant}}})
        data = self._tenants_cm()
        data[tenant] = json.dumps(dict(config or {}, name=tenant, created=time.time()))
        self.kube.apply({"apiVersion": "v1", "kind": "ConfigMap",
                         "metadata": {"name": TENANTS_CONFIGMAP, "namespace": self.system_namespace}, "data": data})

    def get_tenant(self, tenant: str) -> Optional[dict]:
        v = self._tenants_cm().get(tenant)
        return json.loads(v) if v else None

    def delete_tenant(self, tenant: str) -> bool:
        data = self._tenants_cm()
        if tenant not in data:
            return False
        del data[tenant]
        self.kube.apply({"apiVersion": "v1", "kind": "ConfigMap",
                         "metadata": {"name": TENANTS_CONFIGMAP, "namespace": self.system_namespace}, "data": data})
        self.kube.delete("v1", "Namespace", None, tenant_namespace(tenant, self.prefix))
        return True

    def list_tenants(self) -> Dict[str, dict]:
        return {k: json.loads(v) for k, v in self._tenants_cm().items()}
