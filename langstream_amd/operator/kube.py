"""Minimal Kubernetes REST client for the operator and the k8s application store.

Only what LangStream needs: get / list / server-side apply / merge-patch (incl. the
status subresource) / delete of namespaced objects, addressed by (apiVersion, kind).
In-cluster it reads the service-account token and CA; tests pass an explicit base URL.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional
from urllib.parse import quote

import requests

_SA = "/var/run/secrets/kubernetes.io/serviceaccount"

# kind -> plural resource name
PLURALS = {"Secret": "secrets", "Service": "services", "ConfigMap": "configmaps", "Namespace": "namespaces",
           "StatefulSet": "statefulsets", "Job": "jobs", "Pod": "pods", "PersistentVolumeClaim":
           "persistentvolumeclaims", "Application": "applications", "Agent": "agents"}

CR_API = "langstream.ai/v1alpha1"


class KubeError(RuntimeError):
    def __init__(self, status: int, text: str):
        super().__init__(f"kubernetes API {status}: {text[:300]}")
        self.status = status


class KubeClient:
    def __init__(self, base_url: Optional[str] = None, token: Optional[str] = None, verify: Any = None,
                 field_manager: str = "langstream-operator"):
        if base_url is None:
            host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT", "443")
            if not host:
                raise RuntimeError("not running in a cluster: pass base_url")
            base_url = f"https://{host}:{port}"
            if token is None and os.path.exists(f"{_SA}/token"):
                token = open(f"{_SA}/token").read().strip()
            if verify is None and os.path.exists(f"{_SA}/ca.crt"):
                verify = f"{_SA}/ca.crt"
        self.base = base_url.rstrip("/")
        self.s = requests.Session()
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.s.verify = True if verify is None else verify
        self.field_manager = field_manager

    # ---------------------------------------------------------------- paths
    @staticmethod
    def path(api_version: str, kind: str, namespace: Optional[str] = None, name: Optional[str] = None) -> str:
        prefix = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        p = prefix
        if namespace is not None and kind != "Namespace":
            p += f"/namespaces/{quote(namespace)}"
        p += "/" + PLURALS[kind]
        if name is not None:
            p += "/" + quote(name)
        return p

    def _req(self, method: str, path: str, **kw) -> Any:
        r = self.s.request(method, self.base + path, timeout=30, **kw)
        if r.status_code >= 400:
            raise KubeError(r.status_code, r.text)
        return r.json() if r.content else None

    # ---------------------------------------------------------------- verbs
    def get(self, api_version: str, kind: str, namespace: Optional[str], name: str) -> Optional[Dict[str, Any]]:
        try:
            return self._req("GET", self.path(api_version, kind, namespace, name))
        except KubeError as e:
            if e.status == 404:
                return None
            raise

    def list(self, api_version: str, kind: str, namespace: Optional[str] = None,
             label_selector: Optional[str] = None) -> List[Dict[str, Any]]:
        params = {"labelSelector": label_selector} if label_selector else None
        res = self._req("GET", self.path(api_version, kind, namespace), params=params) or {}
        return list(res.get("items") or [])

    def apply(self, obj: Dict[str, Any]) -> Dict[str, Any]:
        """Server-side apply (PATCH application/apply-patch+yaml; JSON is valid YAML)."""
        md = obj["metadata"]
        p = self.path(obj["apiVersion"], obj["kind"], md.get("namespace"), md["name"])
        return self._req("PATCH", p, params={"fieldManager": self.field_manager, "force": "true"},
                         data=json.dumps(obj), headers={"Content-Type": "application/apply-patch+yaml"})

    def merge_patch(self, api_version: str, kind: str, namespace: Optional[str], name: str, patch: Dict[str, Any],
                    subresource: str = "") -> Dict[str, Any]:
        p = self.path(api_version, kind, namespace, name) + (f"/{subresource}" if subresource else "")
        return self._req("PATCH", p, data=json.dumps(patch), headers={"Content-Type": "application/merge-patch+json"})

    def delete(self, api_version: str, kind: str, namespace: Optional[str], name: str) -> bool:
        try:
            self._req("DELETE", self.path(api_version, kind, namespace, name),
                      data=json.dumps({"propagationPolicy": "Foreground"}),
                      headers={"Content-Type": "application/json"})
            return True
        except KubeError as e:
            if e.status == 404:
                return False
            raise


def owner_ref(obj: Dict[str, Any], controller: bool = True) -> Dict[str, Any]:
    md = obj["metadata"]
    return {"apiVersion": obj["apiVersion"], "kind": obj["kind"], "name": md["name"], "uid": md.get("uid", ""),
            "controller": controller, "blockOwnerDeletion": True}
