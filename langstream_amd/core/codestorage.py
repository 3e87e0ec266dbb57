"""Application code storage (reference ``langstream-api/.../codestorage/
CodeStorage.java`` and the ``langstream-codestorage-providers`` modules).

The control plane stores each uploaded application archive (the zip of the app
directory, incl. ``python/``) in a code storage and hands the resulting *code store id*
to the agents, whose init step (``langstream code-download``) fetches and unpacks it.

Providers (``code_storage_for({"type": ..., "configuration": {...}})``):
* ``local`` / ``disk`` -- a directory (``path``); the default for single-node installs;
* ``memory`` -- in-process (tests, dry runs);
* ``s3`` -- any S3-compatible store (``bucket-name`` default ``langstream-code-storage``,
  ``endpoint``, ``access-key``, ``secret-key``, ``region``), SigV4-signed, bucket created
  on first use (``S3CodeStorage.java``);
* ``azure`` / ``azure-blob-storage`` -- a container (``container`` default
  ``langstream-code-storage``, ``endpoint``, ``sas-token`` | ``storage-account-name`` +
  ``storage-account-key`` | ``storage-account-connection-string``)
  (``AzureBlobCodeStorage.java``).

Objects are keyed ``<tenant>/<tenant>_<application>_<version>_<uuid>`` as in the
reference; the archive's metadata (tenant, application, python-code digest) goes in a
``.json`` sidecar object next to it, so ``describe`` needs no provider-specific object
metadata support.
"""
from __future__ import annotations

import json
import os
import threading
import uuid
from dataclasses import asdict, dataclass
from typing import Any, Dict, Optional


@dataclass
class CodeArchiveMetadata:
    tenant: str
    code_store_id: str
    application_id: str
    py_binaries_digest: Optional[str] = None


class CodeStorage:
    """Blob-level operations; subclasses implement ``_put``/``_get``/``_delete``/``_list``."""

    def _put(self, key: str, data: bytes) -> None:
        raise NotImplementedError

    def _get(self, key: str) -> Optional[bytes]:
        raise NotImplementedError

    def _delete(self, key: str) -> None:
        raise NotImplementedError

    def _list(self, prefix: str):
        raise NotImplementedError

    # ------------------------------------------------------------------ SPI
    def store_application_code(self, tenant: str, application_id: str, version: str, data: bytes,
                               py_binaries_digest: Optional[str] = None) -> CodeArchiveMetadata:
        sid = f"{tenant}_{application_id}_{version}_{uuid.uuid4()}"
        md = CodeArchiveMetadata(tenant, sid, application_id, py_binaries_digest)
        self._put(f"{tenant}/{sid}", data)
        self._put(f"{tenant}/{sid}.json", json.dumps(asdict(md)).encode())
        return md

    def download_application_code(self, tenant: str, code_store_id: str) -> bytes:
        data = self._get(f"{tenant}/{code_store_id}")
        if data is None:
            raise KeyError(f"code archive {code_store_id} not found for tenant {tenant}")
        return data

    def describe_application_code(self, tenant: str, code_store_id: str) -> Optional[CodeArchiveMetadata]:
        raw = self._get(f"{tenant}/{code_store_id}.json")
        return CodeArchiveMetadata(**json.loads(raw)) if raw else None

    def delete_application_code(self, tenant: str, code_store_id: str) -> None:
        self._delete(f"{tenant}/{code_store_id}")
        self._delete(f"{tenant}/{code_store_id}.json")

    def delete_application(self, tenant: str, application_id: str) -> None:
        for k in list(self._list(f"{tenant}/{tenant}_{application_id}_")):
            self._delete(k)

    def close(self) -> None:
        pass


class MemoryCodeStorage(CodeStorage):
    def __init__(self, configuration: Optional[Dict[str, Any]] = None):
        self.blobs: Dict[str, bytes] = {}
        self.lock = threading.Lock()

    def _put(self, key, data):
        with self.lock:
            self.blobs[key] = bytes(data)

    def _get(self, key):
        return self.blobs.get(key)

    def _delete(self, key):
        with self.lock:
            self.blobs.pop(key, None)

    def _list(self, prefix):
        return [k for k in list(self.blobs) if k.startswith(prefix)]


class LocalDiskCodeStorage(CodeStorage):
    def __init__(self, configuration: Optional[Dict[str, Any]] = None):
        self.root = os.path.abspath((configuration or {}).get("path") or "langstream-code-storage")
        os.makedirs(self.root, exist_ok=True)

    def _path(self, key: str) -> str:
        p = os.path.normpath(os.path.join(self.root, key))
        if not p.startswith(self.root + os.sep):
            raise ValueError(f"bad code storage key {key!r}")
        return p

    def _put(self, key, data):
        p = self._path(key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp"
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, p)

    def _get(self, key):
        p = self._path(key)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return f.read()

    def _delete(self, key):
        try:
            os.remove(self._path(key))
        except FileNotFoundError:
            pass

    def _list(self, prefix):
        d = os.path.dirname(self._path(prefix + "x"))
        if not os.path.isdir(d):
            return []
        rel = os.path.relpath(d, self.root)
        return [f"{rel}/{n}" for n in os.listdir(d) if f"{rel}/{n}".startswith(prefix)]


class S3CodeStorage(CodeStorage):
    def __init__(self, configuration: Dict[str, Any]):
        from ..agents.storage import S3Client
        c = configuration or {}
        endpoint = str(c.get("endpoint") or "https://s3.amazonaws.com")
        if "://" not in endpoint:
            endpoint = "https://" + endpoint
        self.bucket = c.get("bucket-name") or c.get("bucketName") or "langstream-code-storage"
        self.client = S3Client(endpoint, c.get("access-key") or "", c.get("secret-key") or "", c.get("region") or "")
        if not self.client.bucket_exists(self.bucket):
            self.client.make_bucket(self.bucket)

    def _put(self, key, data):
        self.client.put_object(self.bucket, key, data)

    def _get(self, key):
        return self.client.get_object(self.bucket, key)

    def _delete(self, key):
        self.client.remove_object(self.bucket, key)

    def _list(self, prefix):
        return [k for k in self.client.list_objects(self.bucket, prefix) if k.startswith(prefix)]


class AzureBlobCodeStorage(CodeStorage):
    def __init__(self, configuration: Dict[str, Any]):
        from ..agents.storage import AzureBlobClient
        c = configuration or {}
        if not c.get("endpoint"):
            raise ValueError("azure code storage: endpoint is required")
        self.client = AzureBlobClient(c["endpoint"], c.get("container") or "langstream-code-storage",
                                      sas_token=c.get("sas-token"), account=c.get("storage-account-name"),
                                      key=c.get("storage-account-key"),
                                      connection_string=c.get("storage-account-connection-string"))
        self.client.create_if_not_exists()

    def _put(self, key, data):
        self.client._req("PUT", key, data=data, ok=(200, 201))

    def _get(self, key):
        try:
            return self.client.download(key)
        except IOError as e:
            if "-> 404" in str(e):
                return None
            raise

    def _delete(self, key):
        self.client.delete(key)

    def _list(self, prefix):
        return [n for n in self.client.list_blobs() if n.startswith(prefix)]


PROVIDERS = {"local": LocalDiskCodeStorage, "disk": LocalDiskCodeStorage, "memory": MemoryCodeStorage,
             "s3": S3CodeStorage, "azure": AzureBlobCodeStorage, "azure-blob-storage": AzureBlobCodeStorage}


def code_storage_for(config: Optional[Dict[str, Any]]) -> CodeStorage:
    """``{"type": "s3", "configuration": {...}}`` (the reference's ``codeStorage`` block);
    a flat map with ``type`` is accepted too."""
    config = dict(config or {"type": "memory"})
    typ = str(config.get("type") or "local")
    if typ not in PROVIDERS:
        raise ValueError(f"unknown code storage type {typ!r}; known: {sorted(PROVIDERS)}")
    inner = config.get("configuration")
    if inner is None:
        inner = {k: v for k, v in config.items() if k != "type"}
    return PROVIDERS[typ](inner)
