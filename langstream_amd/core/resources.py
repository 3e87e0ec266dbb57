"""Resource providers (CORE/resources/AIProvidersResourceProvider.java:35-51,
DataSourceResourceProvider.java:27-36, VectorDatabaseResourceProvider.java:31-39).

Validates resource types and returns the configuration handed to agents.  Adds the
MI355X-native ``local-gpu-configuration`` AI resource (in-process GPU engines) and the
``local`` / ``local-gpu`` datasource service (HBM vector store + SQLite tables).
"""
from __future__ import annotations

import copy
from typing import Any, Dict

from ..api.model import Resource

AI_RESOURCE_TYPES = {
    "open-ai-configuration": ("access-key",),
    "hugging-face-configuration": (),
    "vertex-configuration": (),
    "bedrock-configuration": (),
    "ollama-configuration": ("url",),
    "local-gpu-configuration": (),
}
DATASOURCE_SERVICES = ("astra", "astra-vector-db", "cassandra", "jdbc", "opensearch", "pinecone", "milvus", "solr",
                       "local", "local-gpu", "sqlite")
RESOURCE_TYPES = tuple(AI_RESOURCE_TYPES) + ("datasource", "vector-database")


def validate_resource(r: Resource) -> None:
    if r.type not in RESOURCE_TYPES:
        raise ValueError(f"Resource type {r.type} is not supported; known: {sorted(RESOURCE_TYPES)}")
    cfg = r.configuration or {}
    from .config_model import validate_resource as validate_model
    validate_model(r.name or r.id, r.type, cfg)
    if r.type in AI_RESOURCE_TYPES:
        for k in AI_RESOURCE_TYPES[r.type]:
            if r.type == "open-ai-configuration" and cfg.get("provider", "openai") == "local":
                continue
            if cfg.get(k) is None:   # required = present (ClassConfigValidator.java:300-304)
                raise ValueError(f"Resource {r.id} ({r.type}): missing required property '{k}'")
    else:
        svc = cfg.get("service")
        if svc is None:
            raise ValueError(f"Resource {r.id} ({r.type}): missing required property 'service'")
        if svc not in DATASOURCE_SERVICES:
            raise ValueError(f"Resource {r.id}: datasource service {svc} not supported; known: "
                             f"{list(DATASOURCE_SERVICES)}")


def resource_implementation(r: Resource) -> Dict[str, Any]:
    validate_resource(r)
    cfg = copy.deepcopy(r.configuration or {})
    cfg.setdefault("__resource_id", r.id)
    cfg.setdefault("__resource_type", r.type)
    return cfg
