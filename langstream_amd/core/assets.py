"""Planner-side asset providers (CORE/assets/*.java) and the asset manager SPI used at
setup/cleanup time (API/runner/assets/*).

Asset types: cassandra-table, cassandra-keyspace, astra-keyspace, jdbc-table,
milvus-collection, opensearch-index, solr-collection, astra-collection, plus the
MI355X-native ``vector-collection`` (an HBM vector-store collection).
External-database assets validate here; their managers need the database clients,
which are gated at runtime (``agents.vector.datasources``).
"""
from __future__ import annotations

from typing import Any, Dict

from ..api.model import Application, AssetDefinition

ASSET_REQUIRED = {
    "cassandra-table": ("table-name", "keyspace", "datasource", "create-statements"),
    "cassandra-keyspace": ("keyspace", "datasource", "create-statements"),
    "astra-keyspace": ("keyspace", "datasource"),
    "jdbc-table": ("table-name", "datasource", "create-statements"),
    "milvus-collection": ("collection-name", "datasource", "create-statements"),
    "opensearch-index": ("datasource",),            # index-name comes from the datasource
    "solr-collection": ("datasource", "create-statements"),
    "astra-collection": ("collection-name", "datasource", "vector-dimension"),
    "vector-collection": ("collection-name", "datasource"),
}


def validate_asset(asset: AssetDefinition, app: Application) -> Dict[str, Any]:
    if asset.asset_type not in ASSET_REQUIRED:
        raise ValueError(f"Asset type {asset.asset_type} is not supported; known: {sorted(ASSET_REQUIRED)}")
    from .config_model import validate_asset as validate_model
    cfg = validate_model(asset.name or asset.id, asset.asset_type, dict(asset.config or {}))
    for k in ASSET_REQUIRED[asset.asset_type]:
        if cfg.get(k) is None:
            raise ValueError(f"Asset {asset.id} ({asset.asset_type}): missing required property '{k}'")
    ds = cfg.get("datasource")
    if isinstance(ds, str):
        from .genai import resolve_datasource
        cfg["datasource"] = resolve_datasource(ds, app)
    return cfg
