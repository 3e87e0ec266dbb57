"""Asset managers used at application setup / cleanup (API/runner/assets/AssetManager.java:
initialize, assetExists, deployAsset, deleteAssetIfExists)."""
from __future__ import annotations

import logging
from typing import Any, Dict

log = logging.getLogger(__name__)


class AssetManager:
    def __init__(self, asset):
        self.asset = asset
        self.cfg: Dict[str, Any] = asset.config

    def asset_exists(self) -> bool:
        return False

    def deploy_asset(self) -> None:
        pass

    def delete_asset_if_exists(self) -> None:
        pass


class JdbcTableManager(AssetManager):
    """``jdbc-table`` (``JdbcAssetsManagerProvider.java``): existence from the database's
    table catalogue (name as given, upper- and lower-case), ``create-statements`` on
    deploy, ``delete-statements`` on delete -- only when the table exists, and nothing
    else (no implicit DROP)."""

    def _ds(self):
        from .vector.datasources import jdbc_datasource
        return jdbc_datasource(self.cfg["datasource"])

    def asset_exists(self) -> bool:
        return self._ds().table_exists(self.cfg["table-name"])

    def deploy_asset(self) -> None:
        self._ds().script(list(self.cfg.get("create-statements") or []))

    def delete_asset_if_exists(self) -> None:
        if not self.asset_exists():
            log.info("table %s does not exist, skipping the delete statements", self.cfg["table-name"])
            return
        self._ds().script(list(self.cfg.get("delete-statements") or []))


class VectorCollectionManager(AssetManager):
    def asset_exists(self) -> bool:
        from ..engine.vector_store import VectorStoreRegistry
        return VectorStoreRegistry.exists(self.cfg["collection-name"])

    def deploy_asset(self) -> None:
        from ..engine.vector_store import VectorStoreRegistry
        dim = int(self.cfg.get("dimension") or self.cfg.get("dimensions") or 384)
        VectorStoreRegistry.get(self.cfg["collection-name"], dim)

    def delete_asset_if_exists(self) -> None:
        from ..engine.vector_store import VectorStoreRegistry
        VectorStoreRegistry.drop(self.cfg["collection-name"], purge=True)


class CassandraTableManager(AssetManager):
    """``cassandra-table`` / ``cassandra-keyspace`` / ``astra-keyspace`` (reference
    ``VEC/cassandra/CassandraAssetsManagerProvider.java``): existence from
    ``system_schema``, ``create-statements`` / ``delete-statements`` run as CQL."""

    def _session(self):
        from .vector.cql import session_from_datasource
        ds = dict(self.cfg["datasource"])
        ds.pop("keyspace", None)
        return session_from_datasource(ds)

    def asset_exists(self) -> bool:
        s = self._session()
        try:
            if self.asset.asset_type == "cassandra-table":
                rows = s.execute("SELECT table_name FROM system_schema.tables WHERE keyspace_name = ? AND "
                                 "table_name = ?", [self.cfg["keyspace"], self.cfg["table-name"]])
            else:
                rows = s.execute("SELECT keyspace_name FROM system_schema.keyspaces WHERE keyspace_name = ?",
                                 [self.cfg["keyspace"]])
            return bool(rows)
        finally:
            s.close()

    def deploy_asset(self) -> None:
        s = self._session()
        try:
            for stmt in self.cfg.get("create-statements") or []:
                s.execute(stmt)
        finally:
            s.close()

    def delete_asset_if_exists(self) -> None:
        stmts = self.cfg.get("delete-statements")
        if not stmts:
            stmts = [f"DROP TABLE IF EXISTS {self.cfg['keyspace']}.{self.cfg['table-name']}"] \
                if self.asset.asset_type == "cassandra-table" else [f"DROP KEYSPACE IF EXISTS {self.cfg['keyspace']}"]
        s = self._session()
        try:
            for stmt in stmts:
                s.execute(stmt)
        finally:
            s.close()


class UnavailableAssetManager(AssetManager):
    def asset_exists(self) -> bool:
        raise RuntimeError(f"asset type {self.asset.asset_type} needs its database client and network access, which "
                           f"are not available in this build")

    deploy_asset = asset_exists
    delete_asset_if_exists = asset_exists


class AssetManagerRegistry:
    _types = {"jdbc-table": JdbcTableManager, "vector-collection": VectorCollectionManager,
              "cassandra-table": CassandraTableManager, "cassandra-keyspace": CassandraTableManager,
              "astra-keyspace": CassandraTableManager}

    @classmethod
    def register(cls, asset_type: str, factory) -> None:
        cls._types[asset_type] = factory

    @classmethod
    def create(cls, asset) -> AssetManager:
        factory = cls._types.get(asset.asset_type)
        if factory is None:
            from .vector.remote_assets import MANAGERS
            factory = MANAGERS.get(asset.asset_type, UnavailableAssetManager)
        return factory(asset)
