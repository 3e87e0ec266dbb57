"""The local database service behind ``jdbc:herddb:server:`` URLs.

The reference's ``docker run`` image starts a HerdDB server next to the runtime
(``langstream-runtime-tester/src/main/assemble/entrypoint.sh:30-34``, toggled by
``--start-database``, ``LocalRunApplicationCmd.java:87-90``) and maps
``herddb.herddb-dev.svc.cluster.local`` to the container's loopback (``:361``), so the
example secrets' default datasource (``examples/secrets/secrets.yaml:87``:
``jdbc:herddb:server:herddb.herddb-dev.svc.cluster.local:7000``, user ``sa`` / ``hdb``)
works unchanged.  HerdDB's SQL surface in those examples -- ``FLOATA`` columns,
``cosine_similarity(col, CAST(? AS FLOAT ARRAY))`` ordering, composite primary keys,
``UPDATE`` / ``INSERT`` / ``DELETE`` from ``vector-db-sink`` -- is what this service
implements, on SQLite:

* in the process that runs it, ``jdbc:herddb:server:<host>:<port>`` (after the host
  aliases of ``utils/hostmap.py``) resolves to a ``SqliteDataSource`` on the service's
  own database and lock, so ``ORDER BY cosine_similarity(...) DESC LIMIT k`` runs as the
  GPU kNN over the HBM mirror of the vector column (the headline RAG path);
* other processes (replica pods) reach the same database over the service's network
  endpoint, which speaks the PostgreSQL v3 protocol (``pg_standalone.py``) with SCRAM
  authentication of the HerdDB users.  HerdDB's own Netty RPC protocol is not spoken: a
  live HerdDB cluster is not reachable through these URLs, and connecting to one fails at
  the agent's init with that message.
"""
from __future__ import annotations

import re
import threading
from typing import Any, Dict, Optional, Tuple

from .datasources import SqliteDataSource, _cosine
from .pg_standalone import PgStandalone

DEFAULT_PORT = 7000
DEFAULT_USERS = {"sa": "hdb"}

_CAST = re.compile(r"cast\s*\(\s*(\?|\$\d+)\s+as\s+float\s+array\s*\)", re.I)

_lock = threading.Lock()
_servers: Dict[Tuple[str, int], "HerdDBServer"] = {}


_AUTO_PK = re.compile(r"\b(integer|int|long|bigint)\s+auto_increment\s+primary\s+key\b", re.I)
_AUTO = re.compile(r"\s+auto_increment\b", re.I)


def herddb_sql(sql: str) -> str:
    """HerdDB dialect -> SQLite: ``CAST(? AS FLOAT ARRAY)`` binds the JSON vector as is
    (``FLOATA`` columns hold JSON arrays; SQLite keeps any declared type name), and an
    ``integer auto_increment primary key`` column becomes SQLite's rowid alias
    (``INTEGER PRIMARY KEY AUTOINCREMENT``: keys 1, 2, ... as HerdDB generates them)."""
    sql = _CAST.sub(r"\1", sql)
    if "auto_increment" in sql.lower():
        sql = _AUTO.sub("", _AUTO_PK.sub("INTEGER PRIMARY KEY AUTOINCREMENT", sql))
    return sql


def herddb_keys(res: Dict[str, Any]) -> Dict[str, Any]:
    """HerdDB's JDBC driver names the generated-keys column ``key`` whatever the table's
    column is called (JdbcDatabaseIT.testSimpleQueries expects ``{"key": 1}``)."""
    keys = res.get("generatedKeys")
    if isinstance(keys, dict) and keys:
        res["generatedKeys"] = {"key": next(iter(keys.values()))}
    return res


def parse_url(url: str) -> Tuple[str, int]:
    """``jdbc:herddb:server:host[:port][/...]`` -> (host, port); HerdDB's default port 7000.
    (``jdbc:herddb:server:`` also takes comma-separated hosts; the first one is used.)"""
    m = re.match(r"^jdbc:herddb:server:([^/?;]*)", url.strip())
    if not m:
        raise ValueError(f"not a HerdDB server URL: {url!r}")
    hp = m.group(1).split(",")[0] or "localhost"
    host, sep, port = hp.rpartition(":")
    if sep and port.isdigit():
        return host or "localhost", int(port)
    return hp, DEFAULT_PORT


class HerdDBServer:
    """One local database: a shared-cache SQLite database, served in-process and over the
    PostgreSQL-protocol endpoint on ``host:port`` (0 = a free port)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, users: Optional[Dict[str, str]] = None):
        self.uri = f"file:herddb{id(self)}?mode=memory&cache=shared"
        self.lock = threading.RLock()
        self._ds: Optional[SqliteDataSource] = None
        self.pg = PgStandalone(host, port, users=dict(users or DEFAULT_USERS), auth="scram-sha-256",
                               db_uri=self.uri, functions={"cosine_similarity": (2, _cosine)},
                               rewrite=herddb_sql, on_write=self._on_write, db_lock=self.lock,
                               server_version="16.0 (langstream herddb service)")
        self.host, self.port = self.pg.host, self.pg.port

    def start(self) -> "HerdDBServer":
        self.pg.start()
        with _lock:
            _servers[(self.host, self.port)] = self
        return self

    def stop(self) -> None:
        with _lock:
            for k, v in list(_servers.items()):
                if v is self:
                    del _servers[k]
        self.pg.stop()

    @property
    def url(self) -> str:
        return f"jdbc:herddb:server:{self.host}:{self.port}"

    def datasource(self, cfg: Optional[Dict[str, Any]] = None) -> SqliteDataSource:
        with _lock:
            if self._ds is None:
                self._ds = _HerdDBDataSource(dict(cfg or {"url": self.url}), uri=self.uri, lock=self.lock)
            return self._ds

    def _on_write(self, sql: str) -> None:
        # a wire client changed a table: the in-process kNN mirrors of it are stale
        if self._ds is not None:
            self._ds._invalidate_mirrors_for(sql)


class _HerdDBDataSource(SqliteDataSource):
    def fetch_data(self, query, params):
        return super().fetch_data(herddb_sql(query), params)

    def execute_statement(self, query, generated_keys, params):
        return herddb_keys(super().execute_statement(herddb_sql(query), generated_keys, params))

    def script(self, statements):
        return super().script([herddb_sql(s) for s in statements])


def local_server(host: str, port: int) -> Optional[HerdDBServer]:
    """The in-process service ``host:port`` reaches (through the host aliases), if any."""
    from ...utils import hostmap
    h, p = hostmap.resolve(host, port)
    p = int(p if p is not None else port)
    with _lock:
        srv = _servers.get((h, p))
        if srv is None and h in ("localhost", "127.0.0.1", "0.0.0.0", "::1"):
            srv = next((s for (sh, sp), s in _servers.items() if sp == p), None)
        return srv


def _remote_class():
    from .pgwire import PgConnection, PostgresDataSource

    class RemoteHerdDBDataSource(PostgresDataSource):
        """A ``jdbc:herddb:server:`` URL served by another process's database service."""

        def __init__(self, cfg: Dict[str, Any], host: str, port: int):
            self.url = str(cfg.get("url"))
            self.props = {}
            self.host, self.port = host, port
            self.user, self.password = str(cfg.get("user") or "sa"), cfg.get("password") or "hdb"
            self._conn = None
            self._lock = threading.Lock()
            try:
                self.conn()
            except (ConnectionError, OSError) as e:
                raise ConnectionError(
                    f"{self.url}: no local database service answers on {host}:{port} ({e}); "
                    f"jdbc:herddb:server: URLs are served by `langstream run --start-database` "
                    f"(a live HerdDB server's own protocol is not spoken by this build)") from e

        def conn(self):
            with self._lock:
                if self._conn is None:
                    self._conn = PgConnection(self.host, self.port, self.user, self.password, "herd")
                return self._conn

        def fetch_data(self, query, params):
            return super().fetch_data(herddb_sql(query), params)

        def execute_statement(self, query, generated_keys, params):
            return herddb_keys(super().execute_statement(herddb_sql(query), generated_keys, params))

        def script(self, statements):
            return super().script([herddb_sql(x) for x in statements])

    return RemoteHerdDBDataSource


_remote: Dict[Tuple[str, int, str], Any] = {}


def herddb_datasource(cfg: Dict[str, Any]):
    url = str(cfg.get("url") or "")
    host, port = parse_url(url)
    srv = local_server(host, port)
    if srv is not None:
        user, pw = str(cfg.get("user") or "sa"), str(cfg.get("password") or "hdb")
        if srv.pg.users.get(user) != pw:
            raise PermissionError(f"{url}: authentication failed for user {user!r}")
        return srv.datasource(cfg)
    key = (host, port, str(cfg.get("user")))
    with _lock:
        ds = _remote.get(key)
    if ds is None:
        ds = _remote_class()(cfg, host, port)
        with _lock:
            ds = _remote.setdefault(key, ds)
    return ds


def reset() -> None:
    """Close remote connections (tests)."""
    with _lock:
        for ds in _remote.values():
            try:
                ds.close()
            except Exception:  # noqa: BLE001
                pass
        _remote.clear()
