"""The services ``langstream run`` starts next to the application -- the reference's
``docker run`` container.

``langstream-runtime-tester/src/main/assemble/entrypoint.sh:18-34`` starts a single-node
Kafka, MinIO and HerdDB inside the container (``START_BROKER`` / ``START_MINIO`` /
``START_HERDDB``, from ``--start-broker`` / ``--start-s3`` / ``--start-database``,
``LocalRunApplicationCmd.java:77-90,329-335``), and the container maps the Kubernetes
service names the example secrets use to its loopback (``:355-361``).  Here:

* broker   -> the in-tree Kafka-protocol broker (``topics/kafka/broker.py``) on 9092
* s3       -> the S3 stand-in (``agents/s3_standalone.py``) on 9000, MinIO's credentials
* database -> the local database service (``agents/vector/herddb.py``) on 7000, sa / hdb

each on its well-known port when that is free, else on a free port; the host aliases
(``utils/hostmap.py``) send ``localhost:<well-known port>`` and the example secrets'
service names (``my-cluster-kafka-bootstrap.kafka:9092``,
``minio.minio-dev.svc.cluster.local:9000``, ``herddb.herddb-dev.svc.cluster.local:7000``)
to wherever the service listens.

``ApplicationWatcher`` is ``--watch-files`` (``LocalRunApplicationCmd.java:401-412``,
``ApplicationWatcher.java:32-100``): a change under the application's ``python/``
directory is copied into the running code directory and the agents are restarted
through the agent-control API (``POST /commands/restart``), which reloads the user's
Python modules.
"""
from __future__ import annotations

import logging
import os
import shutil
import socket
import threading
import time
from typing import Callable, Dict, List, Optional

from ..utils import hostmap

log = logging.getLogger(__name__)

KAFKA_PORT, S3_PORT, DB_PORT = 9092, 9000, 7000
KAFKA_HOSTS = ("localhost", "my-cluster-kafka-bootstrap.kafka")
S3_HOSTS = ("localhost", "minio.minio-dev.svc.cluster.local")
DB_HOSTS = ("localhost", "herddb.herddb-dev.svc.cluster.local")


def _free(host: str, port: int) -> bool:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind((host, port))
        return True
    except OSError:
        return False
    finally:
        s.close()


class LocalServices:
    def __init__(self, broker: bool = True, s3: bool = True, database: bool = True, host: str = "127.0.0.1",
                 well_known_ports: bool = True):
        self.want_broker, self.want_s3, self.want_db = broker, s3, database
        self.host = host
        self.well_known = well_known_ports
        self.broker = self.s3 = self.database = None
        self.aliases: Dict[str, str] = {}

    def _port(self, port: int) -> int:
        return port if self.well_known and _free(self.host, port) else 0

    def start(self) -> "LocalServices":
        if self.want_broker:
            from ..topics.kafka.broker import KafkaBroker
            self.broker = KafkaBroker(self.host, self._port(KAFKA_PORT)).start()
            self._alias(KAFKA_HOSTS, KAFKA_PORT, self.broker.port)
            log.info("Kafka-protocol broker on %s", self.broker.bootstrap)
        if self.want_s3:
            from ..agents.s3_standalone import S3Standalone
            self.s3 = S3Standalone(self.host, self._port(S3_PORT)).start()
            self._alias(S3_HOSTS, S3_PORT, self.s3.port)
            log.info("S3 service on %s", self.s3.endpoint)
        if self.want_db:
            from ..agents.vector.herddb import HerdDBServer
            self.database = HerdDBServer(self.host, self._port(DB_PORT)).start()
            self._alias(DB_HOSTS, DB_PORT, self.database.port)
            log.info("database service on %s:%d", self.database.host, self.database.port)
        if self.aliases:
            hostmap.add(self.aliases)
        return self

    def _alias(self, hosts, port: int, actual: int) -> None:
        for h in hosts:
            if h == "localhost" and actual == port:
                continue
            self.aliases[f"{h}:{port}"] = f"{self.host}:{actual}"

    def default_instance(self) -> str:
        """``LocalRunApplicationCmd.java:226-244``: with the broker, a kafka streaming cluster
        on ``localhost:9092``; without it the reference falls back to ``noop`` ("you won't be
        able to use topics") -- here to the in-process ``memory`` log, which does carry topics."""
        if self.broker is not None:
            return ("instance:\n  streamingCluster:\n    type: \"kafka\"\n    configuration:\n      admin:\n"
                    "        bootstrap.servers: localhost:9092\n")
        return "instance:\n  streamingCluster:\n    type: \"memory\"\n"

    def stop(self) -> None:
        for svc in (self.database, self.s3, self.broker):
            if svc is not None:
                try:
                    svc.stop()
                except Exception:  # noqa: BLE001
                    log.exception("stopping %r", svc)
        if self.aliases:
            hostmap.remove(list(self.aliases))


class ApplicationWatcher:
    """Polls the application directory; python changes -> sync + restart callback."""

    def __init__(self, app_dir: str, code_dir: Optional[str], on_python_change: Callable[[List[str]], None],
                 interval: float = 0.5):
        self.app_dir = os.path.abspath(app_dir)
        self.code_dir = code_dir
        self.on_python_change = on_python_change
        self.interval = interval
        self._stop = threading.Event()
        self._snap = self._scan()
        self._thread: Optional[threading.Thread] = None
        self.restarts = 0

    def _scan(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        for root, dirs, files in os.walk(self.app_dir):
            dirs[:] = [d for d in dirs if d not in ("__pycache__", ".git")]
            for fn in files:
                p = os.path.join(root, fn)
                try:
                    st = os.stat(p)
                    out[p] = (st.st_mtime_ns, st.st_size)
                except OSError:
                    pass
        return out

    def start(self) -> "ApplicationWatcher":
        self._thread = threading.Thread(target=self._run, name="app-watcher", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            snap = self._scan()
            changed = sorted(p for p in set(snap) | set(self._snap) if snap.get(p) != self._snap.get(p))
            self._snap = snap
            if not changed:
                continue
            py_dir = os.path.join(self.app_dir, "python")
            py = [p for p in changed if p.endswith(".py") or p.startswith(py_dir + os.sep)]
            for p in changed:
                if p not in py:
                    print(f"A file has changed: {p}", flush=True)
            if not py:
                continue
            print("A python file has changed, restarting the application", flush=True)
            if self.code_dir and os.path.isdir(py_dir):
                dst = os.path.join(self.code_dir, "python")
                for p in py:
                    rel = os.path.relpath(p, py_dir)
                    if rel.startswith(".."):
                        continue
                    target = os.path.join(dst, rel)
                    if os.path.exists(p):
                        os.makedirs(os.path.dirname(target), exist_ok=True)
                        shutil.copy2(p, target)
                    elif os.path.exists(target):
                        os.remove(target)
            try:
                self.on_python_change(py)
                self.restarts += 1
            except Exception as e:  # noqa: BLE001
                print(f"Could not reload the agents: {e}", flush=True)


def restart_agents(url: str) -> None:
    """``LocalRunApplicationCmd.restartAgents``: POST the agent-control restart command."""
    import urllib.request
    req = urllib.request.Request(url.rstrip("/") + "/commands/restart", data=b"", method="POST")
    with urllib.request.urlopen(req, timeout=60) as r:
        r.read()


def wait_port(host: str, port: int, timeout: float = 10.0) -> bool:
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            socket.create_connection((host, port), timeout=1).close()
            return True
        except OSError:
            time.sleep(0.05)
    return False
