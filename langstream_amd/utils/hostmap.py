"""Process-wide host aliases -- the ``docker run --add-host`` of the local runner.

The reference's ``langstream docker run`` maps the Kubernetes service names its example
secrets point at to the container's loopback, where the bundled Kafka, MinIO and HerdDB
listen (``LocalRunApplicationCmd.java:355-361``: ``minio.minio-dev.svc.cluster.local``,
``herddb.herddb-dev.svc.cluster.local``, ``my-cluster-kafka-bootstrap.kafka``).  Here
every service runs in this process (or its replica children), so the same effect is an
alias table consulted by ``socket.getaddrinfo``: ``host`` or ``host:port`` -> ``ip`` or
``ip:port``.  A port-level alias lets a stand-in listen on a free port while the
application keeps the URL it was written with (``...:7000``, ``...:9000``).

Every client in the tree resolves through ``getaddrinfo`` (``socket.create_connection``,
urllib, aiohttp's resolver), so the table covers Kafka, S3, JDBC and HTTP alike.
Children inherit it through ``LANGSTREAM_HOST_ALIASES`` (JSON), applied by
``install_from_env`` at agent-pod start.
"""
from __future__ import annotations

import json
import os
import socket
import threading
from typing import Dict, Optional, Tuple

ENV = "LANGSTREAM_HOST_ALIASES"

_lock = threading.Lock()
_aliases: Dict[str, str] = {}
_orig_getaddrinfo = socket.getaddrinfo


def _split(s: str) -> Tuple[str, Optional[int]]:
    host, sep, port = s.rpartition(":")
    if sep and port.isdigit() and host:
        return host.lower(), int(port)
    return s.lower(), None


def resolve(host: str, port: Optional[int]) -> Tuple[str, Optional[int]]:
    """The (host, port) a connection to ``host:port`` really goes to."""
    if not _aliases or not isinstance(host, str):
        return host, port
    h = host.lower()
    tgt = None
    if port is not None:
        tgt = _aliases.get(f"{h}:{int(port)}")
    if tgt is None:
        tgt = _aliases.get(h)
    if tgt is None:
        return host, port
    th, tp = _split(tgt)
    return th, (tp if tp is not None else port)


def _getaddrinfo(host, port, *args, **kwargs):
    if _aliases and isinstance(host, (str, bytes)):
        h = host.decode() if isinstance(host, bytes) else host
        p = None
        if isinstance(port, int):
            p = port
        elif isinstance(port, (str, bytes)) and str(port if isinstance(port, str) else port.decode()).isdigit():
            p = int(port)
        nh, np_ = resolve(h, p)
        if nh != h or np_ != p:
            host, port = nh, (np_ if np_ is not None else port)
    return _orig_getaddrinfo(host, port, *args, **kwargs)


def add(aliases: Dict[str, str]) -> None:
    """Install (or extend) the alias table and export it to child processes."""
    with _lock:
        for k, v in aliases.items():
            _aliases[k.lower()] = v
        socket.getaddrinfo = _getaddrinfo
        os.environ[ENV] = json.dumps(_aliases, sort_keys=True)


def remove(keys) -> None:
    with _lock:
        for k in keys:
            _aliases.pop(k.lower(), None)
        if _aliases:
            os.environ[ENV] = json.dumps(_aliases, sort_keys=True)
        else:
            os.environ.pop(ENV, None)
            socket.getaddrinfo = _orig_getaddrinfo


def current() -> Dict[str, str]:
    with _lock:
        return dict(_aliases)


def install_from_env() -> None:
    raw = os.environ.get(ENV)
    if raw:
        try:
            add(json.loads(raw))
        except ValueError:
            pass
