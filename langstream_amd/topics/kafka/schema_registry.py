"""Confluent Schema Registry REST client (what CachedSchemaRegistryClient does for the
reference: KRT/KafkaTopicConnectionsRuntime.java:232-325, and inside KafkaAvroSerializer /
KafkaAvroDeserializer) plus a small in-process registry server speaking the same REST
subset, for local runs and tests (there is no Confluent registry offline).

Endpoints used (Confluent REST API v1):
  POST /subjects/{subject}/versions  {"schema": "..."}   -> {"id": n}      (register)
  POST /subjects/{subject}           {"schema": "..."}   -> {"id", "version", ...} (lookup)
  GET  /schemas/ids/{id}                                 -> {"schema": "..."}
  GET  /subjects, /subjects/{subject}/versions, /subjects/{subject}/versions/{v|latest}
Auth: ``basic.auth.user.info`` = "user:password" (basic.auth.credentials.source USER_INFO).
"""
from __future__ import annotations

import base64
import json
import threading
import urllib.error
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, Tuple
from urllib.parse import quote, unquote

from ...api.avro import AvroSchema, parse_schema

CONTENT_TYPE = "application/vnd.schemaregistry.v1+json"


class SchemaRegistryError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"schema registry: HTTP {status}: {message}")
        self.status = status


class SchemaRegistryClient:
    """Caching client: schema -> id per subject, id -> schema (ids are global and
    immutable in a registry, so the caches never go stale)."""

    def __init__(self, url: str, basic_auth: Optional[str] = None, timeout: float = 10.0):
        self.urls = [u.strip().rstrip("/") for u in str(url).split(",") if u.strip()]
        if not self.urls:
            raise ValueError("schema.registry.url is empty")
        self.auth = ("Basic " + base64.b64encode(basic_auth.encode()).decode()) if basic_auth else None
        self.timeout = timeout
        self._by_id: Dict[int, AvroSchema] = {}
        self._ids: Dict[Tuple[str, str], int] = {}
        self._lock = threading.Lock()

    @classmethod
    def from_config(cls, *configs: Dict[str, Any]) -> Optional["SchemaRegistryClient"]:
        """From Kafka client property maps (later maps override earlier ones): needs
        ``schema.registry.url``; optional ``basic.auth.user.info``."""
        merged: Dict[str, Any] = {}
        for c in configs:
            merged.update({k: v for k, v in (c or {}).items() if v is not None})
        url = merged.get("schema.registry.url")
        if not url:
            return None
        auth = merged.get("basic.auth.user.info") or merged.get("schema.registry.basic.auth.user.info")
        return cls(str(url), str(auth) if auth else None)

    def _call(self, method: str, path: str, body: Optional[dict] = None) -> Any:
        data = json.dumps(body).encode() if body is not None else None
        last: Optional[Exception] = None
        for base in self.urls:
            req = urllib.request.Request(base + path, data=data, method=method,
                                         headers={"Content-Type": CONTENT_TYPE, "Accept": CONTENT_TYPE})
            if self.auth:
                req.add_header("Authorization", self.auth)
            try:
                with urllib.request.urlopen(req, timeout=self.timeout) as r:
                    return json.loads(r.read() or b"null")
            except urllib.error.HTTPError as e:
                try:
                    msg = json.loads(e.read() or b"{}").get("message", e.reason)
                except Exception:  # noqa: BLE001
                    msg = e.reason
                raise SchemaRegistryError(e.code, str(msg)) from None
            except OSError as e:              # next url of the list
                last = e
        raise SchemaRegistryError(0, f"unreachable ({last})")

    def register(self, subject: str, schema: Any) -> int:
        sc = parse_schema(schema)
        key = (subject, sc.canonical())
        with self._lock:
            if key in self._ids:
                return self._ids[key]
        out = self._call("POST", f"/subjects/{quote(subject, safe='')}/versions",
                         {"schema": json.dumps(sc.to_json())})
        sid = int(out["id"])
        with self._lock:
            self._ids[key] = sid
            self._by_id.setdefault(sid, sc)
        return sid

    def get_id(self, subject: str, schema: Any) -> int:
        """The id of an already registered schema (auto.register.schemas=false)."""
        sc = parse_schema(schema)
        key = (subject, sc.canonical())
        with self._lock:
            if key in self._ids:
                return self._ids[key]
        out = self._call("POST", f"/subjects/{quote(subject, safe='')}", {"schema": json.dumps(sc.to_json())})
        sid = int(out["id"])
        with self._lock:
            self._ids[key] = sid
        return sid

    def get_by_id(self, sid: int) -> AvroSchema:
        with self._lock:
            sc = self._by_id.get(sid)
        if sc is not None:
            return sc
        out = self._call("GET", f"/schemas/ids/{int(sid)}")
        sc = AvroSchema(out["schema"])
        with self._lock:
            self._by_id[sid] = sc
        return sc

    def subjects(self) -> List[str]:
        return list(self._call("GET", "/subjects"))

    def latest(self, subject: str) -> Dict[str, Any]:
        return self._call("GET", f"/subjects/{quote(subject, safe='')}/versions/latest")


def subject_name(topic: str, is_key: bool) -> str:
    """TopicNameStrategy (the reference's and the serializers' default)."""
    return f"{topic}-{'key' if is_key else 'value'}"


# ------------------------------------------------------------------ in-process registry
class SchemaRegistryServer:
    """A minimal Confluent-compatible registry (the REST subset above, in memory)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, basic_auth: Optional[str] = None):
        self._lock = threading.Lock()
        self.schemas: Dict[int, str] = {}                 # id -> schema json
        self._canon_ids: Dict[str, int] = {}              # canonical form -> id
        self.subjects: Dict[str, List[int]] = {}          # subject -> ids by version
        self.auth = ("Basic " + base64.b64encode(basic_auth.encode()).decode()) if basic_auth else None
        reg = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code: int, body: Any):
                raw = json.dumps(body).encode()
                self.send_response(code)
                self.send_header("Content-Type", CONTENT_TYPE)
                self.send_header("Content-Length", str(len(raw)))
                self.end_headers()
                self.wfile.write(raw)

            def _authorized(self) -> bool:
                if reg.auth and self.headers.get("Authorization") != reg.auth:
                    self._send(401, {"error_code": 401, "message": "Unauthorized"})
                    return False
                return True

            def do_GET(self):
                if not self._authorized():
                    return
                parts = [unquote(p) for p in self.path.split("?")[0].strip("/").split("/")]
                with reg._lock:
                    if parts[:2] == ["schemas", "ids"] and len(parts) == 3:
                        s = reg.schemas.get(int(parts[2]))
                        return self._send(200, {"schema": s}) if s else \
                            self._send(404, {"error_code": 40403, "message": "Schema not found"})
                    if parts == ["subjects"]:
                        return self._send(200, sorted(reg.subjects))
                    if parts[0] == "subjects" and len(parts) >= 3 and parts[2] == "versions":
                        ids = reg.subjects.get(parts[1])
                        if not ids:
                            return self._send(404, {"error_code": 40401, "message": "Subject not found"})
                        if len(parts) == 3:
                            return self._send(200, list(range(1, len(ids) + 1)))
                        v = len(ids) if parts[3] == "latest" else int(parts[3])
                        if not 1 <= v <= len(ids):
                            return self._send(404, {"error_code": 40402, "message": "Version not found"})
                        sid = ids[v - 1]
                        return self._send(200, {"subject": parts[1], "version": v, "id": sid,
                                                "schema": reg.schemas[sid]})
                self._send(404, {"error_code": 404, "message": "Not found"})

            def do_POST(self):
                if not self._authorized():
                    return
                parts = [unquote(p) for p in self.path.split("?")[0].strip("/").split("/")]
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    body = json.loads(self.rfile.read(n) or b"{}")
                    sc = AvroSchema(body["schema"])
                except Exception as e:  # noqa: BLE001
                    return self._send(422, {"error_code": 42201, "message": f"Invalid schema: {e}"})
                canon = sc.canonical()
                with reg._lock:
                    if parts[0] == "subjects" and len(parts) == 3 and parts[2] == "versions":
                        sid = reg._canon_ids.get(canon)
                        if sid is None:
                            sid = len(reg.schemas) + 1
                            reg.schemas[sid] = json.dumps(sc.to_json())
                            reg._canon_ids[canon] = sid
                        ids = reg.subjects.setdefault(parts[1], [])
                        if sid not in ids:
                            ids.append(sid)
                        return self._send(200, {"id": sid})
                    if parts[0] == "subjects" and len(parts) == 2:
                        ids = reg.subjects.get(parts[1], [])
                        sid = reg._canon_ids.get(canon)
                        if sid is None or sid not in ids:
                            return self._send(404, {"error_code": 40403, "message": "Schema not found"})
                        return self._send(200, {"subject": parts[1], "version": ids.index(sid) + 1, "id": sid,
                                                "schema": reg.schemas[sid]})
                self._send(404, {"error_code": 404, "message": "Not found"})

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.url = f"http://{host}:{self.httpd.server_address[1]}"
        self._t = threading.Thread(target=self.httpd.serve_forever, name="schema-registry", daemon=True)
        self._t.start()

    def close(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()
