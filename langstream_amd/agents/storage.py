"""Object-storage and Camel sources + the small S3 / Azure Blob REST
clients they (and the webcrawler's S3 state storage) use.

Parity:
* s3-source (``S3Source.java:40-250``): ``bucketName`` (langstream-source),
  ``endpoint``, ``access-key``/``secret-key`` (minioadmin), ``region``, ``idle-time``
  (5 s), ``file-extensions`` ("pdf,docx,html,htm,md,txt", ``*`` = all).  The bucket is
  created if missing; ``read()`` returns ONE not-yet-emitted object (key = object name,
  value = bytes, header ``name``); ``commit()`` DELETES the object.
* azure-blob-storage-source (``AzureBlobStorageSource.java``): ``container``
  (langstream-azure-source), required ``endpoint``, auth by ``sas-token`` or
  ``storage-account-name``/``storage-account-key`` or
  ``storage-account-connection-string``; same read/commit contract.
* camel-source (``CamelSource.java:160-260``): ``component-uri`` +
  ``component-options`` (appended as query parameters), ``max-buffered-records``
  (100), ``key-header``.  Apache Camel is a JVM library, so the rebuild implements
  the commonly used consumer components natively: ``file:<dir>`` (poll a directory;
  commit deletes, or moves to ``.camel/`` with ``noop=false&move=...``), and
  ``timer:<name>?period=<ms>&repeatCount=<n>``.  Other schemes fail at init.

The clients speak plain HTTPS REST (no SDK is available offline): AWS Signature V4 for
S3 (path-style, MinIO compatible) and SharedKey / SAS for Azure Blob.
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import hmac
import logging
import json
import os
import queue
import threading
import time
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Any, Dict, List, Optional, Set

from ..api.agent import AgentSource
from ..api.record import Header, Record, SimpleRecord
from ..api.util import get_int, get_map, get_string, required_non_empty_field
from ..runtime.registry import register_agent

log = logging.getLogger(__name__)

ALL_FILES = "*"
DEFAULT_EXTENSIONS = "pdf,docx,html,htm,md,txt"


def extension_allowed(name: str, extensions: Set[str]) -> bool:
    if ALL_FILES in extensions:
        return True
    i = name.rfind(".")
    ext = "" if i < 0 or i == len(name) - 1 else name[i + 1:]
    return ext in extensions


# ---------------------------------------------------------------- S3 (SigV4, path style)
class S3Client:
    def __init__(self, endpoint: str, access_key: str, secret_key: str, region: str = ""):
        import requests
        self.endpoint = endpoint.rstrip("/")
        self.ak, self.sk = access_key, secret_key
        self.region = region or "us-east-1"
        self.http = requests.Session()

    def _sign(self, method: str, path: str, query: Dict[str, str], payload: bytes) -> Dict[str, str]:
        u = urllib.parse.urlparse(self.endpoint)
        now = _dt.datetime.now(_dt.timezone.utc)
        amz_date = now.strftime("%Y%m%dT%H%M%SZ")
        date = now.strftime("%Y%m%d")
        phash = hashlib.sha256(payload).hexdigest()
        canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(str(v), safe='-_.~')}"
                           for k, v in sorted(query.items()))
        headers = {"host": u.netloc, "x-amz-content-sha256": phash, "x-amz-date": amz_date}
        signed = ";".join(sorted(headers))
        canon_h = "".join(f"{k}:{headers[k]}\n" for k in sorted(headers))
        canon = "\n".join([method, urllib.parse.quote(path, safe="/-_.~"), canon_q, canon_h, signed, phash])
        scope = f"{date}/{self.region}/s3/aws4_request"
        sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, scope, hashlib.sha256(canon.encode()).hexdigest()])

        def h(k, m):
            return hmac.new(k, m.encode(), hashlib.sha256).digest()

        key = h(h(h(h(("AWS4" + self.sk).encode(), date), self.region), "s3"), "aws4_request")
        sig = hmac.new(key, sts.encode(), hashlib.sha256).hexdigest()
        headers["Authorization"] = (f"AWS4-HMAC-SHA256 Credential={self.ak}/{scope}, SignedHeaders={signed}, "
                                    f"Signature={sig}")
        return headers

    def _req(self, method: str, bucket: str, key: str = "", query: Optional[Dict[str, str]] = None,
             data: bytes = b"", ok=(200, 204)):
        path = f"/{bucket}" + (f"/{key}" if key else "")
        query = query or {}
        headers = self._sign(method, path, query, data)
        url = self.endpoint + urllib.parse.quote(path, safe="/-_.~")
        r = self.http.request(method, url, params=query, data=data, headers=headers, timeout=60)
        if r.status_code not in ok:
            raise IOError(f"S3 {method} {path} -> {r.status_code}: {r.text[:200]}")
        return r

    def bucket_exists(self, bucket: str) -> bool:
        try:
            self._req("HEAD", bucket)
            return True
        except IOError:
            return False

    def make_bucket(self, bucket: str) -> None:
        self._req("PUT", bucket, ok=(200, 204, 409))

    def list_objects(self, bucket: str, prefix: str = "") -> List[str]:
        out, token = [], None
        while True:
            q = {"list-type": "2"}
            if prefix:
                q["prefix"] = prefix
            if token:
                q["continuation-token"] = token
            root = ET.fromstring(self._req("GET", bucket, query=q).content)
            ns = root.tag[: root.tag.index("}") + 1] if root.tag.startswith("{") else ""
            out += [c.findtext(f"{ns}Key") for c in root.findall(f"{ns}Contents")]
            if (root.findtext(f"{ns}IsTruncated") or "false").lower() != "true":
                return out
            token = root.findtext(f"{ns}NextContinuationToken")

    def get_object(self, bucket: str, key: str) -> Optional[bytes]:
        try:
            return self._req("GET", bucket, key).content
        except IOError as e:
            if "-> 404" in str(e):
                return None
            raise

    def put_object(self, bucket: str, key: str, data: bytes) -> None:
        self._req("PUT", bucket, key, data=data)

    def remove_object(self, bucket: str, key: str) -> None:
        self._req("DELETE", bucket, key, ok=(200, 204, 404))


# ---------------------------------------------------------------- Azure Blob (SharedKey / SAS)
class AzureBlobClient:
    def __init__(self, endpoint: str, container: str, sas_token: Optional[str] = None,
                 account: Optional[str] = None, key: Optional[str] = None, connection_string: Optional[str] = None):
        import requests
        if connection_string:
            parts = dict(p.split("=", 1) for p in connection_string.split(";") if "=" in p)
            account, key = parts.get("AccountName"), parts.get("AccountKey")
        if not sas_token and not account:
            raise ValueError("Either sas-token, account-name/account-key or account-connection-string must be "
                             "provided")
        self.endpoint = endpoint.rstrip("/")
        self.container = container
        self.sas = sas_token.lstrip("?") if sas_token else None
        self.account, self.key = account, key
        self.http = requests.Session()

    def _headers(self, method: str, path: str, query: Dict[str, str], length: int) -> Dict[str, str]:
        h = {"x-ms-date": _dt.datetime.now(_dt.timezone.utc).strftime("%a, %d %b %Y %H:%M:%S GMT"),
             "x-ms-version": "2021-08-06"}
        if method == "PUT" and "comp" not in query and "restype" not in query:
            h["x-ms-blob-type"] = "BlockBlob"
        if self.sas:
            return h
        canon_h = "".join(f"{k}:{v}\n" for k, v in sorted(h.items()))
        canon_r = f"/{self.account}{path}" + "".join(f"\n{k}:{v}" for k, v in sorted(query.items()))
        sts = "\n".join([method, "", "", str(length) if length else "", "", "", "", "", "", "", "", ""]) + "\n" \
            + canon_h + canon_r
        sig = base64.b64encode(hmac.new(base64.b64decode(self.key), sts.encode(), hashlib.sha256).digest()).decode()
        h["Authorization"] = f"SharedKey {self.account}:{sig}"
        return h

    def _req(self, method: str, blob: str = "", query: Optional[Dict[str, str]] = None, data: bytes = b"",
             ok=(200, 201, 202)):
        query = dict(query or {})
        path = f"/{self.container}" + (f"/{blob}" if blob else "")
        url = self.endpoint + urllib.parse.quote(path)
        params = dict(query)
        if self.sas:
            params.update(urllib.parse.parse_qsl(self.sas))
        r = self.http.request(method, url, params=params, data=data,
                              headers=self._headers(method, path, query, len(data)), timeout=60)
        if r.status_code not in ok:
            raise IOError(f"Azure {method} {path} -> {r.status_code}: {r.text[:200]}")
        return r

    def create_if_not_exists(self) -> None:
        self._req("PUT", query={"restype": "container"}, ok=(201, 409))

    def list_blobs(self) -> List[str]:
        root = ET.fromstring(self._req("GET", query={"restype": "container", "comp": "list"}).content)
        return [b.findtext("Name") for b in root.iter("Blob")]

    def download(self, name: str) -> bytes:
        return self._req("GET", name).content

    def delete(self, name: str) -> None:
        self._req("DELETE", name, ok=(202, 404))


# ---------------------------------------------------------------- sources
class _ObjectRecord(SimpleRecord):
    def __init__(self, name: str, data: bytes):
        super().__init__(name, data, None, int(time.time() * 1000), [Header("name", name)])
        self.object_name = name


class _BlobSourceBase(AgentSource):
    """read(): one not-yet-emitted object; commit(): delete it."""

    def _configure_common(self, configuration: Dict[str, Any]) -> None:
        self.idle_time = get_int("idle-time", 5, configuration)
        self.extensions = set(str(configuration.get("file-extensions", DEFAULT_EXTENSIONS)).split(","))
        self.to_commit: Set[str] = set()
        self._lock = threading.Lock()

    def _list(self) -> List[str]:
        raise NotImplementedError

    def _get(self, name: str) -> bytes:
        raise NotImplementedError

    def _delete(self, name: str) -> None:
        raise NotImplementedError

    def read(self) -> List[Record]:
        for name in self._list():
            if name.endswith("/") or not extension_allowed(name, self.extensions):
                continue
            with self._lock:
                if name in self.to_commit:
                    continue
                self.to_commit.add(name)
            self.processed(0, 1)
            return [_ObjectRecord(name, self._get(name))]
        time.sleep(self.idle_time)
        return []

    def commit(self, records: List[Record]) -> None:
        for r in records:
            name = getattr(r, "object_name", None) or r.key()
            self._delete(name)
            with self._lock:
                self.to_commit.discard(name)


@register_agent("s3-source")
class S3Source(_BlobSourceBase):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.bucket = get_string("bucketName", "langstream-source", configuration)
        self.client = S3Client(get_string("endpoint", "http://minio-endpoint.-not-set:9090", configuration),
                               get_string("access-key", "minioadmin", configuration),
                               get_string("secret-key", "minioadmin", configuration),
                               get_string("region", "", configuration))
        self._configure_common(configuration)

    def start(self) -> None:
        if not self.client.bucket_exists(self.bucket):
            self.client.make_bucket(self.bucket)

    def _list(self):
        return self.client.list_objects(self.bucket)

    def _get(self, name):
        return self.client.get_object(self.bucket, name) or b""

    def _delete(self, name):
        self.client.remove_object(self.bucket, name)

    def build_additional_info(self):
        return {"bucketName": self.bucket}


@register_agent("azure-blob-storage-source")
class AzureBlobStorageSource(_BlobSourceBase):
    def init(self, configuration: Dict[str, Any]) -> None:
        self.client = AzureBlobClient(
            required_non_empty_field(configuration, "endpoint", "azure blob storage source"),
            get_string("container", "langstream-azure-source", configuration),
            get_string("sas-token", None, configuration), get_string("storage-account-name", None, configuration),
            get_string("storage-account-key", None, configuration),
            get_string("storage-account-connection-string", None, configuration))
        self._configure_common(configuration)

    def start(self) -> None:
        self.client.create_if_not_exists()

    def _list(self):
        return self.client.list_blobs()

    def _get(self, name):
        return self.client.download(name)

    def _delete(self, name):
        self.client.delete(name)

    def build_additional_info(self):
        return {"container": self.client.container}


@register_agent("camel-source")
class CamelSource(AgentSource):
    def init(self, configuration: Dict[str, Any]) -> None:
        uri = get_string("component-uri", "", configuration)
        opts = get_map("component-options", {}, configuration)
        for k, v in opts.items():
            if v is not None:
                uri += ("&" if "?" in uri else "?") + f"{k}={urllib.parse.quote_plus(str(v))}"
        self.uri = uri
        self.key_header = get_string("key-header", "", configuration)
        self.q: "queue.Queue" = queue.Queue(maxsize=get_int("max-buffered-records", 100, configuration))
        scheme, _, rest = uri.partition(":")
        self.scheme = scheme
        path, _, qs = rest.partition("?")
        self.path = path.lstrip("/") if scheme == "timer" else path
        self.params = dict(urllib.parse.parse_qsl(qs))
        if scheme not in CAMEL_COMPONENTS:
            raise ValueError(f"camel-source: component '{scheme}' is not supported natively "
                             f"(supported: {', '.join(sorted(CAMEL_COMPONENTS))})")
        self._stop = threading.Event()
        self._inflight: Set[str] = set()

    def start(self) -> None:
        self._thread = threading.Thread(target=self._run, daemon=True, name="camel-" + self.scheme)
        self._thread.start()

    def close(self) -> None:
        self._stop.set()

    def _emit(self, key, value, headers: Dict[str, Any]) -> None:
        if self.key_header and self.key_header in headers:
            key = headers[self.key_header]
        hs = [Header(k, v if isinstance(v, (str, int, float, bool)) or v is None else str(v))
              for k, v in headers.items()]
        while not self._stop.is_set():
            try:
                self.q.put(SimpleRecord(key, value, None, int(time.time() * 1000), hs), timeout=0.5)
                return
            except queue.Full:
                continue

    def _run(self) -> None:
        if self.scheme in ("github", "kafka"):
            try:
                CAMEL_COMPONENTS[self.scheme](self)
            except Exception as e:  # noqa: BLE001
                log.exception("camel %s consumer failed", self.scheme)
                self._error = e
            return
        if self.scheme in ("timer", "scheduler"):
            period = float(self.params.get("period", 1000)) / 1000.0
            repeat = int(self.params.get("repeatCount", 0))
            n = 0
            while not self._stop.is_set() and (repeat <= 0 or n < repeat):
                n += 1
                self._emit(None, "", {"CamelTimerName": self.path, "CamelTimerCounter": n,
                                      "CamelTimerFiredTime": int(time.time() * 1000)})
                self._stop.wait(period)
            return
        directory = self.path
        delay = float(self.params.get("delay", 500)) / 1000.0
        while not self._stop.is_set():
            try:
                names = sorted(os.listdir(directory))
            except OSError:
                names = []
            for fn in names:
                full = os.path.join(directory, fn)
                if fn.startswith(".") or not os.path.isfile(full) or full in self._inflight:
                    continue
                self._inflight.add(full)
                with open(full, "rb") as f:
                    data = f.read()
                self._emit(fn, data, {"CamelFileName": fn, "CamelFileAbsolutePath": os.path.abspath(full),
                                      "CamelFileLength": len(data)})
            self._stop.wait(delay)

    def read(self) -> List[Record]:
        err = getattr(self, "_error", None)
        if err is not None:
            raise err
        try:
            r = self.q.get(timeout=1.0)
        except queue.Empty:
            return []
        self.processed(0, 1)
        return [r]

    def commit(self, records: List[Record]) -> None:
        if self.scheme != "file":
            return
        for r in records:
            path = r.header_value("CamelFileAbsolutePath")
            if not path:
                continue
            if str(self.params.get("noop", "false")).lower() == "true":
                continue
            move = self.params.get("move")
            try:
                if move:
                    dst = os.path.join(os.path.dirname(path), move)
                    os.makedirs(dst, exist_ok=True)
                    os.replace(path, os.path.join(dst, os.path.basename(path)))
                else:
                    os.remove(path)
            except OSError:
                log.warning("camel file: could not finish %s", path)
            self._inflight.discard(path)

    def build_additional_info(self):
        return {"component-uri": self.uri}


def _camel_github(src: "CamelSource") -> None:
    """camel-github consumer: ``github:<type>[/<branch>]?repoOwner=&repoName=&oauthToken=``
    with type PULLREQUESTCOMMENT | PULLREQUEST | COMMIT | TAG | EVENT; polls the GitHub REST
    API every ``delay`` ms (default 5000) and emits each NEW item once (the first poll only
    records what exists, as the Camel consumer does).  ``apiUrl`` overrides the API base."""
    import requests
    typ, _, branch = src.path.partition("/")
    typ = typ.upper()
    p = src.params
    owner, repo = p.get("repoOwner"), p.get("repoName")
    if not owner or not repo:
        raise ValueError("camel github: repoOwner and repoName are required")
    base = p.get("apiUrl", "https://api.github.com").rstrip("/")
    paths = {"PULLREQUESTCOMMENT": f"/repos/{owner}/{repo}/pulls/comments",
             "PULLREQUEST": f"/repos/{owner}/{repo}/pulls", "COMMIT": f"/repos/{owner}/{repo}/commits",
             "TAG": f"/repos/{owner}/{repo}/tags", "EVENT": f"/repos/{owner}/{repo}/events"}
    if typ not in paths:
        raise ValueError(f"camel github: unsupported type {typ}; known: {sorted(paths)}")
    params = {"sha": branch or p.get("branch")} if typ == "COMMIT" and (branch or p.get("branch")) else {}
    headers = {"Accept": "application/vnd.github+json"}
    if p.get("oauthToken"):
        headers["Authorization"] = f"Bearer {p['oauthToken']}"
    delay = float(p.get("delay", 5000)) / 1000.0
    seen: Set[str] = set()
    first = True
    while not src._stop.is_set():
        r = requests.get(base + paths[typ], params=params, headers=headers, timeout=30)
        r.raise_for_status()
        for item in reversed(r.json()):     # oldest first
            ident = str(item.get("id") or item.get("sha") or item.get("name") or json.dumps(item, sort_keys=True))
            if ident in seen:
                continue
            seen.add(ident)
            if not first:
                src._emit(ident, json.dumps(item), {"GitHubType": typ, "GitHubId": ident})
        first = False
        src._stop.wait(delay)


def _camel_kafka(src: "CamelSource") -> None:
    """camel-kafka consumer: ``kafka:<topic>?brokers=host:port[&groupId=..]`` through the
    in-tree Kafka client (consumer group, earliest reset, commit after emission)."""
    from ..topics.kafka.client import GroupConsumer, KafkaClient
    brokers = src.params.get("brokers")
    if not brokers:
        raise ValueError("camel kafka: brokers is required")
    client = KafkaClient(brokers, client_id="camel-kafka")
    c = GroupConsumer(client, src.path, src.params.get("groupId", "camel-" + src.path),
                      src.params.get("autoOffsetReset", "earliest"))
    c.start()
    try:
        while not src._stop.is_set():
            recs = c.poll(500)
            for part, off, ts, k, v, hs in recs:
                key = k.decode("utf-8", "replace") if isinstance(k, bytes) else k
                src._emit(key, v, {"kafka.TOPIC": src.path, "kafka.PARTITION": part, "kafka.OFFSET": off,
                                   **{hk: (hv.decode("utf-8", "replace") if isinstance(hv, bytes) else hv)
                                      for hk, hv in hs}})
            if recs:
                c.commit([(p_, o_) for p_, o_, *_ in recs])
    finally:
        c.close()
        client.close()


# Camel component URI schemes this runtime implements natively; register more here.
CAMEL_COMPONENTS = {"file": None, "timer": None, "scheduler": None, "github": _camel_github, "kafka": _camel_kafka}
