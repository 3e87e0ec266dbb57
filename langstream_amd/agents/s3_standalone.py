"""An S3-protocol object store for local runs -- the MinIO the reference's ``docker run``
image starts (``langstream-runtime-tester/src/main/assemble/entrypoint.sh:24-28``,
``/minio/minio server /tmp``; toggled by ``--start-s3``, ``LocalRunApplicationCmd.java:82-85``).

    python -m langstream_amd.cli s3-standalone --port 9000

It speaks the path-style REST subset the ``s3-source`` agent, the webcrawler's S3 state
storage and the S3 code storage use: bucket HEAD / PUT / DELETE, ListObjectsV2 (prefix,
max-keys, continuation-token), object GET / HEAD / PUT / DELETE.  Requests must carry a
valid AWS Signature V4 for one of the configured access keys (MinIO's default
``minioadmin`` / ``minioadmin``); the canonical request is rebuilt from what arrived on
the wire (method, URI path, sorted query, the signed headers, ``x-amz-content-sha256``).
Objects live in memory, or under ``data_dir`` (one file per object) when given.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
import os
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional, Tuple
from xml.sax.saxutils import escape

_NS = "http://s3.amazonaws.com/doc/2006-03-01/"


class _Store:
    def __init__(self, data_dir: Optional[str]):
        self.dir = data_dir
        self.lock = threading.Lock()
        self.buckets: Dict[str, Dict[str, Tuple[bytes, str]]] = {}
        if data_dir:
            os.makedirs(data_dir, exist_ok=True)
            for b in sorted(os.listdir(data_dir)):
                bd = os.path.join(data_dir, b)
                if not os.path.isdir(bd):
                    continue
                objs = self.buckets.setdefault(b, {})
                for root, _, files in os.walk(bd):
                    for fn in files:
                        p = os.path.join(root, fn)
                        key = urllib.parse.unquote(os.path.relpath(p, bd))
                        with open(p, "rb") as f:
                            data = f.read()
                        objs[key] = (data, _dt.datetime.utcfromtimestamp(os.path.getmtime(p)).isoformat() + "Z")

    def _path(self, bucket: str, key: str) -> str:
        return os.path.join(self.dir, bucket, urllib.parse.quote(key, safe=""))

    def put(self, bucket: str, key: str, data: bytes) -> None:
        with self.lock:
            self.buckets[bucket][key] = (data, _dt.datetime.utcnow().isoformat(timespec="milliseconds") + "Z")
            if self.dir:
                with open(self._path(bucket, key), "wb") as f:
                    f.write(data)

    def delete(self, bucket: str, key: str) -> None:
        with self.lock:
            self.buckets.get(bucket, {}).pop(key, None)
            if self.dir:
                try:
                    os.remove(self._path(bucket, key))
                except OSError:
                    pass

    def make_bucket(self, bucket: str) -> bool:
        with self.lock:
            if bucket in self.buckets:
                return False
            self.buckets[bucket] = {}
            if self.dir:
                os.makedirs(os.path.join(self.dir, bucket), exist_ok=True)
            return True

    def delete_bucket(self, bucket: str) -> int:
        with self.lock:
            if bucket not in self.buckets:
                return 404
            if self.buckets[bucket]:
                return 409
            del self.buckets[bucket]
            if self.dir:
                try:
                    os.rmdir(os.path.join(self.dir, bucket))
                except OSError:
                    pass
            return 204


def _signing_key(secret: str, date: str, region: str, service: str) -> bytes:
    def h(k: bytes, m: str) -> bytes:
        return hmac.new(k, m.encode(), hashlib.sha256).digest()
    return h(h(h(h(("AWS4" + secret).encode(), date), region), service), "aws4_request")


class S3Standalone:
    def __init__(self, host: str = "127.0.0.1", port: int = 0, credentials: Optional[Dict[str, str]] = None,
                 data_dir: Optional[str] = None, verify_signatures: bool = True):
        self.credentials = dict(credentials or {"minioadmin": "minioadmin"})
        self.verify = verify_signatures
        self.store = _Store(data_dir)
        outer = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, *a):
                pass

            def _send(self, code: int, body: bytes = b"", ctype: str = "application/xml",
                      extra: Optional[Dict[str, str]] = None) -> None:
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                for k, v in (extra or {}).items():
                    self.send_header(k, v)
                self.end_headers()
                if self.command != "HEAD":
                    self.wfile.write(body)

            def _error(self, code: int, s3code: str, msg: str) -> None:
                body = (f'<?xml version="1.0" encoding="UTF-8"?><Error><Code>{s3code}</Code>'
                        f"<Message>{escape(msg)}</Message><Resource>{escape(self.path)}</Resource></Error>").encode()
                self._send(code, body)

            def _body(self) -> bytes:
                n = int(self.headers.get("Content-Length") or 0)
                return self.rfile.read(n) if n else b""

            def _route(self) -> Tuple[str, str, Dict[str, str]]:
                raw_path, _, qs = self.path.partition("?")
                path = urllib.parse.unquote(raw_path).lstrip("/")
                bucket, _, key = path.partition("/")
                q = dict(urllib.parse.parse_qsl(qs, keep_blank_values=True))
                return bucket, key, q

            def _authorized(self, payload: bytes) -> bool:
                if not outer.verify:
                    return True
                auth = self.headers.get("Authorization") or ""
                if not auth.startswith("AWS4-HMAC-SHA256 "):
                    return False
                parts = dict(p.strip().split("=", 1) for p in auth[len("AWS4-HMAC-SHA256 "):].split(",") if "=" in p)
                try:
                    ak, date, region, service, _ = parts["Credential"].split("/")
                    signed = parts["SignedHeaders"].split(";")
                    sig = parts["Signature"]
                except (KeyError, ValueError):
                    return False
                secret = outer.credentials.get(ak)
                if secret is None:
                    return False
                raw_path, _, qs = self.path.partition("?")
                pairs = urllib.parse.parse_qsl(qs, keep_blank_values=True)
                canon_q = "&".join(f"{urllib.parse.quote(k, safe='-_.~')}={urllib.parse.quote(v, safe='-_.~')}"
                                   for k, v in sorted(pairs))
                canon_h = "".join(f"{h}:{(self.headers.get(h) or '').strip()}\n" for h in signed)
                phash = self.headers.get("x-amz-content-sha256") or hashlib.sha256(payload).hexdigest()
                if phash not in ("UNSIGNED-PAYLOAD",) and phash != hashlib.sha256(payload).hexdigest():
                    return False
                canon = "\n".join([self.command, raw_path, canon_q, canon_h, ";".join(signed), phash])
                amz_date = self.headers.get("x-amz-date") or ""
                sts = "\n".join(["AWS4-HMAC-SHA256", amz_date, f"{date}/{region}/{service}/aws4_request",
                                 hashlib.sha256(canon.encode()).hexdigest()])
                want = hmac.new(_signing_key(secret, date, region, service), sts.encode(), hashlib.sha256).hexdigest()
                return hmac.compare_digest(want, sig)

            def _handle(self) -> None:
                payload = self._body() if self.command == "PUT" else b""
                if not self._authorized(payload):
                    return self._error(403, "SignatureDoesNotMatch",
                                       "The request signature we calculated does not match the signature you provided.")
                bucket, key, q = self._route()
                st = outer.store
                if not bucket:
                    if self.command != "GET":
                        return self._error(405, "MethodNotAllowed", "service-level operation")
                    with st.lock:
                        names = sorted(st.buckets)
                    xml = "".join(f"<Bucket><Name>{escape(b)}</Name></Bucket>" for b in names)
                    return self._send(200, (f'<?xml version="1.0" encoding="UTF-8"?><ListAllMyBucketsResult '
                                            f'xmlns="{_NS}"><Buckets>{xml}</Buckets></ListAllMyBucketsResult>').encode())
                exists = bucket in st.buckets
                if not key:
                    if self.command == "HEAD":
                        return self._send(200 if exists else 404)
                    if self.command == "PUT":
                        if not st.make_bucket(bucket):
                            return self._error(409, "BucketAlreadyOwnedByYou", bucket)
                        return self._send(200)
                    if self.command == "DELETE":
                        code = st.delete_bucket(bucket)
                        if code == 204:
                            return self._send(204)
                        return self._error(code, "NoSuchBucket" if code == 404 else "BucketNotEmpty", bucket)
                    if not exists:
                        return self._error(404, "NoSuchBucket", bucket)
                    return self._list(bucket, q)
                if not exists:
                    return self._error(404, "NoSuchBucket", bucket)
                if self.command == "PUT":
                    st.put(bucket, key, payload)
                    return self._send(200, extra={"ETag": '"%s"' % hashlib.md5(payload).hexdigest()})
                if self.command == "DELETE":
                    st.delete(bucket, key)
                    return self._send(204)
                with st.lock:
                    obj = st.buckets[bucket].get(key)
                if obj is None:
                    return self._error(404, "NoSuchKey", key)
                data, _ = obj
                self._send(200, data, "application/octet-stream",
                           {"ETag": '"%s"' % hashlib.md5(data).hexdigest()})

            def _list(self, bucket: str, q: Dict[str, str]) -> None:
                prefix = q.get("prefix", "")
                max_keys = max(1, min(1000, int(q.get("max-keys") or 1000)))
                start = q.get("continuation-token") or q.get("start-after") or ""
                with outer.store.lock:
                    items = sorted((k, v[1], len(v[0]), hashlib.md5(v[0]).hexdigest())
                                   for k, v in outer.store.buckets[bucket].items() if k.startswith(prefix))
                items = [it for it in items if it[0] > start] if start else items
                page, more = items[:max_keys], len(items) > max_keys
                xml = "".join(f"<Contents><Key>{escape(k)}</Key><LastModified>{lm}</LastModified>"
                              f"<ETag>&quot;{et}&quot;</ETag><Size>{n}</Size><StorageClass>STANDARD</StorageClass>"
                              f"</Contents>" for k, lm, n, et in page)
                nxt = f"<NextContinuationToken>{escape(page[-1][0])}</NextContinuationToken>" if more else ""
                body = (f'<?xml version="1.0" encoding="UTF-8"?><ListBucketResult xmlns="{_NS}">'
                        f"<Name>{escape(bucket)}</Name><Prefix>{escape(prefix)}</Prefix><KeyCount>{len(page)}</KeyCount>"
                        f"<MaxKeys>{max_keys}</MaxKeys><IsTruncated>{'true' if more else 'false'}</IsTruncated>"
                        f"{nxt}{xml}</ListBucketResult>").encode()
                self._send(200, body)

            do_GET = do_PUT = do_DELETE = do_HEAD = _handle

        self.httpd = ThreadingHTTPServer((host, port), H)
        self.httpd.daemon_threads = True
        self.host, self.port = self.httpd.server_address[:2]
        self._thread: Optional[threading.Thread] = None

    @property
    def endpoint(self) -> str:
        return f"http://{self.host}:{self.port}"

    def start(self) -> "S3Standalone":
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="s3-standalone", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

    # direct access (tests / local tooling)
    def objects(self, bucket: str) -> List[str]:
        with self.store.lock:
            return sorted(self.store.buckets.get(bucket, {}))


def main(argv=None) -> int:
    import argparse
    import signal
    ap = argparse.ArgumentParser(prog="s3-standalone")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9000)
    ap.add_argument("--data-dir", default=None)
    ap.add_argument("--access-key", default="minioadmin")
    ap.add_argument("--secret-key", default="minioadmin")
    a = ap.parse_args(argv)
    srv = S3Standalone(a.host, a.port, {a.access_key: a.secret_key}, a.data_dir).start()
    print(f"s3-standalone listening on {srv.endpoint}", flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    try:
        while not stop.wait(1.0):
            pass
    except KeyboardInterrupt:
        pass
    srv.stop()
    return 0
