"""Code storage providers (local disk, memory, S3 against an in-test S3, Azure Blob against
an in-test blob service) and the control plane / code-download CLI using them.
Mirrors the reference's S3CodeStorageTest / AzureBlobCodeStorageTest (MinIO / Azurite
containers there; in-process fakes here)."""
import io
import os
import threading
import zipfile
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlsplit

import pytest

from langstream_amd.core.codestorage import code_storage_for
from test_sources import _FakeS3, _serve


class _FakeAzure(BaseHTTPRequestHandler):
    store = {}

    def log_message(self, *a):
        pass

    def _ok(self, body=b"", code=200):
        self.send_response(code)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)

    def _parts(self):
        u = urlsplit(self.path)
        assert "sig" in parse_qs(u.query)            # SAS token travels as query parameters
        seg = u.path.strip("/").split("/", 1)
        return seg[0], (seg[1] if len(seg) > 1 else ""), parse_qs(u.query)

    def do_PUT(self):
        c, b, q = self._parts()
        data = self.rfile.read(int(self.headers.get("Content-Length") or 0))
        if q.get("restype") == ["container"]:
            code = 409 if c in self.store else 201
            self.store.setdefault(c, {})
            return self._ok(code=code)
        assert self.headers.get("x-ms-blob-type") == "BlockBlob"
        self.store[c][b] = data
        self._ok(code=201)

    def do_GET(self):
        c, b, q = self._parts()
        if q.get("comp") == ["list"]:
            xml = "".join(f"<Blob><Name>{n}</Name></Blob>" for n in sorted(self.store.get(c, {})))
            return self._ok(f"<EnumerationResults><Blobs>{xml}</Blobs></EnumerationResults>".encode())
        if b in self.store.get(c, {}):
            return self._ok(self.store[c][b])
        self._ok(code=404)

    def do_DELETE(self):
        c, b, _ = self._parts()
        existed = self.store.get(c, {}).pop(b, None) is not None
        self._ok(code=202 if existed else 404)


def _zip(files):
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w") as z:
        for k, v in files.items():
            z.writestr(k, v)
    return buf.getvalue()


def _exercise(cs):
    data = _zip({"pipeline.yaml": "pipeline: []\n", "python/a.py": "x = 1\n"})
    md = cs.store_application_code("t1", "app", "v1", data, "digest-1")
    assert md.code_store_id.startswith("t1_app_v1_")
    assert cs.download_application_code("t1", md.code_store_id) == data
    assert cs.describe_application_code("t1", md.code_store_id).py_binaries_digest == "digest-1"
    md2 = cs.store_application_code("t1", "app", "v2", b"zz")
    other = cs.store_application_code("t1", "other", "v1", b"o")
    cs.delete_application_code("t1", md2.code_store_id)
    with pytest.raises(KeyError):
        cs.download_application_code("t1", md2.code_store_id)
    cs.delete_application("t1", "app")
    assert cs.describe_application_code("t1", md.code_store_id) is None
    assert cs.download_application_code("t1", other.code_store_id) == b"o"


def test_local_and_memory(tmp_path):
    _exercise(code_storage_for({"type": "local", "configuration": {"path": str(tmp_path / "cs")}}))
    _exercise(code_storage_for({"type": "memory"}))
    with pytest.raises(ValueError):
        code_storage_for({"type": "local", "configuration": {"path": str(tmp_path)}})._path("../x")


def test_s3():
    _FakeS3.store = {}
    srv, base = _serve(_FakeS3)
    try:
        cs = code_storage_for({"type": "s3", "configuration": {"endpoint": base, "access-key": "minioadmin",
                                                               "secret-key": "minioadmin"}})
        assert "langstream-code-storage" in _FakeS3.store
        _exercise(cs)
    finally:
        srv.shutdown()


def test_azure():
    _FakeAzure.store = {}
    srv, base = _serve(_FakeAzure)
    try:
        cs = code_storage_for({"type": "azure", "endpoint": base, "container": "code",
                               "sas-token": "?sv=2021&sig=abc"})
        _exercise(cs)
    finally:
        srv.shutdown()


def test_control_plane_uses_code_storage(tmp_path):
    from langstream_amd.cli.main import main
    from langstream_amd.cli.client import zip_directory
    from langstream_amd.webservice.server import ControlPlane
    app = tmp_path / "app"
    (app / "python").mkdir(parents=True)
    (app / "pipeline.yaml").write_text("pipeline:\n  - name: a\n    type: identity\n")
    (app / "python" / "m.py").write_text("X = 1\n")
    cs_cfg = {"type": "local", "configuration": {"path": str(tmp_path / "store")}}
    cp = ControlPlane(code_dir=str(tmp_path / "cache"), code_storage=code_storage_for(cs_cfg))
    cp.store.put_tenant("t")
    cp.deploy("t", "a", zip_directory(str(app)), None, None)
    sa = cp.store.get("t", "a")
    aid = sa.code_archive_id
    assert aid.startswith("t_a_")
    # unchanged python code keeps the archive; a change stores a new one
    cp.deploy("t", "a", zip_directory(str(app)), None, None, update=True)
    assert cp.store.get("t", "a").code_archive_id == aid
    (app / "python" / "m.py").write_text("X = 2\n")
    cp.deploy("t", "a", zip_directory(str(app)), None, None, update=True)
    new = cp.store.get("t", "a").code_archive_id
    assert new != aid
    # the agent init step fetches straight from the storage
    import json
    target = tmp_path / "dl"
    assert main(["code-download", "--tenant", "t", "--application", "a", "--code-archive-id", new,
                 "--target", str(target), "--code-storage", json.dumps(cs_cfg)]) == 0
    assert (target / "python" / "m.py").read_text() == "X = 2\n" or \
        any(p.endswith("m.py") for _, _, fs in os.walk(target) for p in fs)
    cp.delete("t", "a", force=True)
    assert not [n for n in os.listdir(tmp_path / "store" / "t") if n.startswith("t_a_")]
