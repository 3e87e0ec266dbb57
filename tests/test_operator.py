"""Kubernetes operator + Kubernetes application store against an in-process fake API
server (objects by path, server-side apply, merge-patch incl. /status, finalizers,
owner-reference garbage collection).

Mirrors the reference's operator tests (AppControllerIT / AgentControllerIT with a
fabric8 mock server, TenantLimitsCheckerTest, KubernetesApplicationStoreTest)."""
import copy
import json
import threading
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import urlsplit

import pytest

from langstream_amd.core.parser import build_application_instance
from langstream_amd.core.store import StoredApplication
from langstream_amd.operator import FINALIZER, Operator
from langstream_amd.operator.kube import CR_API, KubeClient
from langstream_amd.operator.store import KubernetesApplicationStore


def _merge(dst, src):
    for k, v in src.items():
        if isinstance(v, dict) and isinstance(dst.get(k), dict):
            _merge(dst[k], v)
        else:
            dst[k] = copy.deepcopy(v)


class FakeKube:
    def __init__(self):
        self.objs = {}      # path -> object
        self.lock = threading.Lock()
        fake = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body=None):
                data = json.dumps(body).encode() if body is not None else b""
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n) or b"{}")

            def do_GET(self):
                code, body = fake.get(urlsplit(self.path).path)
                self._send(code, body)

            def do_PATCH(self):
                u = urlsplit(self.path)
                code, body = fake.patch(u.path, self.headers.get("Content-Type", ""), self._body())
                self._send(code, body)

            def do_DELETE(self):
                self._body()
                code, body = fake.delete(urlsplit(self.path).path)
                self._send(code, body)

        self.srv = ThreadingHTTPServer(("127.0.0.1", 0), H)
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()
        self.url = f"http://127.0.0.1:{self.srv.server_address[1]}"

    @staticmethod
    def split(path):
        seg = path.strip("/").split("/")
        pre = seg[:2] if seg[0] == "api" else seg[:3]
        rest = seg[len(pre):]
        return "/" + "/".join(pre), rest

    def get(self, path):
        with self.lock:
            if path in self.objs:
                return 200, self.objs[path]
            pre, rest = self.split(path)
            items = []
            for p, o in self.objs.items():
                if not p.startswith(pre + "/"):
                    continue
                prest = self.split(p)[1]
                if len(rest) == 1 and prest[-2] == rest[0]:                      # all namespaces
                    items.append(o)
                elif len(rest) == 3 and prest[:3] == rest and len(prest) == 4:    # one namespace
                    items.append(o)
            if len(rest) in (1, 3) and not (len(rest) == 3 and rest[0] != "namespaces"):
                return 200, {"items": items}
            return 404, {"reason": "NotFound"}

    def patch(self, path, ctype, body):
        with self.lock:
            sub = None
            if path.endswith("/status"):
                path, sub = path[: -len("/status")], "status"
            cur = self.objs.get(path)
            if "apply-patch" in ctype:
                if cur is None:
                    body.setdefault("metadata", {})["uid"] = uuid.uuid4().hex
                    body["metadata"]["generation"] = 1
                    self.objs[path] = body
                    return 201, body
                gen = cur["metadata"].get("generation", 1)
                if body.get("spec") != cur.get("spec") or body.get("data") != cur.get("data"):
                    gen += 1
                keep = {k: cur["metadata"][k] for k in ("uid", "finalizers", "deletionTimestamp")
                        if k in cur["metadata"]}
                new = copy.deepcopy(body)
                new["metadata"].update(keep)
                new["metadata"]["generation"] = gen
                if "status" in cur and "status" not in new:
                    new["status"] = cur["status"]
                self.objs[path] = new
                return 200, new
            if cur is None:
                return 404, {"reason": "NotFound"}
            if sub == "status":
                _merge(cur.setdefault("status", {}), body.get("status") or {})
            else:
                _merge(cur, body)
                if cur["metadata"].get("deletionTimestamp") and not cur["metadata"].get("finalizers"):
                    self._remove(path)
            return 200, cur

    def _remove(self, path):
        obj = self.objs.pop(path)
        uid = obj["metadata"].get("uid")
        for p, o in list(self.objs.items()):   # owner-reference garbage collection
            if any(r.get("uid") == uid for r in o["metadata"].get("ownerReferences") or []):
                if p in self.objs:
                    self._remove(p)

    def delete(self, path):
        with self.lock:
            cur = self.objs.get(path)
            if cur is None:
                return 404, {"reason": "NotFound"}
            if cur["metadata"].get("finalizers"):
                cur["metadata"]["deletionTimestamp"] = "2026-01-01T00:00:00Z"
            else:
                self._remove(path)
            return 200, {"status": "Success"}

    def kinds(self, plural, ns=None):
        return sorted(p.rsplit("/", 1)[1] for p in self.objs
                      if p.split("/")[-2] == plural and (ns is None or f"/{ns}/" in p))


PIPE = """
topics:
  - name: in-t
    creation-mode: create-if-not-exists
  - name: out-t
    creation-mode: create-if-not-exists
    deletion-mode: delete
pipeline:
  - name: a1
    id: step1
    type: compute
    input: in-t
    configuration:
      fields:
        - name: value.x
          expression: "1"
  - name: a2
    id: step2
    type: drop-fields
    output: out-t
    resources:
      parallelism: 2
    configuration:
      fields: [y]
"""
INSTANCE = """
instance:
  streamingCluster:
    type: noop
  computeCluster:
    type: kubernetes
"""


@pytest.fixture()
def kube():
    f = FakeKube()
    yield f
    f.srv.shutdown()


def _stored(app_id, files, tenant="t1"):
    built = build_application_instance(files, INSTANCE)
    return StoredApplication(application_id=app_id, tenant=tenant, application=getattr(built, "application", built),
                             files=files, instance=INSTANCE, secrets="secrets:\n  - id: s\n    data: {k: v}\n",
                             code_archive_id="abc")


def test_store_and_operator_lifecycle(kube):
    client = KubeClient(kube.url)
    store = KubernetesApplicationStore(client)
    store.put_tenant("t1", {"max-total-resource-units": 10})
    assert store.get_tenant("t1")["name"] == "t1" and "t1" in store.list_tenants()
    assert kube.kinds("namespaces") == ["langstream-t1"]
    store.put(_stored("app1", {"pipeline.yaml": PIPE}))
    assert [a.application_id for a in store.list("t1")] == ["app1"]
    assert store.get("t1", "app1").secrets.startswith("secrets:")

    op = Operator(client)
    res = op.reconcile_all()
    assert res["app/langstream-t1/app1"] == "DEPLOYED"
    assert kube.kinds("agents") == ["app1-step1", "app1-step2"]
    app_cr = client.get(CR_API, "Application", "langstream-t1", "app1")
    assert FINALIZER in app_cr["metadata"]["finalizers"]
    assert store.get("t1", "app1").status == "DEPLOYED"
    # second pass: agent controller builds the workloads
    res = op.reconcile_all()
    assert res["agent/langstream-t1/app1-step2"] == "DEPLOYING"
    sts = client.get("apps/v1", "StatefulSet", "langstream-t1", "app1-step2")
    assert sts["spec"]["replicas"] == 2 and sts["metadata"]["ownerReferences"][0]["kind"] == "Agent"
    assert client.get("v1", "Service", "langstream-t1", "app1-step1")["spec"]["clusterIP"] == "None"
    cfg = client.get("v1", "Secret", "langstream-t1", "app1-step2-config")
    assert cfg is not None
    # ready replicas -> DEPLOYED
    client.merge_patch("apps/v1", "StatefulSet", "langstream-t1", "app1-step2", {"status": {"readyReplicas": 2}},
                       "status")
    assert op.reconcile_all()["agent/langstream-t1/app1-step2"] == "DEPLOYED"

    # update: step2 merged into step1's parallelism -> one composite agent; the stale agent goes
    store.put(_stored("app1", {"pipeline.yaml": PIPE.replace("parallelism: 2", "parallelism: 1")}))
    assert op.reconcile_all()["app/langstream-t1/app1"] == "DEPLOYED"
    assert len(kube.kinds("agents")) == 1

    # delete: finalizer -> cleanup -> CR and (by owner references) the workloads are gone
    assert store.delete("t1", "app1")
    op.reconcile_all()
    assert kube.kinds("applications") == [] and kube.kinds("agents") == [] and kube.kinds("statefulsets") == []


def test_tenant_limits_block_deploy(kube):
    client = KubeClient(kube.url)
    store = KubernetesApplicationStore(client)
    store.put_tenant("t1")
    client.apply({"apiVersion": "v1", "kind": "ConfigMap",
                  "metadata": {"name": "langstream-tenant-limits", "namespace": "langstream"}, "data": {"t1": "2"}})
    store.put(_stored("big", {"pipeline.yaml": PIPE}))       # needs 1 + 2 units
    op = Operator(client)
    assert op.reconcile_all()["app/langstream-t1/big"] == "ERROR_DEPLOYING"
    st = client.get(CR_API, "Application", "langstream-t1", "big")["status"]["status"]
    assert "Not enough resources" in st["reason"]
    assert kube.kinds("agents") == []


def _run_job(client, kube, job_name, monkeypatch, tmp_path):
    """Play the Kubernetes Job controller: run the Job's container command in-process
    against the fake API server, then mark the Job succeeded."""
    import base64
    from langstream_amd.runtime import jobs
    job = client.get("batch/v1", "Job", "langstream-t1", job_name)
    assert job is not None, job_name
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["command"][:3] == ["python", "-m", "langstream_amd.runtime.jobs"]
    secret = job["spec"]["template"]["spec"]["volumes"][0]["secret"]["secretName"]
    cfg = base64.b64decode(client.get("v1", "Secret", "langstream-t1", secret)["data"]["config"]).decode()
    path = tmp_path / f"{job_name}.json"
    path.write_text(cfg)
    monkeypatch.setenv("LANGSTREAM_JOB_PHASE", c["env"][0]["value"])
    monkeypatch.setenv("LANGSTREAM_KUBE_API", kube.url)
    assert jobs.main([c["command"][3], str(path)]) == 0
    client.merge_patch("batch/v1", "Job", "langstream-t1", job_name, {"status": {"succeeded": 1}}, "status")


def test_operator_runs_setup_and_deployer_as_jobs(kube, monkeypatch, tmp_path):
    client = KubeClient(kube.url)
    store = KubernetesApplicationStore(client)
    store.put_tenant("t1")
    store.put(_stored("app2", {"pipeline.yaml": PIPE}))
    op = Operator(client, use_jobs=True)
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DEPLOYING"
    assert kube.kinds("jobs") == ["langstream-runtime-setup-app2-1"] and kube.kinds("agents") == []
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DEPLOYING"       # job still running
    _run_job(client, kube, "langstream-runtime-setup-app2-1", monkeypatch, tmp_path)
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DEPLOYING"
    assert "langstream-runtime-deployer-app2-1" in kube.kinds("jobs")
    _run_job(client, kube, "langstream-runtime-deployer-app2-1", monkeypatch, tmp_path)
    assert kube.kinds("agents") == ["app2-step1", "app2-step2"]                # created by the deployer job
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DEPLOYED"
    assert store.get("t1", "app2").status == "DEPLOYED"
    # a failed setup job of a new revision -> ERROR_SETUP
    store.put(_stored("app2", {"pipeline.yaml": PIPE.replace("parallelism: 2", "parallelism: 1")}))
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DEPLOYING"
    client.merge_patch("batch/v1", "Job", "langstream-t1", "langstream-runtime-setup-app2-2",
                       {"status": {"failed": 2}}, "status")
    assert op.reconcile_all()["app/langstream-t1/app2"] == "ERROR_SETUP"
    # deletion: deployer-cleanup job, then setup-cleanup job, then the CR goes
    assert store.delete("t1", "app2")
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DELETING"
    _run_job(client, kube, "langstream-runtime-deployer-cleanup-app2-2", monkeypatch, tmp_path)
    assert kube.kinds("agents") == []
    assert op.reconcile_all()["app/langstream-t1/app2"] == "DELETING"
    _run_job(client, kube, "langstream-runtime-setup-cleanup-app2-2", monkeypatch, tmp_path)
    op.reconcile_all()
    assert kube.kinds("applications") == []
