"""The reference CLI's command tests, ported
(``langstream-cli/src/test/java/ai/langstream/cli/commands/applications/``:
``ProfilesCmdTest``, ``TenantsCmdTest``, ``AppsCmdTest``, ``GithubRepositoryDownloaderTest``,
``AbstractDeployApplicationCmdTest``, ``UIAppCmdTest``).

Each case runs the CLI in-process as ``CommandTestBase.executeCommand`` does: ``--conf`` a
fresh ``cli.yaml`` whose default profile points at a stub control plane (WireMock there,
``ref_runtime_harness.FakeHTTP`` here) with tenant ``my-tenant``; the result is the exit
code, stdout with trailing whitespace stripped and stderr stripped.
"""
from __future__ import annotations

import base64
import json
import os
from typing import NamedTuple

import pytest
import yaml

from ref_runtime_harness import FakeHTTP
from langstream_amd.cli import sources
from langstream_amd.cli.main import main as cli_main

TENANT = "my-tenant"


class CommandResult(NamedTuple):
    exit_code: int
    out: str
    err: str


@pytest.fixture()
def cli(tmp_path, capsys, monkeypatch):
    wm = FakeHTTP()
    conf = tmp_path / "cli.yaml"
    conf.write_text(f"webServiceUrl: {wm.url}\ntenant: {TENANT}")
    monkeypatch.chdir(tmp_path)
    for k in ("webServiceUrl", "apiGatewayUrl", "tenant", "token"):
        monkeypatch.delenv(f"LANGSTREAM_{k}", raising=False)

    class Cli:
        url = wm.url
        mock = wm
        config_path = conf

        @staticmethod
        def run(*args) -> CommandResult:
            capsys.readouterr()
            code = cli_main(["--conf", str(conf), *args])
            o = capsys.readouterr()
            return CommandResult(code, o.out.rstrip(), o.err.strip())

        @staticmethod
        def config():
            return yaml.safe_load(conf.read_text())
    yield Cli
    wm.close()


# ---------------------------------------------------------------- ProfilesCmdTest
def _table(rows):
    w = max(len(c) for r in rows for c in r)
    return "\n".join("  ".join(c.ljust(w) for c in r) for r in rows).rstrip()


def test_profiles_crud(cli):
    """ProfilesCmdTest.testCrud"""
    r = cli.run("profiles", "create", "new", "--web-service-url", "http://my.localhost:8080", "--tenant", "t",
                "--token", "tok", "--api-gateway-url", "http://my.localhost:8091")
    assert r == (0, "profile new created", "")
    p = cli.config()["profiles"]["new"]
    assert (p["name"], p["webServiceUrl"], p["tenant"], p["token"], p["apiGatewayUrl"]) == \
        ("new", "http://my.localhost:8080", "t", "tok", "http://my.localhost:8091")
    assert cli.run("profiles", "update", "new", "--token", "tok2") == (0, "profile new updated", "")
    p = cli.config()["profiles"]["new"]
    assert p["token"] == "tok2" and p["webServiceUrl"] == "http://my.localhost:8080"

    r = cli.run("profiles", "get", "new")
    assert r.exit_code == 0 and r.err == ""
    assert r.out == _table([["PROFILE", "WEBSERVICEURL", "TENANT", "TOKEN", "CURRENT"],
                            ["new", "http://my.localhost:8080", "t", "********", ""]])
    assert r.out.startswith("PROFILE                   WEBSERVICEURL             TENANT ")

    r = cli.run("profiles", "get", "new", "-o", "json")
    assert r == (0, '{\n  "webServiceUrl" : "http://my.localhost:8080",\n  "apiGatewayUrl" : "http://my.localhost:8091",'
                    '\n  "tenant" : "t",\n  "token" : "tok2",\n  "name" : "new"\n}', "")
    r = cli.run("profiles", "get", "new", "-o", "yaml")
    assert r == (0, '---\nwebServiceUrl: "http://my.localhost:8080"\napiGatewayUrl: "http://my.localhost:8091"\n'
                    'tenant: "t"\ntoken: "tok2"\nname: "new"', "")

    assert cli.run("profiles", "get", "notexists") == \
        (1, "", "Profile notexists not found, maybe you meant one of these: default, new")

    r = cli.run("profiles", "list")
    assert r.exit_code == 0 and r.err == ""
    assert r.out == _table([["PROFILE", "WEBSERVICEURL", "TENANT", "TOKEN", "CURRENT"],
                            ["default", cli.url, TENANT, "", "*"],
                            ["new", "http://my.localhost:8080", "t", "********", ""]])
    assert cli.run("profiles", "get-current") == (0, "default", "")
    assert cli.run("profiles", "set-current", "new") == (0, "profile new set as current", "")
    assert cli.config()["currentProfile"] == "new"
    assert cli.run("profiles", "delete", "new") == (1, "", "Cannot delete the current profile")
    assert cli.run("profiles", "set-current", "default") == (0, "profile default set as current", "")
    assert cli.run("profiles", "delete", "new") == (0, "profile new deleted", "")
    assert cli.config()["currentProfile"] == "default" and "new" not in (cli.config().get("profiles") or {})


def test_profiles_create_and_set(cli):
    """ProfilesCmdTest.testCreateAndSet"""
    assert cli.run("profiles", "create", "new", "--web-service-url", "http://my.localhost:8080", "--set-current") == \
        (0, "profile new created\nprofile new set as current", "")
    assert cli.config()["currentProfile"] == "new"
    assert cli.run("profiles", "create", "new1", "--web-service-url", "http://my.localhost:8080") == \
        (0, "profile new1 created", "")
    assert cli.config()["currentProfile"] == "new"
    assert cli.run("profiles", "update", "new1", "--web-service-url", "http://my.localhost:8080",
                   "--set-current") == (0, "profile new1 updated\nprofile new1 set as current", "")
    assert cli.config()["currentProfile"] == "new1"


@pytest.mark.parametrize("source", ["file", "json", "base64"])
def test_profiles_import(cli, tmp_path, source):
    """ProfilesCmdTest.testImport"""
    js = ('{"webServiceUrl":"http://my.localhost:8080","apiGatewayUrl":"http://my.localhost:8091",'
          '"tenant":"t","token":"tok"}')
    f = tmp_path / "p.json"
    f.write_text(js)
    flag, value = {"file": ("--file", str(f)), "json": ("--inline", js),
                   "base64": ("--inline", "base64:" + base64.b64encode(js.encode()).decode())}[source]
    assert cli.run("profiles", "import", "new", flag, value, "--set-current") == \
        (0, "profile new created\nprofile new set as current", "")
    p = cli.config()["profiles"]["new"]
    assert (p["webServiceUrl"], p["tenant"], p["token"], p["apiGatewayUrl"]) == \
        ("http://my.localhost:8080", "t", "tok", "http://my.localhost:8091")
    assert cli.run("profiles", "import", "new", flag, value, "--set-current") == \
        (1, "", "Profile new already exists")
    assert cli.run("profiles", "import", "new", flag, value, "--set-current", "-u") == \
        (0, "profile new updated\nprofile new set as current", "")


def test_profiles_default_profile(cli):
    """ProfilesCmdTest.testDefaultProfile"""
    r = cli.run("profiles", "get", "default")
    assert r.exit_code == 0 and r.err == ""
    assert r.out == _table([["PROFILE", "WEBSERVICEURL", "TENANT", "TOKEN", "CURRENT"],
                            ["default", cli.url, TENANT, "", "*"]])
    assert cli.run("profiles", "get-current") == (0, "default", "")
    assert cli.run("profiles", "create", "default") == (1, "", "Profile default already exists")
    assert cli.run("profiles", "update", "default", "--token", "tok2", "--web-service-url",
                   "http://my.localhost:8080", "--api-gateway-url", "ws://my.localhost:8091") == \
        (0, "profile default updated", "")
    c = cli.config()
    assert (c["token"], c["tenant"], c["webServiceUrl"], c["apiGatewayUrl"]) == \
        ("tok2", TENANT, "http://my.localhost:8080", "ws://my.localhost:8091")
    assert cli.run("profiles", "import", "default", "--inline",
                   '{"webServiceUrl":"http://my0.localhost/ls","tenant":"a-new"}', "-u") == \
        (0, "profile default updated", "")
    c = cli.config()
    assert c["tenant"] == "a-new" and c["webServiceUrl"] == "http://my0.localhost/ls"
    assert c.get("token") is None and c.get("apiGatewayUrl") is None
    assert cli.run("profiles", "delete", "default") == (1, "", "Profile name default can't be deleted")


def test_profiles_global_param(cli):
    """ProfilesCmdTest.testGlobalParam: ``-p`` picks the profile; a profile without a
    tenant, or an unknown one, fails with the reference's messages."""
    cli.mock.stub("GET", f"/api/applications/{TENANT}", text="[]")
    assert cli.run("apps", "list", "-o", "json") == (0, "[ ]", "")
    assert cli.run("profiles", "create", "new", "--web-service-url", "http://my.localhost:8080", "--set-current") == \
        (0, "profile new created\nprofile new set as current", "")
    assert cli.run("apps", "list", "-o", "json") == \
        (1, "", "Tenant not set. Please set the tenant in the configuration.")
    assert cli.run("-p", "default", "apps", "list", "-o", "json") == (0, "[ ]", "")
    assert cli.run("-p", "notexists", "apps", "list", "-o", "json") == \
        (1, "", "No profile 'notexists' defined in configuration")


# ---------------------------------------------------------------- TenantsCmdTest
def test_tenants_put(cli):
    """TenantsCmdTest.testPut"""
    cli.mock.stub("PUT", "/api/tenants/newt", text='{ "name": "newt" }')
    assert cli.run("tenants", "put", "newt") == (0, "tenant newt created/updated", "")


@pytest.mark.parametrize("units", [None, 10])
def test_tenants_create(cli, units):
    """TenantsCmdTest.testCreate / testCreatemaxTotalResourceUnits"""
    cli.mock.stub("POST", "/api/tenants/newt", body=json.dumps({"maxTotalResourceUnits": units}), text="")
    args = ["--max-total-resource-units", str(units)] if units else []
    assert cli.run("tenants", "create", "newt", *args) == (0, "tenant newt created", "")


def test_tenants_update(cli):
    """TenantsCmdTest.testUpdatemaxTotalResourceUnits"""
    cli.mock.stub("PATCH", "/api/tenants/newt", body='{"maxTotalResourceUnits": 10}', text="")
    assert cli.run("tenants", "update", "newt", "--max-total-resource-units", "10") == (0, "tenant newt updated", "")


def test_tenants_get_delete_list(cli):
    """TenantsCmdTest.testGet / testDelete / testList: bodies printed as the server sent them."""
    cli.mock.stub("GET", "/api/tenants/newt", text='{ "name": "newt" }')
    assert cli.run("tenants", "get", "newt") == (0, '{ "name": "newt" }', "")
    cli.mock.stub("DELETE", "/api/tenants/newt", text="")
    assert cli.run("tenants", "delete", "newt") == (0, "Tenant newt deleted", "")
    cli.mock.stub("GET", "/api/tenants", text="{}")
    assert cli.run("tenants", "list") == (0, "{}", "")


# ---------------------------------------------------------------- AppsCmdTest
def _app(tmp_path):
    d = tmp_path / "langstream"
    d.mkdir()
    (d / "module.yaml").write_text("module: module-1")
    inst = tmp_path / "instance.yaml"
    inst.write_text("instance: {}")
    sec = tmp_path / "secrets.yaml"
    sec.write_text("secrets: []")
    return str(d), str(inst), str(sec)


def _multipart(req):
    """name -> bytes of each part of a recorded multipart request."""
    boundary = req[3]["Content-Type"].split("boundary=", 1)[1].encode()
    out = {}
    for chunk in req[2].encode("latin-1").split(b"--" + boundary)[1:-1]:
        head, _, body = chunk[2:].partition(b"\r\n\r\n")
        name = head.split(b'name="', 1)[1].split(b'"', 1)[0].decode()
        out[name] = body[:-2]
    return out


def _parts(req):
    """Which parts were sent, and whether instance / secrets carry the files' text."""
    mp = _multipart(req)
    return {n: (mp[n] == b"instance: {}" if n == "instance" else mp[n] == b"secrets: []" if n == "secrets" else True)
            for n in mp}


def _zip_names(data):
    import io
    import zipfile
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        return {n: z.read(n) for n in z.namelist()}


@pytest.mark.parametrize("extra,query", [([], "dry-run=false&auto-upgrade=false"),
                                         (["--auto-upgrade"], "dry-run=false&auto-upgrade=true")])
def test_apps_deploy(cli, tmp_path, extra, query):
    """AppsCmdTest.testDeploy / testDeployAutoUpgrade: multipart app zip + instance + secrets."""
    app, inst, sec = _app(tmp_path)
    cli.mock.stub("POST", f"/api/applications/{TENANT}/my-app?{query}", text='{ "name": "my-app" }')
    r = cli.run("apps", "deploy", "my-app", "-s", sec, "-app", app, "-i", inst, *extra)
    assert r.exit_code == 0 and r.err == ""
    assert r.out.endswith("application my-app deployed")
    assert _parts(cli.mock.requests[-1]) == {"app": True, "instance": True, "secrets": True}


def test_apps_deploy_dry_run(cli, tmp_path):
    """AppsCmdTest.testDeployDryRun: the resolved application printed as YAML, or JSON."""
    app, inst, sec = _app(tmp_path)
    cli.mock.stub("POST", f"/api/applications/{TENANT}/my-app?dry-run=true&auto-upgrade=false",
                  text='{ "name": "my-app" }')
    r = cli.run("apps", "deploy", "my-app", "-s", sec, "-app", app, "-i", inst, "--dry-run")
    assert r.exit_code == 0 and r.err == "" and 'name: "my-app"' in r.out
    r = cli.run("apps", "deploy", "my-app", "-s", sec, "-app", app, "-i", inst, "--dry-run", "-o", "json")
    assert r.exit_code == 0 and r.err == "" and '{\n  "name" : "my-app"\n}' in r.out


@pytest.mark.parametrize("extra,query", [([], "auto-upgrade=false&force-restart=false"),
                                         (["--auto-upgrade"], "auto-upgrade=true&force-restart=false"),
                                         (["--force-restart"], "auto-upgrade=false&force-restart=true")])
def test_apps_update(cli, tmp_path, extra, query):
    """AppsCmdTest.testUpdateAll / testUpdateAppWithAutoUpgrade / testUpdateAppWithForceRestart /
    testUpdateInstance / testUpdateSecrets: only the given parts are sent."""
    app, inst, sec = _app(tmp_path)
    cli.mock.stub("PATCH", f"/api/applications/{TENANT}/my-app?{query}", text='{ "name": "my-app" }')
    r = cli.run("apps", "update", "my-app", "-s", sec, "-app", app, "-i", inst, *extra)
    assert r.exit_code == 0 and r.err == "" and r.out.endswith("application my-app updated")
    assert _parts(cli.mock.requests[-1]) == {"app": True, "instance": True, "secrets": True}
    if not extra:
        for flags, parts in ((["-i", inst], {"instance"}), (["-s", sec], {"secrets"}),
                             (["-app", app], {"app"}), (["-app", app, "-i", inst], {"app", "instance"})):
            assert cli.run("apps", "update", "my-app", *flags).exit_code == 0
            assert set(_parts(cli.mock.requests[-1])) == parts
        assert cli.run("apps", "update", "my-app") == (1, "", "no application, instance or secrets file provided")


def test_apps_deploy_with_dependencies(cli, tmp_path):
    """AppsCmdTest.testDeployWithDependencies: a java-library already in java/lib with the
    right SHA-512 is kept (not downloaded again) and zipped with the application; a
    corrupted one is replaced by the download."""
    import hashlib
    content = b"dep-content"
    sha = hashlib.sha512(content).hexdigest()
    assert sha.startswith("e1ebfd0f4e4a624e")      # the reference test's constant
    cli.mock.stub("GET", "/local/get-dependency.jar", text="dep-content")
    app, inst, sec = _app(tmp_path)
    os.makedirs(os.path.join(app, "java", "lib"))
    with open(os.path.join(app, "configuration.yaml"), "w") as f:
        f.write(f'configuration:\n  dependencies:\n    - name: "PostGRES JDBC Driver"\n'
                f'      url: "{cli.url}/local/get-dependency.jar"\n      sha512sum: "{sha}"\n'
                f'      type: "java-library"\n')
    jar = os.path.join(app, "java", "lib", "get-dependency.jar")
    with open(jar, "wb") as f:
        f.write(content)
    cli.mock.stub("POST", f"/api/applications/{TENANT}/my-app?dry-run=false&auto-upgrade=false",
                  text='{ "name": "my-app" }')
    r = cli.run("apps", "deploy", "my-app", "-s", sec, "-app", app, "-i", inst)
    assert r.err == "" and r.exit_code == 0
    assert not any(q[1] == "/local/get-dependency.jar" for q in cli.mock.requests)
    assert _zip_names(_multipart(cli.mock.requests[-1])["app"])["java/lib/get-dependency.jar"] == content
    with open(jar, "wb") as f:
        f.write(b"corrupted")
    r = cli.run("apps", "deploy", "my-app", "-s", sec, "-app", app, "-i", inst)
    assert r.err == "" and r.exit_code == 0 and "File seems corrupted, deleting it" in r.out
    assert "dependency downloaded" in r.out and open(jar, "rb").read() == content


def test_apps_deploy_with_file_placeholders(cli, tmp_path):
    """AppsCmdTest.testDeployWithFilePlaceholders: a ``<file:...>`` reference in the secrets
    is inlined and the file re-sent as the reference's YAML printer writes it."""
    app, inst, _ = _app(tmp_path)
    (tmp_path / "sa.json").write_text('{"client-id":"xxx"}')
    sec = tmp_path / "secrets-ph.yaml"
    sec.write_text("secrets:\n     - name: vertex-ai\n       id: vertex-ai\n       data:\n"
                   "         url: https://us-central1-aiplatform.googleapis.com\n         token: xxx\n"
                   '         serviceAccountJson: "<file:sa.json>"\n         region: us-central1\n'
                   "         project: myproject\n")
    cli.mock.stub("POST", f"/api/applications/{TENANT}/my-app?dry-run=false&auto-upgrade=false",
                  text='{ "name": "my-app" }')
    r = cli.run("apps", "deploy", "my-app", "-s", str(sec), "-app", app, "-i", inst)
    assert r.exit_code == 0 and r.err == ""
    mp = _multipart(cli.mock.requests[-1])
    assert mp["instance"] == b"instance: {}"
    assert mp["secrets"].decode() == (
        '---\nsecrets:\n- name: "vertex-ai"\n  id: "vertex-ai"\n  data:\n'
        '    url: "https://us-central1-aiplatform.googleapis.com"\n    token: "xxx"\n'
        '    serviceAccountJson: "{\\"client-id\\":\\"xxx\\"}"\n    region: "us-central1"\n'
        '    project: "myproject"\n')


def _yaml12_floats(v):
    """PyYAML resolves YAML 1.1 floats only; ``1.0E10`` (a YAML 1.2 float, as the
    reference's YAML printer writes it) comes back as a string."""
    import re
    if isinstance(v, dict):
        return {k: _yaml12_floats(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_yaml12_floats(x) for x in v]
    if isinstance(v, str) and re.fullmatch(r"-?\d\.\d+E-?\d+", v):
        return float(v)
    return v


EXPECTED_GET = os.path.join(os.path.dirname(__file__), "fixtures", "expected-get.json")


def test_apps_get(cli):
    """AppsCmdTest.testGet on the reference's fixture (tests/fixtures/expected-get.json): the raw table,
    JSON re-printed in the reference's layout, YAML, and a mermaid diagram."""
    text = open(EXPECTED_GET).read()
    cli.mock.stub("GET", f"/api/applications/{TENANT}/my-app?stats=false", text=text)
    assert cli.run("apps", "get", "my-app") == \
        (0, "ID          STREAMING   COMPUTE     STATUS      EXECUTORS   REPLICAS  \n"
            "test        kafka       kubernetes  DEPLOYED    2/2         2/2", "")
    r = cli.run("apps", "get", "my-app", "-o", "json")
    assert r.exit_code == 0 and r.err == "" and json.loads(r.out) == json.loads(text)
    assert r.out.startswith('{\n  "application-id" : "test",\n  "application" : {\n    "resources" : {')
    assert '"modules" : [ {\n      "id" : "default",' in r.out
    r = cli.run("apps", "get", "my-app", "-o", "yaml")
    assert r.exit_code == 0 and r.err == "" and r.out.startswith('---\napplication-id: "test"\napplication:\n')
    assert _yaml12_floats(yaml.safe_load(r.out)) == json.loads(text)
    r = cli.run("apps", "get", "my-app", "-o", "mermaid")
    assert r.exit_code == 0 and r.err == "" and r.out != ""


def test_apps_delete(cli):
    """AppsCmdTest.testDelete / testForceDelete"""
    cli.mock.stub("DELETE", f"/api/applications/{TENANT}/my-app?force=false", text="")
    assert cli.run("apps", "delete", "my-app") == (0, "Application 'my-app' marked for deletion", "")
    cli.mock.stub("DELETE", f"/api/applications/{TENANT}/my-app?force=true", text="")
    assert cli.run("apps", "delete", "my-app", "-f") == (0, "Application 'my-app' marked for deletion (forced)", "")


def test_apps_list(cli):
    """AppsCmdTest.testList"""
    cli.mock.stub("GET", f"/api/applications/{TENANT}", text="[]")
    assert cli.run("apps", "list") == (0, "ID         STREAMING  COMPUTE    STATUS     EXECUTORS  REPLICAS", "")
    assert cli.run("apps", "list", "-o", "json") == (0, "[ ]", "")
    assert cli.run("apps", "list", "-o", "yaml") == (0, "--- []", "")


def test_apps_logs(cli):
    """AppsCmdTest.testLogs: text, then JSON lines, as the server sends them."""
    cli.mock.stub("GET", f"/api/applications/{TENANT}/my-app/logs?format=text&follow=true", text="some logs")
    assert cli.run("apps", "logs", "my-app") == (0, "some logs", "")
    line = ('{"replica":"app-1-0","message":"08:53:44.519 [stats-pipeline-python-processor-1] INFO  '
            'a.l.runtime.agent.AgentRunner -- Records: total 5, working 0","timestamp":1697447779798}')
    cli.mock.stub("GET", f"/api/applications/{TENANT}/my-app/logs?format=json&follow=true", text=line)
    assert cli.run("apps", "logs", "my-app", "-o", "json") == (0, line, "")


def test_apps_download(cli, tmp_path):
    """AppsCmdTest.testDownload / testDownloadToFile"""
    cli.mock.stub("GET", f"/api/applications/{TENANT}/my-app/code", text="")
    r = cli.run("apps", "download", "my-app")
    assert r == (0, f"Downloaded application code to {tmp_path / f'{TENANT}-my-app.zip'}", "")
    out = tmp_path / "download.zip"
    assert cli.run("apps", "download", "my-app", "-o", str(out)) == (0, f"Downloaded application code to {out}", "")
    assert out.exists()


# ---------------------------------------------------------------- GithubRepositoryDownloaderTest
def test_parse_github_urls():
    """GithubRepositoryDownloaderTest.testParseUrl / testParseUrlBlob / testParseUrlRoot"""
    assert sources.parse_github("https://github.com/LangStream/langstream/tree/main/examples/applications/"
                                "astradb-sink") == ("LangStream", "langstream", "main", "examples/applications/astradb-sink")
    assert sources.parse_github("https://github.com/LangStream/langstream/blob/v0.0.13/examples/instances/astra.yaml") \
        == ("LangStream", "langstream", "v0.0.13", "examples/instances/astra.yaml")
    owner, repo, branch, directory = sources.parse_github("https://github.com/LangStream/langstream/tree/main")
    assert (owner, repo, branch) == ("LangStream", "langstream", "main") and not directory


def test_github_download_cache_update_and_fallback(tmp_path, monkeypatch):
    """GithubRepositoryDownloaderTest.testDownload: no cache -> a temporary clone; with the
    cache -> <home>/ghrepos/<owner>/<repo>/<branch>, reused in-process, updated by a new
    process; a failed update drops the cache and clones to a temporary directory."""
    home = tmp_path / "home"
    home.mkdir()
    monkeypatch.setattr(sources, "cli_home", lambda: str(home))
    fail = {"update": False}

    def clone(owner, repo, branch, dest):
        os.makedirs(os.path.join(dest, "examples", ".."), exist_ok=True)
        os.makedirs(os.path.join(dest, ".git"), exist_ok=True)
        os.makedirs(os.path.join(dest, "examples"), exist_ok=True)
        with open(os.path.join(dest, "examples", "my-file"), "w") as f:
            f.write(f"content! {branch}")

    def update(dest, branch):
        if fail["update"]:
            raise IOError("inject failure")
        with open(os.path.join(dest, "examples", "my-file"), "w") as f:
            f.write(f"content updated! {branch}")
        return "xxx"
    monkeypatch.setattr(sources, "_clone", clone)
    monkeypatch.setattr(sources, "_update", update)
    monkeypatch.setattr(sources, "_cloned", {})

    def content(d):
        return open(os.path.join(d, "my-file")).read()
    d = sources.download_github("https://localhost/LangStream/langstream/tree/main/examples", use_cache=False)
    assert content(d) == "content! main" and not (home / "ghrepos").exists()
    cached = str(home / "ghrepos" / "LangStream" / "langstream2" / "main" / "examples")
    d = sources.download_github("https://localhost/LangStream/langstream2/tree/main/examples", use_cache=True)
    assert content(d) == "content! main" and d == cached
    d = sources.download_github("https://localhost/LangStream/langstream2/tree/main/examples", use_cache=True)
    assert content(d) == "content! main" and d == cached           # same process: reused as is
    monkeypatch.setattr(sources, "_cloned", {})                    # a new CLI process
    d = sources.download_github("https://localhost/LangStream/langstream2/tree/main/examples", use_cache=True)
    assert content(d) == "content updated! main" and d == cached
    fail["update"] = True
    monkeypatch.setattr(sources, "_cloned", {})
    d = sources.download_github("https://localhost/LangStream/langstream2/tree/main/examples", use_cache=True)
    assert content(d) == "content! main" and not (home / "ghrepos").exists()


# ---------------------------------------------------------------- AbstractDeployApplicationCmdTest
def test_remote_file():
    """AbstractDeployApplicationCmdTest.testRemoteFile"""
    from ref_runtime_harness import FakeHTTP
    fake = FakeHTTP()
    fake.stub("GET", "/my-remote-dir/my-remote-file", text="content!")
    try:
        assert open(sources.download_https(fake.url + "/my-remote-dir/my-remote-file")).read() == "content!"
        with pytest.raises(RuntimeError, match="Received status code: 404"):
            sources.download_https(fake.url + "/unknown")
    finally:
        fake.close()


def test_dependencies(tmp_path):
    """AbstractDeployApplicationCmdTest.testDependencies: a wrong or empty checksum fails
    after the download, a missing type fails, two dependencies with the right SHA-512
    download (the second finds the first's file already there)."""
    from ref_runtime_harness import FakeHTTP
    fake = FakeHTTP()
    fake.stub("GET", "/the-dep.jar", text="content!")
    sha = ("bed0f8673c13f8431d5e4f5e4a0e496b2eddc4a18e03cff19256964a6132521a485afa59ace702b76c2832274d1c3914e3fec0221"
           "fee9d698eaedc7f5810a284")
    url = fake.url + "/the-dep.jar"

    def run(deps):
        d = tmp_path / f"app{len(list(tmp_path.iterdir()))}"
        d.mkdir()
        (d / "configuration.yaml").write_text(yaml.safe_dump({"configuration": {"dependencies": deps}}))
        sources.download_dependencies(str(d), lambda m: None)
        return d
    try:
        for bad in ("-", ""):
            with pytest.raises(IOError, match=f"File at {url}, seems corrupted"):
                run([{"name": "My dep", "url": url, "sha512sum": bad, "type": "java-library"}])
        with pytest.raises(RuntimeError, match="dependency type must be set"):
            run([{"name": "My dep", "url": url}])
        d = run([{"name": "My dep", "url": url, "sha512sum": sha, "type": "java-library"},
                 {"name": "My dep2", "url": url, "sha512sum": sha, "type": "java-library"}])
        assert (d / "java" / "lib" / "the-dep.jar").read_text() == "content!"
    finally:
        fake.close()


# ---------------------------------------------------------------- UIAppCmdTest
def test_open_browser(tmp_path):
    """UIAppCmdTest.openBrowser: an open command that exists is launched, one that does
    not is reported as not launched."""
    from langstream_amd.cli.app_ui import check_and_launch
    exe = tmp_path / "open-cmd"
    exe.write_text("#!/bin/sh\necho hello\n")
    exe.chmod(0o500)
    assert check_and_launch(str(exe), 80) is True
    assert check_and_launch("_no_such_command_", 80) is False
