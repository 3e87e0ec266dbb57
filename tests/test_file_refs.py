"""${ENV:-default} and <file:...> resolution in instance / secrets files (parity:
langstream-cli/.../LocalFileReferenceResolver.java:37-160 and its test
LocalFileReferenceResolverTest.java), and planning of every reference example app with
the reference instance + secrets files when the reference checkout is present."""
import os

import pytest
import yaml

from langstream_amd.core.file_refs import resolve_file_references, substitute_env

REF = "/root/reference/examples"


def test_env_substitution_semantics():
    env = {"HOME_X": "/h", "EMPTY": "", "NAME": "HOME_X"}
    assert substitute_env("${HOME_X:-d}", env) == "/h"
    assert substitute_env("${USE_DEFAULT:-defaultValue}", env) == "defaultValue"
    assert substitute_env("${home_x:-defaultValue}", env) == "defaultValue"      # case-sensitive
    assert substitute_env("${EMPTY:-d}", env) == "d"
    assert substitute_env("${UNSET}", env) == "${UNSET}"                           # left as-is
    assert substitute_env("$${HOME_X}", env) == "${HOME_X}"                        # escaped
    assert substitute_env("a${HOME_X}b${X:-${HOME_X}}", env) == "a/hb/h"          # nested default
    assert substitute_env("${secrets.open-ai.access-key}", env) == "${secrets.open-ai.access-key}"


def test_file_references_text_and_binary(tmp_path):
    (tmp_path / "some-text-file.txt").write_text("text content with \" and ' and \n")
    (tmp_path / "b.bin").write_bytes(bytes([1, 2, 3]))
    content = ("secrets:\n  - id: a\n    data:\n      list: [\"<file:some-text-file.txt>\", \"<file:b.bin>\"]\n"
               "      port: ${SOLR_PORT_TEST_UNSET:-8983}\n")
    out = yaml.safe_load(resolve_file_references(content, str(tmp_path), env={}))
    data = out["secrets"][0]["data"]
    assert data["list"] == ["text content with \" and ' and \n", "base64:AQID"]
    assert data["port"] == "8983"           # substituted values stay strings


def test_no_references_returns_content_unchanged(tmp_path):
    content = "secrets:\n  - name: vertex-ai\n    id: vertex-ai\n"
    assert resolve_file_references(content, str(tmp_path)) == content


def test_invalid_yaml_fails_fast(tmp_path):
    with pytest.raises(ValueError):
        resolve_file_references("a: [unclosed", str(tmp_path))


# The reference rejects these with its own example secrets file, for the same reasons:
REF_REJECTS = {
    # ${secrets.s3-credentials.*}: no such secret (ApplicationPlaceholderResolver.java:345-364)
    "chatbot-rag-memory": "s3-credentials",
    # 'datasource' resources support astra/cassandra/jdbc/opensearch/astra-vector-db only
    # (DataSourceResourceProvider.java:34-42); milvus is a 'vector-database' service
    "query-milvus": "MilvusDatasource",
    # ${secrets.pinecone.api-key} is null: the secret has 'access-key' (PineconeDatasourceConfig api-key required)
    "query-pinecone": "api-key",
    # the OpenSearch vector-database resource has no index-name (OpenSearchDatasourceConfig.java:103)
    "rag-aws": "index-name",
}


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
@pytest.mark.parametrize("app", sorted(os.listdir(os.path.join(REF, "applications")))
                         if os.path.isdir(REF) else [])
def test_reference_example_apps_plan(app, monkeypatch):
    """Every reference example application plans against the reference secrets file
    with the kafka-docker instance (env unset: every ${VAR:-default} takes its default),
    except the ones the reference's own planner rejects with these files (REF_REJECTS)."""
    from langstream_amd.core.deployer import ApplicationDeployer
    from langstream_amd.core.parser import build_from_directory
    for k in list(os.environ):
        if k.isupper() and k not in ("PATH", "HOME", "PYTHONPATH", "TMPDIR"):
            monkeypatch.delenv(k, raising=False)
    d = os.path.join(REF, "applications", app)
    if app in REF_REJECTS:
        with pytest.raises(ValueError, match=REF_REJECTS[app]):
            info = build_from_directory(d, os.path.join(REF, "instances", "kafka-docker.yaml"),
                                        os.path.join(REF, "secrets", "secrets.yaml"))
            ApplicationDeployer().create_implementation("app", info.application)
        return
    info = build_from_directory(d, os.path.join(REF, "instances", "kafka-docker.yaml"),
                                os.path.join(REF, "secrets", "secrets.yaml"))
    plan = ApplicationDeployer().create_implementation("app", info.application)
    assert plan.agents or plan.application.gateways is not None
