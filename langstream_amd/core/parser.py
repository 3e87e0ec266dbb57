"""YAML application parser (ModelBuilder).

Parity: CORE/parser/ModelBuilder.java -- file dispatch :410-456, configuration.yaml
:467-501, gateway validation :503-622, pipeline files :659-810 (auto ids :749-769,
implicit chaining :779-801), instance/secrets :812-874, archetypes :78-184, package
digests :275-349.
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml

from ..api.model import (DEAD_LETTER, DEFAULT_MODULE, ON_FAILURE_VALUES, AgentConfiguration, Application,
                         AssetDefinition, ComputeCluster, Connection, Dependency, ErrorsSpec, Gateway, Instance,
                         Resource, ResourcesSpec, Secret, Secrets, StreamingCluster, TopicDefinition)


def _load_yaml(content: str) -> Any:
    return yaml.safe_load(content) if content and content.strip() else None


@dataclass
class ApplicationWithPackageInfo:
    application: Application
    has_app_definition: bool = False
    has_instance_definition: bool = False
    has_secret_definition: bool = False
    py_binaries_digest: Optional[str] = None
    java_binaries_digest: Optional[str] = None


def validate_errors_spec(spec: Optional[ErrorsSpec]) -> ErrorsSpec:
    if spec is None:
        return ErrorsSpec.DEFAULT
    if spec.on_failure is not None and spec.on_failure not in ON_FAILURE_VALUES:
        raise ValueError(f"on-failure must be one of {list(ON_FAILURE_VALUES)}, got {spec.on_failure}")
    if spec.retries is not None and spec.retries < 0:
        raise ValueError("retries must be >= 0")
    return spec


def _validate_kv(kvs) -> None:
    for kv in kvs or []:
        if not kv.key or not str(kv.key).strip():
            raise ValueError("'key' is required for filter")
        for name, v in (("value", kv.value), ("valueFromParameters", kv.value_from_parameters),
                        ("valueFromAuthentication", kv.value_from_authentication)):
            if v is not None and not str(v).strip():
                raise ValueError(f"'{name}' cannot be blank for filter")


def validate_gateway(g: Gateway, raw: dict) -> None:
    if not g.id or not str(g.id).strip():
        raise ValueError("Gateway id is required")
    if g.type is None:
        raise ValueError("Gateway type is required")
    has = lambda k: raw.get(k) is not None  # noqa: E731
    if g.type == "consume":
        for k, n in (("produce-options", "produce-options"), ("chat-options", "chat-options"),
                     ("service-options", "service-options")):
            if has(k):
                raise ValueError(f"Gateway of type 'consume' cannot have {n}")
        _validate_kv(g.consume_options)
    elif g.type == "produce":
        for k in ("consume-options", "chat-options", "service-options"):
            if has(k):
                raise ValueError(f"Gateway of type 'produce' cannot have {k}")
    elif g.type == "chat":
        for k in ("consume-options", "produce-options", "service-options"):
            if has(k):
                raise ValueError(f"Gateway of type 'chat' cannot have {k}")
        if g.topic is not None:
            raise ValueError("Gateway of type 'chat' cannot have topic. Use chat-options.question-topic and "
                             "chat-options.answers-topic instead")
        if g.chat_options is None:
            raise ValueError("Gateway of type 'chat' must have chat-options")
        if g.chat_options.answers_topic is None:
            raise ValueError("Gateway of type 'chat' must have chat-options.answers-topic")
        if g.chat_options.questions_topic is None:
            raise ValueError("Gateway of type 'chat' must have chat-options.questions-topic")
    elif g.type == "service":
        for k in ("consume-options", "produce-options", "chat-options"):
            if has(k):
                raise ValueError(f"Gateway of type 'service' cannot have {k}")
        so = g.service_options
        if so is None:
            raise ValueError("Gateway of type 'service' must have service-options")
        if so.agent_id is None:
            if so.input_topic is None:
                raise ValueError("Gateway of type 'service' must have service-options.input-topic")
            if so.output_topic is None:
                raise ValueError("Gateway of type 'service' must have service-options.output-topic")
        elif so.input_topic is not None or so.output_topic is not None:
            raise ValueError("Gateway of type 'service' with service-options.agent-id must not include "
                             "service-options.input-topic and service-options.output-topic")


def parse_configuration(content: str, app: Application, defaults: dict) -> None:
    doc = _load_yaml(content) or {}
    conf = doc.get("configuration")
    if conf is None:
        raise ValueError("configuration entry is not present in configuration.yaml")
    if conf.get("defaults") and conf["defaults"].get("globals") is not None:
        defaults["globals"] = conf["defaults"]["globals"]
    for r in conf.get("resources") or []:
        rid = r.get("id") or r.get("name")
        if rid is None:
            raise ValueError("Resource 'name' or 'id' is required")
        app.resources[rid] = Resource(id=rid, name=r.get("name") or rid, type=r.get("type"),
                                      configuration=r.get("configuration") or {})
    deps = conf.get("dependencies")
    if deps:
        app.dependencies = [Dependency(name=d.get("name"), url=d.get("url"), sha512sum=d.get("sha512sum"),
                                       type=d.get("type", "java-library")) for d in deps]
        for d in app.dependencies:
            if d.type != "java-library":
                raise ValueError(f"Unsupported dependency type {d.type}")


def parse_gateways(content: str, app: Application) -> None:
    doc = _load_yaml(content) or {}
    gws = []
    for raw in doc.get("gateways") or []:
        g = Gateway.from_dict(raw)
        validate_gateway(g, raw)
        gws.append(g)
    app.gateways = gws


def parse_pipeline_file(filename: str, content: str, app: Application) -> None:
    try:
        doc = _load_yaml(content) or {}
    except yaml.YAMLError as e:
        raise ValueError(f"Cannot parse file {filename} : {e}") from e
    module_id = doc.get("module") or DEFAULT_MODULE
    module = app.get_module(module_id)
    pid = doc.get("id") or filename.replace(".yaml", "").replace(".yml", "")
    pipeline = module.add_pipeline(pid)
    pipeline.name = doc.get("name")
    res = ResourcesSpec.from_dict(doc.get("resources"))
    pipeline.resources = res.with_defaults_from(ResourcesSpec.DEFAULT) if res else ResourcesSpec.DEFAULT
    err = ErrorsSpec.from_dict(doc.get("errors"))
    pipeline.errors = err.with_defaults_from(ErrorsSpec.DEFAULT) if err else ErrorsSpec.DEFAULT
    validate_errors_spec(pipeline.errors)
    for t in doc.get("topics") or []:
        module.add_topic(TopicDefinition.from_dict(t))
    for a in doc.get("assets") or []:
        module.add_asset(AssetDefinition.from_dict(a))
    last: Optional[AgentConfiguration] = None
    auto_id = 1
    for raw in doc.get("pipeline") or []:
        ag = AgentConfiguration(
            id=None if raw.get("id") is None else str(raw.get("id")), name=raw.get("name"), type=raw.get("type"),
            configuration=dict(raw.get("configuration") or {}),
            resources=(ResourcesSpec.from_dict(raw.get("resources")) or ResourcesSpec()).with_defaults_from(
                pipeline.resources),
            errors=(ErrorsSpec.from_dict(raw.get("errors")) or ErrorsSpec()).with_defaults_from(pipeline.errors),
            executor=raw.get("executor"),
        )
        if not ag.type or not str(ag.type).strip():
            if ag.id is not None:
                raise ValueError(f"Agent type is always required (check agent id {ag.id})")
            if ag.name is not None:
                raise ValueError(f"Agent type is always required (check agent name {ag.name})")
            raise ValueError("Agent type is always required (there is an agent without type, id or name)")
        errors = validate_errors_spec(ag.errors)
        if ag.id is None:
            prefix = "" if module.id == DEFAULT_MODULE else module.id + "-"
            ag.id = f"{prefix}{pipeline.id}-{ag.type}-{auto_id}"
            auto_id += 1
        if raw.get("input") is not None:
            ag.input = Connection.from_topic(module.resolve_topic(raw["input"]))
        if raw.get("output") is not None:
            ag.output = Connection.from_topic(module.resolve_topic(raw["output"]))
        if last is not None and ag.input is None:
            ag.input = Connection.from_agent(last)
            if last.output is None:
                last.output = Connection.from_agent(ag)
                if ag.errors.on_failure == DEAD_LETTER:
                    last.output = last.output.with_deadletter(True)
        if errors.on_failure == DEAD_LETTER and ag.input is not None:
            ag.input = ag.input.with_deadletter(True)
        pipeline.add_agent_configuration(ag)
        last = ag


def parse_instance(content: str, app: Application, default_globals: Optional[dict]) -> None:
    doc = _load_yaml(content) or {}
    inst = doc.get("instance") or {}
    sc = inst.get("streamingCluster")
    cc = inst.get("computeCluster")
    instance = Instance(
        streaming_cluster=StreamingCluster(sc.get("type"), sc.get("configuration") or {}) if sc else None,
        compute_cluster=ComputeCluster(cc.get("type"), cc.get("configuration") or {}) if cc
        else ComputeCluster("kubernetes", {}),
        globals=dict(inst.get("globals") or {}),
    )
    if default_globals:
        for k, v in default_globals.items():
            instance.globals.setdefault(k, v)
    app.instance = instance


def parse_secrets(content: str, app: Application) -> None:
    doc = _load_yaml(content) or {}
    ids = set()
    secrets = {}
    for s in doc.get("secrets") or []:
        sid = s.get("id")
        if sid is None or not str(sid).strip():
            raise ValueError(f"Found secret without id: {s}")
        if sid in ids:
            raise ValueError(f"Found duplicate secret id: {sid}")
        ids.add(sid)
        secrets[sid] = Secret(id=sid, name=s.get("name"), data=s.get("data") or {})
    app.secrets = Secrets(secrets)


def build_application_instance(files: Dict[str, str], instance_content: Optional[str] = None,
                               secrets_content: Optional[str] = None,
                               from_archetype: bool = False) -> ApplicationWithPackageInfo:
    """files: mapping file name -> content of every ``*.yaml`` in the app directory."""
    app = Application()
    info = ApplicationWithPackageInfo(app)
    defaults: dict = {}
    # configuration.yaml first (defaults), then gateways, then pipelines (sorted for determinism)
    order = sorted(files, key=lambda f: (f != "configuration.yaml", f != "gateways.yaml", f))
    for fname in order:
        if not fname.endswith(".yaml"):
            continue
        content = files[fname]
        if fname == "instance.yaml":
            if not from_archetype:
                raise ValueError("instance.yaml must not be included in the application zip")
            instance_content = instance_content or content
        elif fname == "secrets.yaml":
            if not from_archetype:
                raise ValueError("secrets.yaml must not be included in the application zip")
            secrets_content = secrets_content or content
        elif fname == "configuration.yaml":
            info.has_app_definition = True
            parse_configuration(content, app, defaults)
        elif fname == "gateways.yaml":
            info.has_app_definition = True
            parse_gateways(content, app)
        elif fname == "archetype.yaml":
            _load_yaml(content)  # validation only
        else:
            info.has_app_definition = True
            parse_pipeline_file(fname, content, app)
    if instance_content is not None:
        info.has_instance_definition = True
        parse_instance(instance_content, app, defaults.get("globals"))
    elif defaults.get("globals"):
        app.instance = Instance(None, ComputeCluster("kubernetes", {}), dict(defaults["globals"]))
    if secrets_content is not None:
        info.has_secret_definition = True
        parse_secrets(secrets_content, app)
    return info


def read_app_directory(path: str) -> Dict[str, str]:
    files = {}
    for fn in sorted(os.listdir(path)):
        full = os.path.join(path, fn)
        if os.path.isfile(full) and fn.endswith(".yaml"):
            with open(full, encoding="utf-8") as f:
                files[fn] = f.read()
    return files


def build_from_directory(app_dir: str, instance_file: Optional[str] = None,
                         secrets_file: Optional[str] = None) -> ApplicationWithPackageInfo:
    # instance / secrets files get ${ENV:-default} and <file:...> resolution, as the
    # reference CLI does for them (LocalFileReferenceResolver.java:37-160)
    from .file_refs import read_yaml_with_references
    inst = read_yaml_with_references(instance_file) if instance_file else None
    sec = read_yaml_with_references(secrets_file) if secrets_file else None
    info = build_application_instance(read_app_directory(app_dir), inst, sec)
    info.py_binaries_digest = directory_digest(os.path.join(app_dir, "python"))
    info.java_binaries_digest = directory_digest(os.path.join(app_dir, "java", "lib"))
    return info


def directory_digest(path: str) -> Optional[str]:
    """SHA-256 'code changed?' digest, ModelBuilder.java:275-361: a depth-first walk where
    each directory's entries (files and sub-directories together) are visited in name
    order, every file contributing its path relative to ``path`` and then its bytes;
    None when there is no file."""
    if not os.path.isdir(path):
        return None
    h = hashlib.sha256()
    seen = [False]

    def walk(cur: str) -> None:
        for name in sorted(os.listdir(cur)):
            full = os.path.join(cur, name)
            if os.path.isdir(full):
                walk(full)
            elif os.path.isfile(full):
                h.update(os.path.relpath(full, path).replace(os.sep, "/").encode())
                with open(full, "rb") as f:
                    h.update(f.read())
                seen[0] = True

    walk(path)
    return h.hexdigest() if seen[0] else None


# ---------------------------------------------------------------- archetypes
def build_from_archetype(archetype_dir: str, parameters: Dict[str, Any]) -> ApplicationWithPackageInfo:
    files, inst, sec = archetype_application_files(archetype_dir, parameters)
    return build_application_instance(files, inst, sec, from_archetype=True)


def archetype_application_files(archetype_dir: str, parameters: Dict[str, Any]):
    """(application files, instance.yaml text, secrets.yaml text) of an archetype with its
    parameters applied.  An archetype is an app directory plus ``archetype.yaml`` declaring parameters bound
    to ``globals.<path>`` or ``secrets.<id>.<path>`` (``ModelBuilder.java:78-190``): the
    archetype's own instance.yaml and secrets.yaml (both required) are kept, and each
    parameter's value is set at its binding path, creating nested maps on the way
    (``nested-map.key2.key2-1`` replaces one leaf of a map the instance declares)."""
    import copy
    files = read_app_directory(archetype_dir)
    spec = _load_yaml(files.get("archetype.yaml", "")) or {}
    arche = spec.get("archetype") or {}
    if "instance.yaml" not in files:
        raise ValueError("An archetype must always contain an instance.yaml file")
    if "secrets.yaml" not in files:
        raise ValueError("An archetype must always contain an secrets.yaml file")
    instance = (_load_yaml(files.pop("instance.yaml")) or {}).get("instance") or {}
    secret_list = (_load_yaml(files.pop("secrets.yaml")) or {}).get("secrets") or []
    globals_: Dict[str, Any] = copy.deepcopy(instance.get("globals") or {})
    secrets: Dict[str, Any] = {s.get("id"): copy.deepcopy(s.get("data") or {}) for s in secret_list}
    for section in arche.get("sections") or []:
        for p in section.get("parameters") or []:
            name, binding = p.get("name"), p.get("binding")
            if binding is None:
                continue
            value = parameters[name] if name in parameters else p.get("default")
            if p.get("required") and value is None:
                raise ValueError(f"Missing required archetype parameter {name}")
            path = binding.split(".")
            if path[0] == "globals":
                ctx = globals_
            elif path[0] == "secrets":
                ctx = secrets
            else:
                raise ValueError(f"Invalid binding {binding}")
            for key in path[1:-1]:
                nxt = ctx.get(key)
                if not isinstance(nxt, dict):
                    nxt = ctx[key] = {}
                ctx = nxt
            ctx[path[-1]] = value
    new_instance = {k: v for k, v in instance.items() if k != "globals"}
    new_instance["globals"] = globals_
    inst = yaml.safe_dump({"instance": new_instance})
    sec = yaml.safe_dump({"secrets": [{**{k: v for k, v in s.items() if k != "data"}, "data": secrets.get(s.get("id"))}
                                      for s in secret_list]})
    files.pop("archetype.yaml", None)
    return files, inst, sec
