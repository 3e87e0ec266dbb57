"""Placeholder resolution for applications.

Parity: CORE/common/ApplicationPlaceholderResolver.java:59-377.
Context = {cluster: {type, configuration}, globals: instance.globals, secrets: {id: data}}.
* ``${a.b.c}`` as the WHOLE value -> the referenced object (type preserved)
* inside a string -> interpolation; non-string values are JSON-encoded, null -> ""
* legacy ``{{ }}`` / ``{{{ }}}`` only for ``secrets.*`` / ``globals.*`` (0.x apps);
  mustache-style references to anything else are left untouched for the agents.
Applies to instance, resources, module topics (names), asset configs, agent
configurations and connections, gateway topic / events-topic and auth config.
"""
from __future__ import annotations

import copy
import dataclasses
import json
from typing import Any, Dict, Optional

from ..api.model import Application, Connection, Instance, Resource, StreamingCluster, ComputeCluster


def create_context(app: Application) -> Dict[str, Any]:
    ctx: Dict[str, Any] = {}
    if app.instance is not None:
        sc = app.instance.streaming_cluster
        ctx["cluster"] = {"type": sc.type, "configuration": copy.deepcopy(sc.configuration)} if sc else None
        ctx["globals"] = copy.deepcopy(app.instance.globals or {})
    secrets = {}
    if app.secrets is not None:
        for k, s in app.secrets.secrets.items():
            secrets[k] = copy.deepcopy(s.data)
    ctx["secrets"] = secrets
    return ctx


def resolve_reference(placeholder: str, context: Any) -> Any:
    placeholder = placeholder.strip()
    cur = context
    parts = placeholder.split(".")
    for i, p in enumerate(parts):
        if cur is None:
            raise ValueError(f"Cannot resolve reference {placeholder}: {'.'.join(parts[:i])} is empty")
        if not isinstance(cur, dict):
            raise ValueError(f"Cannot resolve property {p} on {cur!r} (reference {placeholder})")
        if i < len(parts) - 1 and cur.get(p) is None:
            raise ValueError(f"Cannot resolve reference {placeholder}: property {p} is not set")
        cur = cur.get(p)
    return cur


def _to_str(v: Any) -> str:
    if v is None:
        return ""
    if isinstance(v, str):
        return v
    # Jackson's compact form: "123-[1,2]" (ApplicationPlaceholderResolverTest.testResolve)
    return json.dumps(v, separators=(",", ":"), ensure_ascii=False)


def resolve_in_string(template: str, context: Dict[str, Any]) -> str:
    if "${" not in template and "{{" in template and "}}" in template:
        if "{{{" in template:
            return _interpolate(template, context, "{{{", "}}}", ("secrets", "globals"))
        return _interpolate(template, context, "{{", "}}", ("secrets", "globals"))
    return _interpolate(template, context, "${", "}", None)


def _interpolate(template: str, context, prefix: str, suffix: str, allowed_roots) -> str:
    pos = template.find(prefix)
    if pos < 0:
        return template
    out = []
    position = 0
    while pos >= 0:
        out.append(template[position:pos])
        end = template.find(suffix, pos)
        if end < 0:
            raise ValueError("Invalid placeholder: " + template)
        ph = template[pos + len(prefix): end].strip()
        if allowed_roots is not None and not any(ph.startswith(r) for r in allowed_roots):
            return template  # mustache template for the agent, not a placeholder
        out.append(_to_str(resolve_reference(ph, context)))
        position = end + len(suffix)
        pos = template.find(prefix, position)
    out.append(template[position:])
    return "".join(out)


def resolve_single_value(context: Dict[str, Any], template: Any) -> Any:
    if not isinstance(template, str):
        return template
    ref = template.strip()
    if not (ref.startswith("${") and ref.endswith("}")):
        return resolve_in_string(template, context)
    if ref.find("{") == ref.rfind("{"):
        return resolve_reference(ref[2:-1], context)
    return resolve_in_string(template, context)


def resolve_value(context: Dict[str, Any], v: Any) -> Any:
    if isinstance(v, dict):
        return {k: resolve_value(context, x) for k, x in v.items()}
    if isinstance(v, list):
        return [resolve_value(context, x) for x in v]
    if isinstance(v, str):
        return resolve_single_value(context, v)
    return v


def resolve_map(context, m: Optional[dict]) -> dict:
    return {} if m is None else resolve_value(context, m)


def _resolve_connection(context, c: Optional[Connection]) -> Optional[Connection]:
    if c is None or c.connection_type != "TOPIC":
        return c
    return Connection(c.connection_type, _str(resolve_single_value(context, c.definition)), c.enable_dead_letter_queue)


def _str(v):
    return None if v is None else str(v)


def resolve_placeholders(app: Application) -> Application:
    app = app.copy()
    ctx = create_context(app)
    if app.instance is not None:
        inst = app.instance
        sc = inst.streaming_cluster
        cc = inst.compute_cluster
        app.instance = Instance(
            StreamingCluster(sc.type, resolve_map(ctx, sc.configuration)) if sc else None,
            ComputeCluster(cc.type, resolve_map(ctx, cc.configuration)) if cc else None,
            resolve_map(ctx, inst.globals))
    app.resources = {k: Resource(r.id, r.name, r.type, resolve_map(ctx, r.configuration))
                     for k, r in app.resources.items()}
    for module in app.modules.values():
        new_topics = {}
        for name, t in module.topics.items():
            nt = t.copy()
            nt.name = _str(resolve_single_value(ctx, nt.name))
            new_topics[_str(resolve_single_value(ctx, name))] = nt
        module.topics = new_topics
        for a in module.assets:
            a.config = resolve_map(ctx, a.config)
        for p in module.pipelines.values():
            for ag in p.agents:
                ag.configuration = resolve_map(ctx, ag.configuration)
                ag.input = _resolve_connection(ctx, ag.input)
                ag.output = _resolve_connection(ctx, ag.output)
    for g in app.gateways:
        if g.authentication is not None and g.authentication.configuration:
            g.authentication = dataclasses.replace(
                g.authentication, configuration=resolve_map(ctx, g.authentication.configuration))
        g.topic = _str(resolve_single_value(ctx, g.topic))
        g.events_topic = _str(resolve_single_value(ctx, g.events_topic))
    return app
