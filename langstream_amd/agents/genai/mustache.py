"""Mustache templates for prompts / http bodies (the reference uses JMustache:
``Mustache.compiler().compile(...)`` in ChatCompletionsStep.java:84-95, with the 0.x
``{{% }}`` legacy syntax mapped by MustacheCompatibilityUtils).

Supported: ``{{ name.path }}`` (HTML-escaped like JMustache's default escaper),
``{{{ raw }}}`` / ``{{& raw}}``, sections ``{{# list}}...{{/ list}}`` (iterate lists,
enter maps, truthy guards), inverted ``{{^ x}}...{{/ x}}``, comments ``{{! }}``,
``{{.}}`` / ``{{this}}`` for the current element, and parent-context fallback.
"""
from __future__ import annotations

import functools
import json
import re
from typing import Any, List

_TAG = re.compile(r"\{\{\{\s*(.+?)\s*\}\}\}|\{\{\s*([#^/&!]?)\s*(.*?)\s*\}\}", re.S)
_ESC = {"&": "&amp;", "'": "&#39;", '"': "&quot;", "<": "&lt;", ">": "&gt;", "`": "&#x60;", "=": "&#x3D;"}


_ESC_TABLE = str.maketrans(_ESC)


def _escape(s: str) -> str:
    return s.translate(_ESC_TABLE)


def _to_str(v: Any) -> str:
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    if isinstance(v, float) and v.is_integer():
        return str(v)
    return str(v)


class _Node:
    __slots__ = ("kind", "name", "children")

    def __init__(self, kind, name=None, children=None):
        self.kind = kind
        self.name = name
        self.children = children


def _parse(template: str) -> List[_Node]:
    root: List[_Node] = []
    stack = [(None, root)]
    pos = 0
    for m in _TAG.finditer(template):
        if m.start() > pos:
            stack[-1][1].append(_Node("text", template[pos:m.start()]))
        pos = m.end()
        if m.group(1) is not None:
            stack[-1][1].append(_Node("raw", m.group(1).strip()))
            continue
        sigil, name = m.group(2), m.group(3).strip()
        if sigil == "!":
            continue
        if sigil in ("#", "^"):
            node = _Node("section" if sigil == "#" else "inverted", name, [])
            stack[-1][1].append(node)
            stack.append((name, node.children))
        elif sigil == "/":
            if len(stack) == 1 or stack[-1][0] != name:
                raise ValueError(f"Mismatched section close {{{{/{name}}}}}")
            stack.pop()
        elif sigil == "&":
            stack[-1][1].append(_Node("raw", name))
        else:
            stack[-1][1].append(_Node("var", name))
    if len(stack) != 1:
        raise ValueError(f"Unclosed section {stack[-1][0]}")
    if pos < len(template):
        root.append(_Node("text", template[pos:]))
    return root


_MISSING = object()


def _lookup(name: str, stack: List[Any]) -> Any:
    if name in (".", "this"):
        return stack[-1]
    parts = name.split(".")
    for ctx in reversed(stack):
        v = _resolve_first(ctx, parts[0])
        if v is _MISSING:
            continue
        for p in parts[1:]:
            v = _resolve_first(v, p)
            if v is _MISSING:
                return None
        return v
    return None


def _resolve_first(ctx: Any, key: str) -> Any:
    if isinstance(ctx, dict):
        return ctx[key] if key in ctx else _MISSING
    if isinstance(ctx, (list, tuple)) and key.isdigit():
        i = int(key)
        return ctx[i] if i < len(ctx) else _MISSING
    if isinstance(ctx, str):
        try:
            d = json.loads(ctx)
        except ValueError:
            return _MISSING
        return d[key] if isinstance(d, dict) and key in d else _MISSING
    return _MISSING


def _render(nodes: List[_Node], stack: List[Any], out: List[str]) -> None:
    for n in nodes:
        k = n.kind
        if k == "text":
            out.append(n.name)
        elif k == "var":
            out.append(_escape(_to_str(_lookup(n.name, stack))))
        elif k == "raw":
            out.append(_to_str(_lookup(n.name, stack)))
        elif k == "section":
            v = _lookup(n.name, stack)
            if isinstance(v, (list, tuple)):
                for item in v:
                    _render(n.children, stack + [item], out)
            elif isinstance(v, dict):
                _render(n.children, stack + [v], out)
            elif v not in (None, False, "", 0):
                _render(n.children, stack + [v], out)
        elif k == "inverted":
            v = _lookup(n.name, stack)
            if v in (None, False, "", 0) or (isinstance(v, (list, tuple, dict)) and not v):
                _render(n.children, stack, out)


class Template:
    def __init__(self, template: str):
        if template is None:
            template = ""
        if "{{%" in template:  # legacy 0.x syntax
            template = template.replace("{{%", "{{")
        self.source = template
        self._nodes = _parse(template)

    def render(self, context: Any) -> str:
        out: List[str] = []
        _render(self._nodes, [context], out)
        return "".join(out)


@functools.lru_cache(maxsize=1024)
def compile_template(template: str) -> Template:
    return Template(template)


def render(template: str, context: Any) -> str:
    return compile_template(template).render(context)
