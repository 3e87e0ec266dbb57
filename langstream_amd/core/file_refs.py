"""Local file and environment references in app / instance / secrets YAML files.

Parity: langstream-cli/.../util/LocalFileReferenceResolver.java:37-160 -- applied by the
CLI to every YAML file it reads from disk, before the files reach the parser:

* the file must parse as YAML (fail fast), and is returned untouched when it contains
  neither ``<file:`` nor ``${``;
* every STRING value (map values and list items, recursively; keys are left alone) is
  first passed through an environment substitution with Apache ``StringSubstitutor``
  semantics: ``${VAR}`` -> the variable's value (left as-is when unset),
  ``${VAR:-default}`` -> the value, or ``default`` when unset or empty, ``$${VAR}`` ->
  the literal ``${VAR}``; a default may itself hold ``${...}`` references;
* then each ``<file:path>`` is replaced by the file's contents, the path relative to the
  directory of the YAML file: text files (``.txt .yaml .yml .json .text``) verbatim,
  anything else as ``base64:<base64 of the bytes>``.

Substituted values stay strings (so ``"${PORT:-8983}"`` becomes ``"8983"``); the config
validator coerces them to the declared types.
"""
from __future__ import annotations

import base64
import os
import re
from typing import Any, Callable, Mapping, Optional

import yaml

_FILE = re.compile(r"<file:(.*?)>")
_TEXT_EXT = ("txt", "yaml", "yml", "json", "text")


def substitute_env(s: str, env: Optional[Mapping[str, str]] = None) -> str:
    """``StringSubstitutor(System.getenv()).replace(s)``."""
    env = os.environ if env is None else env
    out = []
    i, n = 0, len(s)
    while i < n:
        if s.startswith("$${", i):           # escaped: keep one '$' and the reference verbatim
            end = _match_brace(s, i + 2)
            if end < 0:
                out.append(s[i:])
                break
            out.append(s[i + 1:end + 1])
            i = end + 1
            continue
        if s.startswith("${", i):
            end = _match_brace(s, i + 1)
            if end < 0:
                out.append(s[i:])
                break
            body = s[i + 2:end]
            name, sep, default = body.partition(":-")
            name = substitute_env(name, env)
            val = env.get(name)
            if val is None or (sep and val == ""):
                val = substitute_env(default, env) if sep else s[i:end + 1]
            out.append(val)
            i = end + 1
            continue
        out.append(s[i])
        i += 1
    return "".join(out)


def _match_brace(s: str, open_idx: int) -> int:
    """Index of the '}' closing the '{' at ``open_idx`` (nested ``${...}`` allowed)."""
    depth = 0
    for j in range(open_idx, len(s)):
        c = s[j]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return j
    return -1


def read_file_reference(base_dir: str, filename: str) -> str:
    path = os.path.join(base_dir, filename)
    try:
        if filename.lower().endswith(_TEXT_EXT):
            with open(path, encoding="utf-8") as f:
                return f.read()
        with open(path, "rb") as f:
            return "base64:" + base64.b64encode(f.read()).decode()
    except OSError as e:
        raise ValueError(f"Cannot read file {path}") from e


def resolve_references_in_string(s: str, read_file: Callable[[str], str],
                                 env: Optional[Mapping[str, str]] = None) -> str:
    s = substitute_env(s, env)
    return _FILE.sub(lambda m: read_file(m.group(1)), s)


def _walk(v: Any, read_file, env) -> Any:
    if isinstance(v, str):
        return resolve_references_in_string(v, read_file, env)
    if isinstance(v, dict):
        return {k: _walk(x, read_file, env) for k, x in v.items()}
    if isinstance(v, list):
        return [_walk(x, read_file, env) for x in v]
    return v


def resolve_file_references(content: str, base_dir: str, env: Optional[Mapping[str, str]] = None) -> str:
    """Resolve ``${ENV}`` and ``<file:...>`` references in one YAML document."""
    try:
        data = yaml.safe_load(content)
    except yaml.YAMLError as e:
        raise ValueError(f"Cannot parse YAML file: {e}") from e
    if not _FILE.search(content) and "${" not in content:
        return content
    if data is None:
        return content
    resolved = _walk(data, lambda fn: read_file_reference(base_dir, fn), env)
    # re-serialised as the reference's YAML printer writes it (AppsCmdTest.testDeployWithFilePlaceholders)
    from ..cli.printer import jackson_yaml
    return jackson_yaml(resolved) + "\n"


def read_yaml_with_references(path: str, env: Optional[Mapping[str, str]] = None) -> str:
    with open(path, encoding="utf-8") as f:
        content = f.read()
    return resolve_file_references(content, os.path.dirname(os.path.abspath(path)), env)
