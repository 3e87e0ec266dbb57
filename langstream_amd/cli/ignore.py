"""``.langstreamignore``: gitignore-style exclusion of files from the application zip the
CLI uploads (``langstream-cli/.../commands/GitIgnoreParser.java:30-205``, used by
``utils/ApplicationPackager.java:44-80``).

Rule semantics follow the reference, not full git: each pattern is a Java ``glob:``
matched against the path relative to the ignore file's directory; a pattern with a
slash before its last character is anchored there, otherwise it also matches at any
depth (``**/<pattern>``); a trailing slash restricts it to directories; ``!`` negates;
the last matching rule wins.  Comments, blank lines, ``***`` and double asterisks not at
either end or between slashes are ignored.  A matched directory is not descended into
by the packager, but the parser itself does not propagate a match to children
(``lll*`` does not match ``lll/m``), as in the reference.
"""
from __future__ import annotations

import os
import re
from typing import List, Optional, Tuple

_Rule = Tuple["re.Pattern[str]", bool, bool]   # (regex, negation, directory_only)


def glob_to_regex(glob: str) -> str:
    """Java ``FileSystem.getPathMatcher("glob:...")`` syntax as a regex: ``*`` within one
    path component, ``**`` across components, ``?`` one non-separator character,
    ``[...]`` classes (``[!...]`` negated), ``{a,b}`` alternatives, ``\\`` escapes."""
    out, i, n, in_group = [], 0, len(glob), False
    while i < n:
        c = glob[i]
        if c == "\\" and i + 1 < n:
            out.append(re.escape(glob[i + 1]))
            i += 2
            continue
        if c == "*":
            if i + 1 < n and glob[i + 1] == "*":
                out.append(".*")
                i += 2
                continue
            out.append("[^/]*")
        elif c == "?":
            out.append("[^/]")
        elif c == "[":
            j = glob.find("]", i + 1)
            if j < 0:
                raise ValueError(f"unclosed character class in glob {glob!r}")
            body = glob[i + 1:j]
            neg = body.startswith("!")
            if neg:
                body = body[1:]
            body = body.replace("\\", "\\\\").replace("^", "\\^")
            out.append(("[^/" if neg else "[") + body + "]")
            i = j
        elif c == "{" and not in_group:
            out.append("(?:")
            in_group = True
        elif c == "}" and in_group:
            out.append(")")
            in_group = False
        elif c == "," and in_group:
            out.append("|")
        else:
            out.append(re.escape(c))
        i += 1
    return "".join(out)


def rules_from_pattern(pattern: str) -> List[_Rule]:
    if not pattern.strip() or pattern.startswith("#") or "***" in pattern:
        return []
    negation = pattern.startswith("!")
    if negation:
        pattern = pattern[1:]
    for m in re.finditer(r"\*\*", pattern):
        s = m.start()
        if s not in (0, len(pattern) - 2) and (pattern[s - 1] != "/" or pattern[s + 2:s + 3] != "/"):
            return []
    if pattern.strip() == "/":
        return []
    if pattern.startswith("**/"):
        pattern = pattern[3:]
    anchored = "/" in pattern[:-1]
    if anchored:
        pattern = pattern.lstrip("/")
    directory_only = pattern.endswith("/")
    if directory_only:
        pattern = pattern[:-1]
    if pattern.startswith("\\#"):
        pattern = pattern[1:]
    # trailing spaces dropped unless escaped
    stripped = pattern.rstrip(" ")
    if stripped.endswith("\\") and len(stripped) < len(pattern):
        pattern = stripped[:-1] + pattern[len(stripped):]
    else:
        pattern = stripped
    rules = [(re.compile(glob_to_regex(pattern), re.S), negation, directory_only)]
    if not anchored:
        rules.append((re.compile(glob_to_regex("**/" + pattern), re.S), negation, directory_only))
    return rules


class IgnoreRules:
    def __init__(self, rules: List[_Rule], base: str):
        self.rules = rules
        self.base = os.path.abspath(base)

    @classmethod
    def from_file(cls, path: str) -> "IgnoreRules":
        rules: List[_Rule] = []
        with open(path, encoding="utf-8") as f:
            for line in f:
                rules.extend(rules_from_pattern(line.strip()))
        return cls(rules, os.path.dirname(os.path.abspath(path)))

    def matches(self, path: str, is_dir: bool) -> bool:
        rel = os.path.relpath(os.path.abspath(path), self.base).replace(os.sep, "/")
        hit = False
        for rx, neg, dir_only in self.rules:
            if dir_only and not is_dir:
                continue
            if rx.fullmatch(rel):
                hit = not neg
        return hit


def load_ignore(app_dir: str) -> Optional[IgnoreRules]:
    p = os.path.join(app_dir, ".langstreamignore")
    return IgnoreRules.from_file(p) if os.path.isfile(p) else None
