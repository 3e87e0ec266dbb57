"""HTML document normalisation as the reference's crawler emits pages.

The reference's webcrawler parses every fetched page into a document tree (jsoup) and
emits ``document.html()``: the page re-serialised from the tree, pretty-printed
(``WebCrawler.java:259-277``).  Downstream agents (text extraction, splitting) and the
reference's own expectations (``WebCrawlerSourceIT.test``) see that form, so
:func:`parse` here builds the same tree shape and :func:`to_html` prints it with the same
layout rules:

* tree: implicit ``<html>``/``<head>``/``<body>``; head-only elements (``title``,
  ``meta``, ``link``, ``style``, ``script``, ...) before the first body content go to
  ``<head>``; void elements never take children; an end tag closes up to its matching
  open element (unmatched end tags are dropped); a block start tag closes an open ``<p>``,
  ``<li>`` closes the open ``<li>``, ``<dt>``/``<dd>`` and ``<tr>``/``<td>``/``<th>`` close
  their open siblings;
* layout: one space of indent per depth; a block element, or any element whose parent
  formats as a block, starts on a new line unless it is an inline element that follows
  other content; whitespace runs in text collapse to one space and are trimmed at the
  edges of block-formatted parents; whitespace-only text next to a line break is
  dropped; ``pre``/``textarea``/``title`` keep their whitespace; ``script``/``style``
  contents are printed verbatim;
* escaping: ``&``, ``<``, ``>`` and U+00A0 in text; ``&``, ``"`` and U+00A0 in
  attribute values; boolean attributes with an empty value print as the bare name.

:func:`parse` also returns the ``href`` targets of ``<a>`` elements in document order,
which the crawler follows.
"""
from __future__ import annotations

import html.parser
import re
from typing import List, Optional, Tuple

BLOCK = frozenset((
    "html", "head", "body", "frameset", "script", "noscript", "style", "meta", "link", "title", "frame",
    "noframes", "section", "nav", "aside", "hgroup", "header", "footer", "p", "h1", "h2", "h3", "h4", "h5",
    "h6", "ul", "ol", "pre", "div", "blockquote", "hr", "address", "figure", "figcaption", "form", "fieldset",
    "ins", "del", "dl", "dt", "dd", "li", "table", "caption", "thead", "tfoot", "tbody", "colgroup", "col", "tr",
    "th", "td", "video", "audio", "canvas", "details", "menu", "plaintext", "template", "article", "main", "svg",
    "math", "center", "dir", "applet", "marquee", "listing"))
# known inline elements (everything else unknown also prints inline, but formats its
# children as a block, as the reference's tag table does for unregistered tags)
INLINE = frozenset((
    "object", "base", "font", "tt", "i", "b", "u", "big", "small", "em", "strong", "dfn", "code", "samp", "kbd",
    "var", "cite", "abbr", "time", "acronym", "mark", "ruby", "rt", "rp", "rtc", "a", "img", "br", "wbr", "map",
    "q", "sub", "sup", "bdo", "iframe", "embed", "span", "input", "select", "textarea", "label", "button",
    "optgroup", "option", "legend", "datalist", "keygen", "output", "progress", "meter", "area", "param", "source",
    "track", "summary", "command", "device", "basefont", "bgsound", "menuitem", "data", "bdi", "s", "strike",
    "nobr", "rb", "text", "mi", "mo", "msup", "mn", "mtext"))
FORMAT_INLINE = frozenset(("title", "a", "p", "h1", "h2", "h3", "h4", "h5", "h6", "pre", "address", "li", "th",
                           "td", "script", "style", "ins", "del", "s", "button"))
VOID = frozenset(("meta", "link", "base", "frame", "img", "br", "wbr", "embed", "hr", "input", "keygen", "col",
                  "command", "device", "area", "basefont", "bgsound", "menuitem", "param", "source", "track"))
PRESERVE_WS = frozenset(("pre", "plaintext", "title", "textarea", "listing"))
RAW = frozenset(("script", "style"))
HEAD_ONLY = frozenset(("base", "basefont", "bgsound", "link", "meta", "title", "style", "script", "noscript",
                       "template"))
BOOLEAN_ATTRS = frozenset((
    "allowfullscreen", "async", "autofocus", "checked", "compact", "declare", "default", "defer", "disabled",
    "formnovalidate", "hidden", "inert", "ismap", "itemscope", "multiple", "muted", "nohref", "noresize",
    "noshade", "novalidate", "nowrap", "open", "readonly", "required", "reversed", "seamless", "selected",
    "sortable", "truespeed", "typemustmatch"))
_CLOSES_P = BLOCK - frozenset(("html", "head", "body", "script", "style", "meta", "link", "title", "noscript",
                               "ins", "del", "frame", "noframes", "col", "colgroup", "caption", "thead", "tfoot",
                               "tbody", "tr", "th", "td", "li", "dt", "dd", "video", "audio", "canvas", "svg",
                               "math", "template", "applet", "marquee"))
_WS = re.compile(r"[ \t\n\r\f]+")


def _is_block(tag: str) -> bool:
    return tag in BLOCK


def _format_as_block(tag: str) -> bool:
    if tag in FORMAT_INLINE or tag in INLINE:
        return False
    return True


class Node:
    __slots__ = ("parent", "index")

    def __init__(self):
        self.parent: Optional["Element"] = None
        self.index = 0


class Text(Node):
    __slots__ = ("text",)

    def __init__(self, text: str):
        super().__init__()
        self.text = text

    def blank(self) -> bool:
        return not self.text.strip(" \t\n\r\f")


class Data(Text):
    """script / style contents: printed verbatim."""
    __slots__ = ()


class Comment(Node):
    __slots__ = ("data",)

    def __init__(self, data: str):
        super().__init__()
        self.data = data


class Doctype(Node):
    __slots__ = ("decl",)

    def __init__(self, decl: str):
        super().__init__()
        self.decl = decl


class Element(Node):
    __slots__ = ("tag", "attrs", "children")

    def __init__(self, tag: str, attrs=None):
        super().__init__()
        self.tag = tag
        self.attrs: List[Tuple[str, str]] = []
        self.merge(attrs or [])
        self.children: List[Node] = []

    def merge(self, attrs) -> None:
        have = {k for k, _ in self.attrs}
        for k, v in attrs:
            if k not in have:
                self.attrs.append((k, "" if v is None else v))
                have.add(k)

    def append(self, n: Node) -> None:
        if isinstance(n, Text) and not isinstance(n, Data) and self.children and \
                type(self.children[-1]) is Text:
            self.children[-1].text += n.text
            return
        n.parent = self
        n.index = len(self.children)
        self.children.append(n)


class Document(Element):
    __slots__ = ()

    def __init__(self):
        super().__init__("#document")


class _Builder(html.parser.HTMLParser):
    def __init__(self):
        super().__init__(convert_charrefs=True)
        self.doc = Document()
        self.html = Element("html")
        self.head = Element("head")
        self.body = Element("body")
        self.html.append(self.head)
        self.html.append(self.body)
        self.in_body = False
        self.head_stack: List[Element] = [self.head]
        self.stack: List[Element] = [self.body]
        self.doctype: Optional[Doctype] = None
        self.hrefs: List[str] = []

    # ---- helpers
    def _cur(self) -> Element:
        return self.stack[-1] if self.in_body else self.head_stack[-1]

    def _enter_body(self) -> None:
        self.in_body = True

    def _close(self, tag: str, stop=("body",)) -> bool:
        for i in range(len(self.stack) - 1, 0, -1):
            t = self.stack[i].tag
            if t == tag:
                del self.stack[i:]
                return True
            if t in stop:
                break
        return False

    def _in_stack(self, tag: str, barrier=()) -> bool:
        for e in reversed(self.stack):
            if e.tag == tag:
                return True
            if e.tag in barrier:
                return False
        return False

    # ---- parser callbacks
    def handle_decl(self, decl):
        if decl.lower().startswith("doctype") and self.doctype is None:
            self.doctype = Doctype(decl)

    def handle_starttag(self, tag, attrs):
        if tag == "html":
            self.html.merge(attrs)
            return
        if tag == "head":
            if not self.in_body:
                self.head.merge(attrs)
            return
        if tag == "body":
            self._enter_body()
            self.body.merge(attrs)
            return
        if not self.in_body and tag in HEAD_ONLY and len(self.head_stack) == 1:
            e = Element(tag, attrs)
            self.head.append(e)
            if tag not in VOID:
                self.head_stack.append(e)
            return
        if not self.in_body:
            if len(self.head_stack) > 1:      # inside <title>/<noscript>...: keep it there
                e = Element(tag, attrs)
                self.head_stack[-1].append(e)
                if tag not in VOID:
                    self.head_stack.append(e)
                return
            self._enter_body()
        # implied end tags
        if tag in _CLOSES_P and self._in_stack("p", barrier=("table", "td", "th", "button")):
            self._close("p")
        if tag == "li" and self._in_stack("li", barrier=("ul", "ol")):
            self._close("li", stop=("ul", "ol", "body"))
        elif tag in ("dt", "dd"):
            for t in ("dt", "dd"):
                if self._in_stack(t, barrier=("dl",)):
                    self._close(t, stop=("dl", "body"))
        elif tag in ("td", "th"):
            for t in ("td", "th"):
                if self._in_stack(t, barrier=("tr", "table")):
                    self._close(t, stop=("tr", "table", "body"))
        elif tag == "tr" and self._in_stack("tr", barrier=("table",)):
            self._close("tr", stop=("table", "body"))
        elif tag == "option" and self.stack[-1].tag == "option":
            self.stack.pop()
        e = Element(tag, attrs)
        self.stack[-1].append(e)
        if tag == "a":
            for k, v in e.attrs:
                if k == "href":
                    self.hrefs.append(v)
        if tag not in VOID:
            self.stack.append(e)

    def handle_startendtag(self, tag, attrs):
        self.handle_starttag(tag, attrs)
        if tag not in VOID:
            self.handle_endtag(tag)

    def handle_endtag(self, tag):
        if tag in ("html", "body", "head"):
            if tag == "head" and not self.in_body:
                del self.head_stack[1:]
            return
        if not self.in_body:
            for i in range(len(self.head_stack) - 1, 0, -1):
                if self.head_stack[i].tag == tag:
                    del self.head_stack[i:]
                    return
            return
        self._close(tag)

    def handle_data(self, data):
        cur = self._cur()
        if cur.tag in RAW:
            cur.append(Data(data))
            return
        if not self.in_body:
            if len(self.head_stack) > 1:
                cur.append(Text(data))
                return
            if not data.strip(" \t\n\r\f"):
                return
            self._enter_body()
            cur = self._cur()
        cur.append(Text(data))

    def handle_comment(self, data):
        self._cur().append(Comment(data))


def parse(markup: str) -> Tuple[Document, List[str]]:
    b = _Builder()
    b.feed(markup)
    b.close()
    if b.doctype is not None:
        b.doc.append(b.doctype)
    b.doc.append(b.html)
    return b.doc, b.hrefs


# ---------------------------------------------------------------- serialisation
def _escape(s: str, attr: bool) -> str:
    s = s.replace("&", "&amp;").replace(" ", "&nbsp;")
    if attr:
        return s.replace('"', "&quot;")
    return s.replace("<", "&lt;").replace(">", "&gt;")


def _preserve(n: Optional[Node]) -> bool:
    depth = 0
    while isinstance(n, Element) and depth < 6:
        if n.tag in PRESERVE_WS:
            return True
        n = n.parent
        depth += 1
    return False


def _prev(n: Node) -> Optional[Node]:
    return n.parent.children[n.index - 1] if n.parent is not None and n.index > 0 else None


def _next(n: Node) -> Optional[Node]:
    if n.parent is None or n.index + 1 >= len(n.parent.children):
        return None
    return n.parent.children[n.index + 1]


def _effectively_first(n: Node) -> bool:
    if n.index == 0:
        return True
    if n.index == 1:
        p = _prev(n)
        return isinstance(p, Text) and p.blank()
    return False


def _should_indent(e: Element) -> bool:
    p = e.parent
    as_block = _is_block(e.tag) or (isinstance(p, Element) and _format_as_block(p.tag))
    inlineable = (not _is_block(e.tag)) and (p is None or isinstance(p, Document) or _is_block(p.tag)) \
        and not _effectively_first(e) and e.tag != "br"
    return as_block and not inlineable and not _preserve(p)


def _indent(out: List[str], depth: int) -> None:
    out.append("\n" + " " * depth)


def _text(n: Text, depth: int, out: List[str]) -> None:
    p = n.parent
    if isinstance(n, Data) or _preserve(p):
        out.append(n.text if isinstance(n, Data) else _escape(n.text, False))
        return
    like_block = isinstance(p, Element) and not isinstance(p, Document) and \
        (_is_block(p.tag) or _format_as_block(p.tag))
    trim_lead = (like_block and n.index == 0) or isinstance(p, Document)
    nxt, prv = _next(n), _prev(n)
    trim_trail = like_block and nxt is None
    blank = n.blank()
    could_skip = (isinstance(nxt, Element) and _should_indent(nxt)) or \
        (isinstance(nxt, Text) and nxt.blank()) or (isinstance(prv, Element) and _is_block(prv.tag))
    if could_skip and blank:
        return
    if (n.index == 0 and isinstance(p, Element) and _format_as_block(p.tag) and not blank) or \
            (n.index > 0 and isinstance(prv, Element) and prv.tag == "br"):
        _indent(out, depth)
    s = _WS.sub(" ", n.text)
    if trim_lead:
        s = s.lstrip(" ")
    if trim_trail:
        s = s.rstrip(" ")
    out.append(_escape(s, False))


def _attrs(e: Element) -> str:
    parts = []
    for k, v in e.attrs:
        if k in BOOLEAN_ATTRS and (v == "" or v.lower() == k):
            parts.append(" " + k)
        else:
            parts.append(f' {k}="{_escape(v, True)}"')
    return "".join(parts)


def _node(n: Node, depth: int, out: List[str]) -> None:
    if isinstance(n, Text):
        _text(n, depth, out)
        return
    if isinstance(n, Comment):
        p = n.parent
        if _effectively_first(n) and isinstance(p, Element) and not isinstance(p, Document) and \
                _format_as_block(p.tag):
            _indent(out, depth)
        out.append(f"<!--{n.data}-->")
        return
    if isinstance(n, Doctype):
        if n.index > 0:
            out.append("\n")
        rest = n.decl[len("doctype"):].strip()
        out.append("<!doctype" + (" " + rest if rest else "") + ">")
        return
    e: Element = n  # type: ignore[assignment]
    if _should_indent(e):
        _indent(out, depth)
    out.append(f"<{e.tag}{_attrs(e)}>")
    if e.tag in VOID:
        return
    for c in e.children:
        _node(c, depth + 1, out)
    if e.children and _format_as_block(e.tag) and not _preserve(e.parent):
        _indent(out, depth)
    out.append(f"</{e.tag}>")


def to_html(doc: Document) -> str:
    out: List[str] = []
    for c in doc.children:
        _node(c, 0, out)
    return "".join(out).strip()


def normalize(markup: str) -> Tuple[str, List[str]]:
    """(pretty-printed document HTML, ``<a href>`` targets in document order)."""
    doc, hrefs = parse(markup)
    return to_html(doc), hrefs
