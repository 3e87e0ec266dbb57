"""Text-processing agents (TXT/*): text-extractor, language-detector, text-normaliser,
document-to-json, text-splitter.

* text-splitter: recursive character splitter (TXT/RecursiveCharacterTextSplitter.java:22-86,
  TXT/TextSplitter.java merge/overlap logic, TXT/TextSplitterAgent.java:30-124): separators
  ["\\n\\n","\\n"," ",""], chunk_size 200, chunk_overlap 100, keep_separator false,
  length_function cl100k_base (native C++ BPE counter) or length; one record per chunk
  with the ORIGINAL key and headers chunk_id / chunk_text_length / chunk_num_tokens /
  text_num_chunks.
* text-extractor: Tika AutoDetect in the reference; here: plain text, HTML, XML, JSON,
  DOCX/PPTX/XLSX/ODT (zip + XML), RTF, and PDF text streams (uncompressed / Flate).
* language-detector: character 1-3-gram profiles scored naive-Bayes (the n-gram
  approach of Tika's LanguageIdentifier in the reference) -> header ``language``
  (configurable), ``allowedLanguages`` filter.
"""
from __future__ import annotations

import html
import html.parser
import io
import json
import re
import zipfile
import zlib
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api.agent import SingleRecordAgentProcessor
from ..api.record import Header, SimpleRecord
from ..runtime.registry import register_agent


def to_text(v: Any) -> str:
    if v is None:
        return ""
    if isinstance(v, bytes):
        return v.decode("utf-8", errors="replace")
    if isinstance(v, str):
        return v
    if isinstance(v, (dict, list)):
        return json.dumps(v)
    return str(v)


# ---------------------------------------------------------------- splitter
class RecursiveCharacterTextSplitter:
    def __init__(self, separators: Optional[List[str]] = None, keep_separator: bool = False, chunk_size: int = 200,
                 chunk_overlap: int = 100, length_function: Callable[[str], int] = len):
        if chunk_overlap > chunk_size:
            raise ValueError(f"Got a larger chunk overlap ({chunk_overlap}) than chunk size ({chunk_size}), "
                             f"should be smaller.")
        self.separators = separators if separators is not None else ["\n\n", "\n", " ", ""]
        self.keep_separator = keep_separator
        self.chunk_size = chunk_size
        self.chunk_overlap = chunk_overlap
        self.length = length_function

    @staticmethod
    def _split_regex(text: str, sep: str, keep: bool) -> List[str]:
        if sep:
            if keep:
                ms = list(re.finditer(f"({sep})", text))
                if not ms:
                    splits = [text]
                else:
                    splits = []
                    if ms[0].start() != 0:
                        splits.append(text[: ms[0].start()])
                    for i, m in enumerate(ms):
                        end = ms[i + 1].start() if i + 1 < len(ms) else len(text)
                        splits.append(m.group() + text[m.end(): end])
            else:
                splits = re.split(sep, text)
        else:
            splits = list(text)
        return [s for s in splits if s]

    def _join(self, docs: List[str], sep: str) -> Optional[str]:
        t = sep.join(docs).strip()
        return t or None

    def _merge(self, splits: List[Tuple[str, int]], sep: str) -> List[str]:
        """``splits``: (piece, length) pairs -- each piece's length is computed once by
        the caller (the length function is a BPE count: the dominant cost of a split)."""
        docs: List[str] = []
        cur: List[str] = []
        cur_len: List[int] = []
        total = 0
        sep_len = self.length(sep) if sep else 0
        for d, ln in splits:
            if total + ln + (sep_len if cur else 0) > self.chunk_size:
                if cur:
                    doc = self._join(cur, sep)
                    if doc is not None:
                        docs.append(doc)
                    while total > self.chunk_overlap or (
                            total + ln + (sep_len if cur else 0) > self.chunk_size and total > 0):
                        total -= cur_len[0] + (sep_len if len(cur) > 1 else 0)
                        cur.pop(0)
                        cur_len.pop(0)
            cur.append(d)
            cur_len.append(ln)
            total += ln + (sep_len if len(cur) > 1 else 0)
        doc = self._join(cur, sep)
        if doc is not None:
            docs.append(doc)
        return docs

    def _split(self, text: str, separators: List[str]) -> List[str]:
        final: List[str] = []
        separator = separators[-1]
        new_seps: List[str] = []
        for i, s in enumerate(separators):
            if s == "":
                separator = s
                break
            if re.search(s, text):
                separator = s
                new_seps = separators[i + 1:]
                break
        splits = self._split_regex(text, separator, self.keep_separator)
        good: List[Tuple[str, int]] = []
        sep_use = "" if self.keep_separator else separator
        for s in splits:
            ln = self.length(s)
            if ln < self.chunk_size:
                good.append((s, ln))
            else:
                if good:
                    final.extend(self._merge(good, sep_use))
                    good = []
                if not new_seps:
                    final.append(s)
                else:
                    final.extend(self._split(s, new_seps))
        if good:
            final.extend(self._merge(good, sep_use))
        return final

    def split_text(self, text: str) -> List[str]:
        return self._split(text, self.separators)


@register_agent("text-splitter")
class TextSplitterAgent(SingleRecordAgentProcessor):
    def init(self, configuration: Dict[str, Any]) -> None:
        st = str(configuration.get("splitter_type", "RecursiveCharacterTextSplitter"))
        if st != "RecursiveCharacterTextSplitter":
            raise ValueError(f"Unknown splitter type: {st}, only RecursiveCharacterTextSplitter is supported")
        lf = str(configuration.get("length_function", "cl100k_base"))
        if lf == "length":
            self.length = len
        else:
            from ..tokenizers import cl100k_counter
            self.length = cl100k_counter()
        self.splitter = RecursiveCharacterTextSplitter(
            configuration.get("separators", ["\n\n", "\n", " ", ""]),
            str(configuration.get("keep_separator", "false")).lower() == "true",
            int(configuration.get("chunk_size", 200)), int(configuration.get("chunk_overlap", 100)), self.length)

    def process_record(self, record):
        chunks = self.splitter.split_text(to_text(record.value()))
        n = len(chunks)
        out = []
        for i, c in enumerate(chunks):
            hs = list(record.headers()) + [Header("chunk_id", str(i)), Header("chunk_text_length", str(len(c))),
                                           Header("chunk_num_tokens", str(self.length(c))),
                                           Header("text_num_chunks", str(n))]
            out.append(SimpleRecord.copy_from(record, key=record.key(), value=c, headers=hs))
        return out


# ---------------------------------------------------------------- normaliser / document-to-json
@register_agent("text-normaliser")
class TextNormaliserAgent(SingleRecordAgentProcessor):
    def init(self, configuration):
        self.lower = str(configuration.get("make-lowercase", "true")).lower() == "true"
        self.trim = str(configuration.get("trim-spaces", "true")).lower() == "true"

    def process_record(self, record):
        t = to_text(record.value())
        if self.trim:
            t = trim_spaces(t)
        if self.lower:
            t = t.lower()
        return [SimpleRecord.copy_from(record, value=t)]


def trim_spaces(s: str) -> str:
    """TextNormaliserAgent.trimSpaces: the same replacement chain, in order -- tabs to a
    space, space runs to one, one pass of triple newlines to double, (space + blank line)
    runs to one, (space + newline) runs to a newline, newline + space to a newline, trim."""
    s = re.sub(r"\t+", " ", s)
    s = re.sub(r" +", " ", s)
    s = s.replace("\n\n\n", "\n\n")
    s = re.sub(r"( \n\n)+", " \n\n", s)
    s = re.sub(r"( \n)+", "\n", s)
    s = s.replace("\n ", "\n")
    return s.strip(_JAVA_TRIM)   # String.trim: code points <= U+0020 only


_JAVA_TRIM = "".join(chr(c) for c in range(33))


@register_agent("document-to-json")
class DocumentToJsonAgent(SingleRecordAgentProcessor):
    def init(self, configuration):
        self.field = configuration.get("text-field", "text")
        self.copy_props = str(configuration.get("copy-properties", "true")).lower() == "true"

    def process_record(self, record):
        # DocumentToJsonAgent.java: the value becomes the JSON TEXT of {text-field: text,
        # header: value...} (compact, as Jackson writes it); byte header values as UTF-8 text
        out = {self.field: to_text(record.value())}
        if self.copy_props:
            for h in record.headers():
                v = h.value
                out[h.key] = v.decode("utf-8", errors="replace") if isinstance(v, (bytes, bytearray)) else v
        return [SimpleRecord.copy_from(record, value=json.dumps(out, separators=(",", ":"), ensure_ascii=False))]


# ---------------------------------------------------------------- extraction
class _HTMLText(html.parser.HTMLParser):
    SKIP = {"script", "style", "head", "noscript"}
    BLOCK = {"p", "div", "br", "li", "h1", "h2", "h3", "h4", "h5", "h6", "tr", "section", "article", "pre"}

    def __init__(self):
        super().__init__(convert_charrefs=True)
        self.parts: List[str] = []
        self.skip = 0

    def handle_starttag(self, tag, attrs):
        if tag in self.SKIP:
            self.skip += 1
        elif tag in self.BLOCK:
            self.parts.append("\n")

    def handle_endtag(self, tag):
        if tag in self.SKIP and self.skip:
            self.skip -= 1
        elif tag in self.BLOCK:
            self.parts.append("\n")

    def handle_data(self, data):
        if not self.skip:
            self.parts.append(data)


def html_to_text(s: str) -> str:
    p = _HTMLText()
    p.feed(s)
    t = "".join(p.parts)
    t = re.sub(r"[ \t\r]+", " ", t)
    return re.sub(r"\n\s*\n+", "\n\n", t).strip()


def _xml_text(data: bytes) -> str:
    s = data.decode("utf-8", errors="replace")
    s = re.sub(r"</w:p>|</a:p>|</text:p>|<w:br/>", "\n", s)
    s = re.sub(r"<[^>]+>", "", s)
    return html.unescape(s)


_PDF_ESC = {ord("n"): "\n", ord("r"): "\r", ord("t"): "\t", ord("b"): "\b", ord("f"): "\f"}
_PDF_DELIM = b"()<>[]{}/%"


def _pdf_bytes_to_str(raw: bytes) -> str:
    if raw[:2] == b"\xfe\xff":                      # UTF-16BE with BOM (PDF text strings)
        return raw[2:].decode("utf-16-be", errors="replace")
    return raw.decode("latin-1")


def _pdf_literal(buf: bytes, i: int):
    """Literal string starting after '(' at i: balanced parentheses, backslash escapes
    (\\n \\r \\t \\b \\f \\( \\) \\\\, octal \\ddd, line continuation).  Returns (bytes, next i)."""
    out = bytearray()
    depth = 1
    n = len(buf)
    while i < n:
        c = buf[i]
        if c == 0x5C:                                   # backslash
            i += 1
            if i >= n:
                break
            e = buf[i]
            if e in _PDF_ESC:
                out += _PDF_ESC[e].encode("latin-1")
                i += 1
            elif 0x30 <= e <= 0x37:
                j = i
                while j < n and j < i + 3 and 0x30 <= buf[j] <= 0x37:
                    j += 1
                out.append(int(buf[i:j], 8) & 0xFF)
                i = j
            elif e in (0x0D, 0x0A):                      # escaped end of line: continuation
                i += 1
                if e == 0x0D and i < n and buf[i] == 0x0A:
                    i += 1
            else:
                out.append(e)
                i += 1
            continue
        if c == 0x28:
            depth += 1
        elif c == 0x29:
            depth -= 1
            if depth == 0:
                return bytes(out), i + 1
        out.append(c)
        i += 1
    return bytes(out), i


def _pdf_tokens(buf: bytes):
    """Content-stream tokens: ('s', bytes) strings, ('n', float) numbers, ('[', None),
    (']', None) and ('op', name) operators; dictionaries / names are skipped."""
    i, n = 0, len(buf)
    while i < n:
        c = buf[i]
        if c in b" \t\r\n\x0c\x00":
            i += 1
        elif c == 0x25:                                 # comment
            while i < n and buf[i] not in b"\r\n":
                i += 1
        elif c == 0x28:
            sv, i = _pdf_literal(buf, i + 1)
            yield "s", sv
        elif c == 0x3C and i + 1 < n and buf[i + 1] == 0x3C:   # << dict >>: skip markers
            i += 2
        elif c == 0x3E and i + 1 < n and buf[i + 1] == 0x3E:
            i += 2
        elif c == 0x3C:                                 # <hex string>
            j = buf.find(b">", i)
            j = n if j < 0 else j
            hx = re.sub(rb"[^0-9A-Fa-f]", b"", buf[i + 1:j])
            if len(hx) % 2:
                hx += b"0"
            yield "s", bytes.fromhex(hx.decode())
            i = j + 1
        elif c == 0x5B:
            yield "[", None
            i += 1
        elif c == 0x5D:
            yield "]", None
            i += 1
        elif c == 0x2F:                                 # /Name
            i += 1
            while i < n and buf[i] not in b" \t\r\n\x0c" and buf[i] not in _PDF_DELIM:
                i += 1
        else:
            j = i
            while j < n and buf[j] not in b" \t\r\n\x0c\x00" and buf[j] not in _PDF_DELIM:
                j += 1
            if j == i:
                i += 1
                continue
            tok = buf[i:j]
            i = j
            try:
                yield "n", float(tok)
            except ValueError:
                yield "op", tok.decode("latin-1")


def _pdf_content_text(buf: bytes) -> str:
    """Text of one content stream: Tj / TJ / ' / " show strings; TJ displacements below
    -200 thousandths of an em become a space; Td / TD / T* / ' / " / ET start a new line
    (Td with a zero vertical move continues the line)."""
    out: List[str] = []
    stack: list = []
    arr = None
    for kind, v in _pdf_tokens(buf):
        if kind == "[":
            arr = []
        elif kind == "]":
            stack.append(("a", arr or []))
            arr = None
        elif arr is not None:
            arr.append((kind, v))
        elif kind != "op":
            stack.append((kind, v))
        else:
            if v == "Tj" and stack and stack[-1][0] == "s":
                out.append(_pdf_bytes_to_str(stack[-1][1]))
            elif v == "TJ" and stack and stack[-1][0] == "a":
                for k2, v2 in stack[-1][1]:
                    if k2 == "s":
                        out.append(_pdf_bytes_to_str(v2))
                    elif k2 == "n" and v2 < -200:
                        out.append(" ")
            elif v in ("'", '"') and stack and stack[-1][0] == "s":
                out.append("\n" + _pdf_bytes_to_str(stack[-1][1]))
            elif v in ("T*", "ET"):
                out.append("\n")
            elif v in ("Td", "TD") and len(stack) >= 2 and stack[-1][0] == "n":
                out.append("\n" if stack[-1][1] != 0 else " ")
            stack.clear()
    return "".join(out)


def _pdf_text(data: bytes) -> str:
    """PDF text through the object-level extractor (agents/pdf.py: page tree, object
    streams, font encodings and ToUnicode CMaps); a damaged file it cannot parse falls
    back to the literal strings of every text-drawing stream."""
    from .pdf import pdf_text
    try:
        text = pdf_text(data)
        if text:
            return text
    except DecompressionBombError:
        raise
    except Exception:  # noqa: BLE001 - damaged structure: the stream scan below
        pass
    return _pdf_text_streams(data)


def _pdf_text_streams(data: bytes) -> str:
    out = []
    for m in re.finditer(rb"stream\r?\n(.*?)\r?\nendstream", data, re.S):
        raw = m.group(1)
        try:
            raw = bounded_inflate(raw)
        except zlib.error:
            pass
        if b"BT" not in raw:                            # images, fonts, xref streams
            continue
        out.append(_pdf_content_text(raw))
        out.append("\n")
    text = "".join(out)
    text = re.sub(r"[ \t]+\n", "\n", text)
    return re.sub(r"\n{2,}", "\n", text).strip()


def _email_text(s: str) -> str:
    """RFC 822 / MIME message: subject + the text/plain parts (text/html parts as text
    when there is no plain part)."""
    import email
    from email import policy
    msg = email.message_from_string(s, policy=policy.default)
    plain, htmls = [], []
    for part in (msg.walk() if msg.is_multipart() else [msg]):
        ctype = part.get_content_type()
        if part.get_content_maintype() == "multipart" or part.get_filename():
            continue
        try:
            body = part.get_content()
        except Exception:  # noqa: BLE001 - undecodable part
            continue
        if not isinstance(body, str):
            continue
        if ctype == "text/plain":
            plain.append(body.strip())
        elif ctype == "text/html":
            htmls.append(html_to_text(body).strip())
    head = str(msg.get("subject") or "").strip()
    return "\n".join([head] + (plain or htmls) if head else (plain or htmls)).strip()


_EMAIL_HEAD = re.compile(r"^(?:(?:From|To|Subject|Date|Message-ID|MIME-Version|Received|Return-Path)"
                         r":[^\n]*\n)+", re.I)


# Decompression-bomb guard.  Tika's AutoDetectParser runs under SecureContentHandler,
# which rejects a document whose output exceeds 100x its input once past 1M characters
# (the reference's TikaTextExtractorAgent.java:41 inherits it).  Every inflate here --
# gzip wrappers, zip members (OOXML / ODF / EPUB), PDF FlateDecode streams -- goes
# through a bounded streaming decompressor with the same shape of limit plus a hard
# ceiling, and nested gzip wrappers are limited in depth.
MAX_EXPANSION_RATIO = 100
MIN_EXPANSION_ALLOWANCE = 1 << 20
MAX_INFLATED_BYTES = 256 << 20
MAX_NESTING = 3


class DecompressionBombError(ValueError):
    pass


def inflate_limit(compressed_len: int) -> int:
    return min(MAX_INFLATED_BYTES, max(MIN_EXPANSION_ALLOWANCE, MAX_EXPANSION_RATIO * compressed_len))


def bounded_inflate(data: bytes, wbits: int = zlib.MAX_WBITS, limit: Optional[int] = None) -> bytes:
    """zlib / raw-deflate / gzip (wbits 15 / -15 / 31) decompression that stops with
    DecompressionBombError once the output passes ``limit`` (default inflate_limit)."""
    limit = inflate_limit(len(data)) if limit is None else limit
    d = zlib.decompressobj(wbits)
    out = bytearray()
    buf = data
    while buf:
        chunk = d.decompress(buf, limit + 1 - len(out))
        out += chunk
        if len(out) > limit:
            raise DecompressionBombError(f"decompressed size exceeds {limit} bytes "
                                         f"({len(data)} compressed)")
        buf = d.unconsumed_tail
        if d.eof:
            # gzip members may be concatenated: continue with the next one
            rest = d.unused_data
            if wbits == 31 and rest[:2] == b"\x1f\x8b":
                d = zlib.decompressobj(wbits)
                buf = rest
                continue
            break
        if not chunk and not buf:
            break
    out += d.flush()
    if len(out) > limit:
        raise DecompressionBombError(f"decompressed size exceeds {limit} bytes")
    return bytes(out)


def _zip_read(z: "zipfile.ZipFile", name: str, budget: List[int]) -> bytes:
    """One zip member, refused when its declared size or its actual inflated size would
    exceed the document's remaining budget (shared by all members)."""
    info = z.getinfo(name)
    if info.file_size > budget[0]:
        raise DecompressionBombError(f"zip member {name}: {info.file_size} bytes over the budget")
    out = bytearray()
    with z.open(info) as f:
        while True:
            chunk = f.read(1 << 16)
            if not chunk:
                break
            out += chunk
            if len(out) > budget[0]:
                raise DecompressionBombError(f"zip member {name} inflates past the budget")
    budget[0] -= len(out)
    return bytes(out)


def extract_text(data: Any, _depth: int = 0) -> str:
    """Text of a document (the reference runs Tika's AutoDetectParser,
    TikaTextExtractorAgent.java:36-58): PDF, OOXML (docx / pptx / xlsx), ODF, EPUB, RTF,
    HTML / XHTML / XML, MIME e-mail, gzip-wrapped content and UTF-8/16 text (BOMs).
    Compressed content is inflated under the bomb guard above (DecompressionBombError)."""
    if isinstance(data, str):
        s = data.lstrip("\ufeff").lstrip()
        if s[:1] == "<" and re.search(r"<(html|body|p|div)\b", s[:2000], re.I):
            return html_to_text(s)
        if s[:5] == "<?xml" or (s[:1] == "<" and re.match(r"<[A-Za-z_][\w:.-]*[\s>/]", s)):
            # generic XML: element text, elements separated by a space
            t = html.unescape(re.sub(r"<[^>]+>", "", re.sub(r"</[^>]+>", " ", s)))
            return re.sub(r"[ \t]+", " ", re.sub(r"\s*\n\s*", "\n", t)).strip()
        if _EMAIL_HEAD.match(s):
            return _email_text(s)
        return s
    if not isinstance(data, (bytes, bytearray)):
        return to_text(data)
    b = bytes(data)
    if b[:4] == b"%PDF":
        return _pdf_text(b)
    if b[:2] == b"\x1f\x8b":
        if _depth >= MAX_NESTING:
            raise DecompressionBombError(f"gzip nested deeper than {MAX_NESTING} levels")
        try:
            inner = bounded_inflate(b, 31)
        except zlib.error:
            inner = None
        if inner is not None:
            return extract_text(inner, _depth + 1)
    if b[:2] in (b"\xff\xfe", b"\xfe\xff"):
        return extract_text(b.decode("utf-16"), _depth)
    if b[:2] == b"PK":
        try:
            with zipfile.ZipFile(io.BytesIO(b)) as z:
                names = z.namelist()
                budget = [inflate_limit(len(b))]
                if "META-INF/container.xml" in names and any(n.endswith((".xhtml", ".html", ".htm")) for n in names):
                    # EPUB: the content documents in spine order (the OPF manifest / spine)
                    return _epub_text(z, names, budget)
                parts = [n for n in names if n in ("word/document.xml", "content.xml")]
                parts += sorted(n for n in names if re.match(r"ppt/slides/slide\d+\.xml", n))
                parts += [n for n in names if n == "xl/sharedStrings.xml"]
                return "\n".join(_xml_text(_zip_read(z, n, budget)) for n in parts).strip()
        except zipfile.BadZipFile:
            pass
    if b[:5] == b"{\\rtf":
        s = b.decode("latin-1")
        s = re.sub(r"\\[a-z]+-?\d* ?|[{}]", "", s)
        return s.strip()
    s = b.decode("utf-8", errors="replace")
    return extract_text(s, _depth)


def _epub_text(z: "zipfile.ZipFile", names, budget: List[int]) -> str:
    import posixpath
    order = []
    try:
        cont = _zip_read(z, "META-INF/container.xml", budget).decode("utf-8", "replace")
        opf = re.search(r'full-path="([^"]+)"', cont).group(1)
        o = _zip_read(z, opf, budget).decode("utf-8", "replace")
        base = posixpath.dirname(opf)
        items = dict(re.findall(r'<item\b[^>]*?id="([^"]+)"[^>]*?href="([^"]+)"', o))
        items.update({i: h for h, i in re.findall(r'<item\b[^>]*?href="([^"]+)"[^>]*?id="([^"]+)"', o)})
        for idref in re.findall(r'<itemref\b[^>]*?idref="([^"]+)"', o):
            if idref in items:
                order.append(posixpath.normpath(posixpath.join(base, items[idref])))
    except DecompressionBombError:
        raise
    except Exception:  # noqa: BLE001 - no usable OPF: document order
        order = []
    if not order:
        order = sorted(n for n in names if n.endswith((".xhtml", ".html", ".htm")))
    return "\n".join(html_to_text(_zip_read(z, n, budget).decode("utf-8", "replace")).strip()
                     for n in order if n in names).strip()


@register_agent("text-extractor")
class TextExtractorAgent(SingleRecordAgentProcessor):
    def process_record(self, record):
        return [SimpleRecord.copy_from(record, value=extract_text(record.value()))]


# ---------------------------------------------------------------- language detection
# Character n-gram profiles (the technique of Tika's LanguageIdentifier, which the
# reference uses: TXT/LanguageDetectorAgent.java:30-76, over Tika's legacy profile set of
# 18 languages + en): each language's profile is the 1-3-gram distribution of original
# generic training prose (agents/langid_data.py -- none of it is a test sentence); a text
# is scored by the naive-Bayes log-likelihood of its n-grams under each profile (add-k
# smoothed) and labelled with the best language, or "unknown" when it has no letters.
from .langid_data import SAMPLES as _SAMPLES  # noqa: E402
_WORD = re.compile(r"[^\W\d_]+", re.UNICODE)


def _ngrams(text: str):
    for w in _WORD.findall(text.lower()):
        p = f" {w} "
        for n in (1, 2, 3):
            for i in range(len(p) - n + 1):
                g = p[i:i + n]
                if g.strip():
                    yield g


def _build_profiles():
    import math
    from collections import Counter
    profs = {}
    for lang, txt in _SAMPLES.items():
        c = Counter(_ngrams(txt))
        tot = {n: sum(v for g, v in c.items() if len(g) == n) for n in (1, 2, 3)}
        vocab = {n: sum(1 for g in c if len(g) == n) for n in (1, 2, 3)}
        # add-0.5 smoothing per n-gram order; unseen grams get the floor log-prob
        profs[lang] = ({g: math.log((v + 0.5) / (tot[len(g)] + 0.5 * (vocab[len(g)] + 1))) for g, v in c.items()},
                       {n: math.log(0.5 / (tot[n] + 0.5 * (vocab[n] + 1))) for n in (1, 2, 3)})
    return profs


_PROFILES = _build_profiles()


def detect_language(text: str) -> str:
    grams = list(_ngrams(text))
    if not grams:
        return "unknown"
    best, score = "unknown", float("-inf")
    for lang, (lp, floor) in _PROFILES.items():
        sc = sum(lp.get(g, floor[len(g)]) * len(g) for g in grams)   # longer grams weigh more
        if sc > score:
            best, score = lang, sc
    return best


@register_agent("language-detector")
class LanguageDetectorAgent(SingleRecordAgentProcessor):
    def init(self, configuration):
        self.prop = configuration.get("property", "language")
        al = configuration.get("allowedLanguages") or []
        self.allowed = set(al if isinstance(al, list) else [a.strip() for a in str(al).split(",") if a.strip()])

    def process_record(self, record):
        lang = detect_language(to_text(record.value()))
        if self.allowed and lang not in self.allowed:
            return []
        return [SimpleRecord.with_headers(record, [Header(self.prop, lang)])]
