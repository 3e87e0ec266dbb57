"""PDF text extraction for the text-extractor agent.

The reference extracts PDF text with Tika's PDFParser (PDFBox underneath;
TikaTextExtractorAgent.java:41 -> AutoDetectParser).  What makes real-world PDFs
readable, and what this module implements:

* objects found by scanning ``N G obj`` (no trust in the xref table, which is often
  stale), plus the objects packed in **object streams** (``/Type /ObjStm``, PDF 1.5+,
  what Word and pdfTeX write by default);
* stream filters: FlateDecode (under the bomb guard of agents/text.py), ASCIIHexDecode,
  ASCII85Decode, LZWDecode, RunLengthDecode, and filter chains;
* the page tree (``/Root /Pages /Kids``, inherited ``/Resources``) so text comes out in
  page order, content-stream arrays, and **Form XObjects** (``Do``) with their own
  resources;
* fonts: ``/ToUnicode`` CMaps (``bfchar`` / ``bfrange``, multi-byte codespaces), Type0
  composite fonts (``/Identity-H`` two-byte CIDs: Word's subset TrueType fonts),
  simple-font ``/Encoding`` names (WinAnsi, MacRoman, Standard, PDFDoc) and
  ``/Differences`` arrays with glyph names mapped to Unicode (pdfTeX's Type1 subsets:
  ``/fi``, ``/quoteright``, ``/uni2013``, accented names, ligature names ``f_f``);
* text layout: ``Td`` / ``TD`` / ``T*`` / ``Tm`` / ``'`` / ``"`` line breaks, ``TJ``
  displacements beyond -200/1000 em as word spaces.

Anything else (images, Type3 glyph procedures, encrypted files) yields no text, as a
best effort, never an exception the agent would turn into a failed record.
"""
from __future__ import annotations

import re
import unicodedata
from typing import Any, Dict, List, Optional, Tuple

__all__ = ["pdf_text"]


class Ref:
    __slots__ = ("num", "gen")

    def __init__(self, num: int, gen: int):
        self.num, self.gen = num, gen

    def __repr__(self):
        return f"Ref({self.num},{self.gen})"


class Name(str):
    """A PDF name object (/Foo -> Name('Foo'))."""


_WS = b" \t\r\n\x0c\x00"
_DELIM = b"()<>[]{}/%"


# ------------------------------------------------------------------ object syntax
class _Lexer:
    def __init__(self, buf: bytes, pos: int = 0):
        self.buf, self.pos, self.n = buf, pos, len(buf)

    def skip_ws(self):
        b, n = self.buf, self.n
        while self.pos < n:
            c = b[self.pos]
            if c in _WS:
                self.pos += 1
            elif c == 0x25:                      # comment to end of line
                while self.pos < n and b[self.pos] not in b"\r\n":
                    self.pos += 1
            else:
                break

    def token(self) -> Tuple[str, Any]:
        """Next token: ('num', v) ('name', s) ('str', bytes) ('kw', s) ('<<',) ('>>',)
        ('[',) (']',) or ('eof', None)."""
        self.skip_ws()
        b, n = self.buf, self.n
        if self.pos >= n:
            return "eof", None
        c = b[self.pos]
        if c == 0x2F:                            # /Name with #xx escapes
            j = self.pos + 1
            while j < n and b[j] not in _WS and b[j] not in _DELIM:
                j += 1
            raw = b[self.pos + 1:j]
            self.pos = j
            if b"#" in raw:
                raw = re.sub(rb"#([0-9A-Fa-f]{2})", lambda m: bytes([int(m.group(1), 16)]), raw)
            return "name", Name(raw.decode("latin-1"))
        if c == 0x28:
            s, self.pos = _literal(b, self.pos + 1)
            return "str", s
        if c == 0x3C:
            if self.pos + 1 < n and b[self.pos + 1] == 0x3C:
                self.pos += 2
                return "<<", None
            j = b.find(b">", self.pos)
            j = n if j < 0 else j
            hx = re.sub(rb"[^0-9A-Fa-f]", b"", b[self.pos + 1:j])
            if len(hx) % 2:
                hx += b"0"
            self.pos = j + 1
            return "str", bytes.fromhex(hx.decode())
        if c == 0x3E:
            self.pos += 2 if self.pos + 1 < n and b[self.pos + 1] == 0x3E else 1
            return ">>", None
        if c == 0x5B:
            self.pos += 1
            return "[", None
        if c == 0x5D:
            self.pos += 1
            return "]", None
        if c in b"{}":
            self.pos += 1
            return "kw", chr(c)
        j = self.pos
        while j < n and b[j] not in _WS and b[j] not in _DELIM:
            j += 1
        if j == self.pos:
            self.pos += 1
            return "kw", chr(c)
        tok = b[self.pos:j]
        self.pos = j
        try:
            return "num", (float(tok) if b"." in tok else int(tok))
        except ValueError:
            return "kw", tok.decode("latin-1")

    def parse(self, depth: int = 0) -> Any:
        """One object (refs ``N G R`` resolved syntactically into Ref)."""
        if depth > 64:
            raise ValueError("PDF object nesting too deep")
        kind, v = self.token()
        if kind == "num":
            save = self.pos
            k2, v2 = self.token()
            if k2 == "num" and isinstance(v, int) and isinstance(v2, int):
                k3, v3 = self.token()
                if k3 == "kw" and v3 == "R":
                    return Ref(v, v2)
            self.pos = save
            return v
        if kind in ("name", "str"):
            return v
        if kind == "[":
            arr = []
            while True:
                self.skip_ws()
                if self.pos >= self.n:
                    return arr
                if self.buf[self.pos] == 0x5D:
                    self.pos += 1
                    return arr
                arr.append(self.parse(depth + 1))
        if kind == "<<":
            d: Dict[str, Any] = {}
            while True:
                k, key = self.token()
                if k in (">>", "eof"):
                    return d
                if k != "name":
                    continue
                d[key] = self.parse(depth + 1)
        if kind == "kw":
            return {"true": True, "false": False, "null": None}.get(v, v)
        return None


_ESC = {ord("n"): b"\n", ord("r"): b"\r", ord("t"): b"\t", ord("b"): b"\b", ord("f"): b"\f"}


def _literal(buf: bytes, i: int) -> Tuple[bytes, int]:
    """Literal string starting after '(' at i: balanced parentheses, backslash escapes,
    octal \\ddd, line continuation.  Returns (bytes, next i)."""
    out = bytearray()
    depth, n = 1, len(buf)
    while i < n:
        c = buf[i]
        if c == 0x5C:
            i += 1
            if i >= n:
                break
            e = buf[i]
            if e in _ESC:
                out += _ESC[e]
                i += 1
            elif 0x30 <= e <= 0x37:
                j = i
                while j < n and j < i + 3 and 0x30 <= buf[j] <= 0x37:
                    j += 1
                out.append(int(buf[i:j], 8) & 0xFF)
                i = j
            elif e in (0x0D, 0x0A):
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


# ------------------------------------------------------------------ filters
def _ascii_hex(data: bytes) -> bytes:
    s = re.sub(rb"[^0-9A-Fa-f]", b"", data.split(b">")[0])
    if len(s) % 2:
        s += b"0"
    return bytes.fromhex(s.decode())


def _ascii85(data: bytes) -> bytes:
    s = re.sub(rb"\s", b"", data)
    if s.startswith(b"<~"):
        s = s[2:]
    s = s.split(b"~>")[0]
    out = bytearray()
    grp: List[int] = []
    for c in s:
        if c == ord("z") and not grp:
            out += b"\0\0\0\0"
            continue
        if not 33 <= c <= 117:
            continue
        grp.append(c - 33)
        if len(grp) == 5:
            v = 0
            for d in grp:
                v = v * 85 + d
            out += (v & 0xFFFFFFFF).to_bytes(4, "big")
            grp = []
    if grp:
        k = len(grp)
        grp += [84] * (5 - k)
        v = 0
        for d in grp:
            v = v * 85 + d
        out += (v & 0xFFFFFFFF).to_bytes(4, "big")[: k - 1]
    return bytes(out)


def _lzw(data: bytes, early: int = 1, limit: int = 1 << 28) -> bytes:
    out = bytearray()
    table = [bytes([i]) for i in range(256)] + [b"", b""]
    width, bitbuf, nbits, prev = 9, 0, 0, None
    for byte in data:
        bitbuf = (bitbuf << 8) | byte
        nbits += 8
        while nbits >= width:
            nbits -= width
            code = (bitbuf >> nbits) & ((1 << width) - 1)
            if code == 256:                       # clear
                table = table[:258]
                width, prev = 9, None
                continue
            if code == 257:                       # EOD
                return bytes(out)
            if code < len(table):
                entry = table[code]
                if prev is not None:
                    table.append(prev + entry[:1])
            elif prev is not None:
                entry = prev + prev[:1]
                table.append(entry)
            else:
                return bytes(out)
            out += entry
            if len(out) > limit:
                from .text import DecompressionBombError
                raise DecompressionBombError("LZW stream inflates past the limit")
            prev = entry
            if len(table) + early >= (1 << width) and width < 12:
                width += 1
    return bytes(out)


def _run_length(data: bytes) -> bytes:
    out = bytearray()
    i, n = 0, len(data)
    while i < n:
        L = data[i]
        if L == 128:
            break
        if L < 128:
            out += data[i + 1:i + 2 + L]
            i += L + 2
        else:
            out += data[i + 1:i + 2] * (257 - L)
            i += 2
    return bytes(out)


def _png_unpredict(data: bytes, columns: int, colors: int = 1, bpc: int = 8) -> bytes:
    bpp = max(1, colors * bpc // 8)
    row_len = (columns * colors * bpc + 7) // 8
    out = bytearray()
    prev = bytearray(row_len)
    i = 0
    while i < len(data):
        ft = data[i]
        row = bytearray(data[i + 1:i + 1 + row_len])
        i += 1 + row_len
        for x in range(len(row)):
            a = row[x - bpp] if x >= bpp else 0
            b = prev[x] if x < len(prev) else 0
            c = prev[x - bpp] if x >= bpp else 0
            if ft == 1:
                row[x] = (row[x] + a) & 0xFF
            elif ft == 2:
                row[x] = (row[x] + b) & 0xFF
            elif ft == 3:
                row[x] = (row[x] + ((a + b) >> 1)) & 0xFF
            elif ft == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                row[x] = (row[x] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)) & 0xFF
        out += row
        prev = row
    return bytes(out)


# ------------------------------------------------------------------ encodings / glyph names
_DIACRITICS = {"acute": "ACUTE", "grave": "GRAVE", "circumflex": "CIRCUMFLEX", "dieresis": "DIAERESIS",
               "tilde": "TILDE", "ring": "RING ABOVE", "cedilla": "CEDILLA", "caron": "CARON",
               "macron": "MACRON", "breve": "BREVE", "ogonek": "OGONEK", "dotaccent": "DOT ABOVE",
               "hungarumlaut": "DOUBLE ACUTE", "commaaccent": "CEDILLA"}
_GLYPHS = {
    "space": " ", "exclam": "!", "quotedbl": '"', "numbersign": "#", "dollar": "$", "percent": "%",
    "ampersand": "&", "quotesingle": "'", "quoteright": "’", "quoteleft": "‘", "parenleft": "(",
    "parenright": ")", "asterisk": "*", "plus": "+", "comma": ",", "hyphen": "-", "period": ".",
    "slash": "/", "zero": "0", "one": "1", "two": "2", "three": "3", "four": "4", "five": "5", "six": "6",
    "seven": "7", "eight": "8", "nine": "9", "colon": ":", "semicolon": ";", "less": "<", "equal": "=",
    "greater": ">", "question": "?", "at": "@", "bracketleft": "[", "backslash": "\\", "bracketright": "]",
    "asciicircum": "^", "underscore": "_", "grave": "`", "braceleft": "{", "bar": "|", "braceright": "}",
    "asciitilde": "~", "bullet": "•", "endash": "–", "emdash": "—", "quotedblleft": "“",
    "quotedblright": "”", "quotesinglbase": "‚", "quotedblbase": "„", "ellipsis": "…",
    "fi": "fi", "fl": "fl", "ff": "ff", "ffi": "ffi", "ffl": "ffl", "dagger": "†",
    "daggerdbl": "‡", "trademark": "™", "copyright": "©", "registered": "®",
    "degree": "°", "plusminus": "±", "multiply": "×", "divide": "÷", "minus": "−",
    "section": "§", "paragraph": "¶", "periodcentered": "·", "germandbls": "ß",
    "ae": "æ", "AE": "Æ", "oe": "œ", "OE": "Œ", "oslash": "ø", "Oslash": "Ø",
    "lslash": "ł", "Lslash": "Ł", "dotlessi": "ı", "exclamdown": "¡",
    "questiondown": "¿", "guillemotleft": "«", "guillemotright": "»",
    "guilsinglleft": "‹", "guilsinglright": "›", "cent": "¢", "sterling": "£",
    "yen": "¥", "florin": "ƒ", "currency": "¤", "Euro": "€", "euro": "€",
    "nbspace": " ", "sfthyphen": "­", "ordfeminine": "ª", "ordmasculine": "º",
    "mu": "µ", "perthousand": "‰", "fraction": "⁄", "logicalnot": "¬",
    "brokenbar": "¦", "onehalf": "½", "onequarter": "¼", "threequarters": "¾",
    "onesuperior": "¹", "twosuperior": "²", "threesuperior": "³", "eth": "ð",
    "Eth": "Ð", "thorn": "þ", "Thorn": "Þ", "dieresis": "¨", "acute": "´",
    "cedilla": "¸", "macron": "¯", "circumflex": "ˆ", "tilde": "˜", "caron": "ˇ",
    "breve": "˘", "dotaccent": "˙", "ring": "˚", "ogonek": "˛",
    "hungarumlaut": "˝", "arrowright": "→", "arrowleft": "←", "infinity": "∞",
    "lessequal": "≤", "greaterequal": "≥", "notequal": "≠", "approxequal": "≈",
    "summation": "∑", "product": "∏", "radical": "√", "integral": "∫",
    "partialdiff": "∂", "Delta": "Δ", "Omega": "Ω", "pi": "π", "alpha": "α",
    "beta": "β", "gamma": "γ", "delta": "δ", "epsilon": "ε", "lambda": "λ",
    "sigma": "σ", "theta": "θ", "dotlessj": "ȷ", "visiblespace": "␣",
}


def glyph_to_unicode(name: str) -> str:
    """Adobe Glyph List naming rules (the subset real fonts use): explicit names,
    uniXXXX[XXXX...], uXXXX[XX], suffixes (.sc, .alt), ligature components (f_f_i), single
    letters and digits, accented Latin letters built from the diacritic suffix."""
    if not name:
        return ""
    base = name.split(".", 1)[0]
    if "_" in base and base not in _GLYPHS:
        return "".join(glyph_to_unicode(p) for p in base.split("_"))
    if base in _GLYPHS:
        return _GLYPHS[base]
    m = re.fullmatch(r"uni((?:[0-9A-F]{4})+)", base)
    if m:
        h = m.group(1)
        return "".join(chr(int(h[i:i + 4], 16)) for i in range(0, len(h), 4))
    m = re.fullmatch(r"u([0-9A-F]{4,6})", base)
    if m:
        return chr(int(m.group(1), 16))
    if len(base) == 1 and base.isalnum():
        return base
    for suf, uname in _DIACRITICS.items():
        if base.endswith(suf) and len(base) == len(suf) + 1 and base[0].isalpha():
            case = "CAPITAL" if base[0].isupper() else "SMALL"
            try:
                return unicodedata.lookup(f"LATIN {case} LETTER {base[0].upper()} WITH {uname}")
            except KeyError:
                break
    m = re.fullmatch(r"(?:g|cid|glyph)(\d+)", base)
    if m:
        return ""                                  # anonymous glyph ids carry no text
    return ""


def _std_encoding() -> List[str]:
    t = [chr(i) if 32 <= i < 127 else "" for i in range(256)]
    t[0x27], t[0x60] = "’", "‘"
    hi = {0xA1: "¡", 0xA2: "¢", 0xA3: "£", 0xA4: "⁄", 0xA5: "¥", 0xA6: "ƒ",
          0xA7: "§", 0xA8: "¤", 0xA9: "'", 0xAA: "“", 0xAB: "«", 0xAC: "‹",
          0xAD: "›", 0xAE: "fi", 0xAF: "fl", 0xB1: "–", 0xB2: "†", 0xB3: "‡",
          0xB4: "·", 0xB6: "¶", 0xB7: "•", 0xB8: "‚", 0xB9: "„", 0xBA: "”",
          0xBB: "»", 0xBC: "…", 0xBD: "‰", 0xBF: "¿", 0xC1: "`", 0xC2: "´",
          0xC3: "ˆ", 0xC4: "˜", 0xC5: "¯", 0xC6: "˘", 0xC7: "˙", 0xC8: "¨",
          0xCA: "˚", 0xCB: "¸", 0xCD: "˝", 0xCE: "˛", 0xCF: "ˇ", 0xD0: "—",
          0xE1: "Æ", 0xE3: "ª", 0xE8: "Ł", 0xE9: "Ø", 0xEA: "Œ", 0xEB: "º",
          0xF1: "æ", 0xF5: "ı", 0xF8: "ł", 0xF9: "ø", 0xFA: "œ", 0xFB: "ß"}
    for k, v in hi.items():
        t[k] = v
    return t


def _codec_table(codec: str) -> List[str]:
    t = []
    for i in range(256):
        try:
            t.append(bytes([i]).decode(codec))
        except UnicodeDecodeError:
            t.append("")
    return t


def _pdfdoc_table() -> List[str]:
    t = _codec_table("latin-1")
    extra = {0x80: "•", 0x81: "†", 0x82: "‡", 0x83: "…", 0x84: "—", 0x85: "–",
             0x86: "ƒ", 0x87: "⁄", 0x88: "‹", 0x89: "›", 0x8A: "−", 0x8B: "‰",
             0x8C: "„", 0x8D: "“", 0x8E: "”", 0x8F: "‘", 0x90: "’", 0x91: "‚",
             0x92: "™", 0x93: "fi", 0x94: "fl", 0x95: "Ł", 0x96: "Œ", 0x97: "Š",
             0x98: "Ÿ", 0x99: "Ž", 0x9A: "ı", 0x9B: "ł", 0x9C: "œ", 0x9D: "š",
             0x9E: "ž", 0xA0: "€"}
    for k, v in extra.items():
        t[k] = v
    return t


_ENCODINGS: Dict[str, List[str]] = {}


def _encoding(name: str) -> List[str]:
    if not _ENCODINGS:
        win = _codec_table("cp1252")
        _ENCODINGS.update({"WinAnsiEncoding": win, "MacRomanEncoding": _codec_table("mac_roman"),
                           "StandardEncoding": _std_encoding(), "PDFDocEncoding": _pdfdoc_table(),
                           "MacExpertEncoding": _std_encoding()})
    return _ENCODINGS.get(name, _ENCODINGS["StandardEncoding"])


def pdfdoc_string(raw: bytes) -> str:
    """A PDF text string (metadata, annotations): UTF-16BE with BOM, UTF-8 with BOM, or
    PDFDocEncoding."""
    if raw[:2] == b"\xfe\xff":
        return raw[2:].decode("utf-16-be", errors="replace")
    if raw[:3] == b"\xef\xbb\xbf":
        return raw[3:].decode("utf-8", errors="replace")
    t = _encoding("PDFDocEncoding")
    return "".join(t[c] for c in raw)


# ------------------------------------------------------------------ CMaps
class _CMap:
    """ToUnicode CMap: code ranges (byte lengths) + code -> text."""

    def __init__(self):
        self.ranges: List[Tuple[int, bytes, bytes]] = []     # (nbytes, lo, hi)
        self.map: Dict[bytes, str] = {}

    @staticmethod
    def _utf16(raw: bytes) -> str:
        if len(raw) % 2:
            raw = b"\0" + raw
        return raw.decode("utf-16-be", errors="replace")

    @classmethod
    def parse(cls, data: bytes) -> "_CMap":
        cm = cls()
        lx = _Lexer(data)
        stack: List[Any] = []
        mode = None
        while True:
            kind, v = lx.token()
            if kind == "eof":
                break
            if kind == "[":
                lx.pos -= 1
                stack.append(lx.parse())
                continue
            if kind in ("str", "num", "name"):
                stack.append(v)
                continue
            if kind != "kw":
                continue
            if v in ("begincodespacerange", "beginbfchar", "beginbfrange", "begincidrange", "begincidchar"):
                mode = v
                stack.clear()
            elif v == "endcodespacerange":
                for i in range(0, len(stack) - 1, 2):
                    lo, hi = stack[i], stack[i + 1]
                    if isinstance(lo, bytes) and isinstance(hi, bytes):
                        cm.ranges.append((len(lo), lo, hi))
                mode = None
            elif v == "endbfchar":
                for i in range(0, len(stack) - 1, 2):
                    src, dst = stack[i], stack[i + 1]
                    if isinstance(src, bytes):
                        cm.map[src] = cls._utf16(dst) if isinstance(dst, bytes) else \
                            glyph_to_unicode(dst) if isinstance(dst, str) else ""
                mode = None
            elif v == "endbfrange":
                for i in range(0, len(stack) - 2, 3):
                    lo, hi, dst = stack[i], stack[i + 1], stack[i + 2]
                    if not (isinstance(lo, bytes) and isinstance(hi, bytes)):
                        continue
                    a, b = int.from_bytes(lo, "big"), int.from_bytes(hi, "big")
                    if b - a > 65535:
                        continue
                    for k, code in enumerate(range(a, b + 1)):
                        key = code.to_bytes(len(lo), "big")
                        if isinstance(dst, list):
                            if k < len(dst) and isinstance(dst[k], bytes):
                                cm.map[key] = cls._utf16(dst[k])
                        elif isinstance(dst, bytes) and dst:
                            # increment the last byte of the destination (PDF 32000 9.10.3)
                            base = int.from_bytes(dst, "big") + k
                            cm.map[key] = cls._utf16(base.to_bytes(len(dst), "big"))
                mode = None
            elif v in ("endcidrange", "endcidchar"):
                mode = None
        _ = mode
        return cm

    def code_lengths(self) -> List[int]:
        return sorted({r[0] for r in self.ranges}) or sorted({len(k) for k in self.map}) or [1]

    def split(self, raw: bytes) -> List[bytes]:
        """Cut a show-string into codes using the codespace ranges (PDF 32000 9.7.6.2)."""
        if not self.ranges:
            ln = self.code_lengths()[0]
            return [raw[i:i + ln] for i in range(0, len(raw), ln)]
        out, i, n = [], 0, len(raw)
        while i < n:
            for ln, lo, hi in sorted(self.ranges, key=lambda r: r[0]):
                c = raw[i:i + ln]
                if len(c) == ln and all(lo[k] <= c[k] <= hi[k] for k in range(ln)):
                    out.append(c)
                    i += ln
                    break
            else:
                out.append(raw[i:i + 1])
                i += 1
        return out


# ------------------------------------------------------------------ the document
class _Font:
    def __init__(self, doc: "_Doc", d: Dict[str, Any]):
        self.composite = d.get("Subtype") == "Type0"
        self.cmap: Optional[_CMap] = None
        tu = doc.resolve(d.get("ToUnicode"))
        if isinstance(tu, tuple):
            try:
                self.cmap = _CMap.parse(doc.stream_data(tu))
            except Exception:  # noqa: BLE001 - unusable CMap: fall back to the encoding
                self.cmap = None
        self.table: List[str] = _encoding("StandardEncoding")
        enc = doc.resolve(d.get("Encoding"))
        if not self.composite:
            base = None
            diffs = None
            if isinstance(enc, str):
                base = enc
            elif isinstance(enc, dict):
                base = doc.resolve(enc.get("BaseEncoding"))
                diffs = doc.resolve(enc.get("Differences"))
            if base is None and d.get("Subtype") == "TrueType":
                base = "WinAnsiEncoding"
            if isinstance(base, str):
                self.table = list(_encoding(base))
            if isinstance(diffs, list):
                self.table = list(self.table)
                code = 0
                for item in diffs:
                    item = doc.resolve(item)
                    if isinstance(item, (int, float)):
                        code = int(item)
                    elif isinstance(item, str):
                        if 0 <= code < 256:
                            self.table[code] = glyph_to_unicode(item)
                        code += 1
        self.identity = self.composite and isinstance(enc, str) and enc.startswith("Identity")

    def decode(self, raw: bytes) -> str:
        if self.cmap is not None:
            codes = self.cmap.split(raw) if (self.composite or self.cmap.ranges) else [bytes([c]) for c in raw]
            out = []
            for c in codes:
                t = self.cmap.map.get(c)
                if t is None:
                    if self.composite:
                        continue
                    t = self.table[c[0]] if len(c) == 1 else ""
                out.append(t)
            return "".join(out)
        if self.composite:
            # no ToUnicode: Identity-H CIDs of fonts whose CIDs are Unicode (some generators)
            if len(raw) % 2 == 0:
                s = raw.decode("utf-16-be", errors="ignore")
                return "".join(ch for ch in s if ch.isprintable() or ch in "\n\t")
            return ""
        return "".join(self.table[c] for c in raw)


class _Doc:
    def __init__(self, data: bytes):
        from .text import inflate_limit
        self.data = data
        self.objs: Dict[int, Any] = {}
        # file offset of the definition each object number currently resolves to: a later
        # definition (an incremental update appended to the file) supersedes an earlier one,
        # whether either sits at the top level or inside an object stream
        self._pos: Dict[int, int] = {}
        self.streams: Dict[int, Tuple[Dict[str, Any], int, int]] = {}
        self._fonts: Dict[int, _Font] = {}
        # ONE decompression budget for the whole document (Tika-style 100x of the file,
        # at least 1 MiB), shared by every FlateDecode / LZW stream like text._zip_read's
        self._budget = inflate_limit(len(data))
        self._decoded: Dict[int, bytes] = {}
        self._scan()

    # -- object table
    def _scan(self):
        data = self.data
        for m in re.finditer(rb"(?<![0-9])(\d+)\s+(\d+)\s+obj\b", data):
            num = int(m.group(1))
            lx = _Lexer(data, m.end())
            try:
                obj = lx.parse()
            except Exception:  # noqa: BLE001 - damaged object: skip it
                continue
            lx.skip_ws()
            if isinstance(obj, dict) and data.startswith(b"stream", lx.pos):
                s = lx.pos + 6
                if data[s:s + 2] == b"\r\n":
                    s += 2
                elif data[s:s + 1] in (b"\n", b"\r"):
                    s += 1
                ln = obj.get("Length")
                e = -1
                if isinstance(ln, int) and 0 <= ln and data.startswith(b"endstream", self._skip_eol(s + ln)):
                    e = s + ln
                if e < 0:
                    e = data.find(b"endstream", s)
                    if e < 0:
                        continue
                    while e > s and data[e - 1] in b"\r\n":
                        e -= 1
                self.objs[num] = ("stream", num)
                self.streams[num] = (obj, s, e)
            else:
                self.objs[num] = obj
            self._pos[num] = m.start()
        # objects inside object streams, in file order: an entry replaces a definition
        # that comes EARLIER in the file (an update appended an object stream), never a
        # later one (an update appended a top-level object)
        for num, (d, _, _) in sorted(self.streams.items(), key=lambda kv: self._pos.get(kv[0], 0)):
            if d.get("Type") == "ObjStm":
                try:
                    self._load_objstm(num, d)
                except Exception:  # noqa: BLE001 - damaged object stream
                    continue

    def _skip_eol(self, i: int) -> int:
        while i < len(self.data) and self.data[i] in b"\r\n \t":
            i += 1
        return i

    def _load_objstm(self, num: int, d: Dict[str, Any]):
        raw = self.stream_data(("stream", num))
        n = int(self.resolve(d.get("N", 0)) or 0)
        first = int(self.resolve(d.get("First", 0)) or 0)
        lx = _Lexer(raw)
        pairs = []
        for _ in range(n):
            k1, onum = lx.token()
            k2, off = lx.token()
            if k1 != "num" or k2 != "num":
                break
            pairs.append((int(onum), int(off)))
        here = self._pos.get(num, 0)
        for onum, off in pairs:
            if onum == num or self._pos.get(onum, -1) > here:
                continue
            try:
                self.objs[onum] = _Lexer(raw, first + off).parse()
            except Exception:  # noqa: BLE001
                continue
            self._pos[onum] = here

    def resolve(self, v: Any, depth: int = 0) -> Any:
        while isinstance(v, Ref) and depth < 32:
            v = self.objs.get(v.num)
            depth += 1
        return v

    def stream_dict(self, v: Any) -> Optional[Dict[str, Any]]:
        v = self.resolve(v)
        if isinstance(v, tuple) and v and v[0] == "stream" and v[1] in self.streams:
            return self.streams[v[1]][0]
        return None

    def _spend(self, n: int):
        from .text import DecompressionBombError
        self._budget -= n
        if self._budget < 0:
            raise DecompressionBombError("PDF streams inflate past the document's budget")

    def stream_data(self, v: Any) -> bytes:
        v = self.resolve(v)
        if not (isinstance(v, tuple) and v[0] == "stream"):
            return b""
        num = v[1]
        if num not in self._decoded:
            self._decoded[num] = self._decode(num)
        return self._decoded[num]

    def _decode(self, num: int) -> bytes:
        from .text import bounded_inflate
        d, s, e = self.streams[num]
        raw = self.data[s:e]
        filters = self.resolve(d.get("Filter"))
        parms = self.resolve(d.get("DecodeParms"))
        if not isinstance(filters, list):
            filters = [filters] if filters else []
        if not isinstance(parms, list):
            parms = [parms] * len(filters)
        for f, p in zip(filters, parms):
            f = self.resolve(f)
            p = self.resolve(p) or {}
            if f in ("FlateDecode", "Fl"):
                try:
                    raw = bounded_inflate(raw, limit=max(0, self._budget))
                except Exception as ex:  # noqa: BLE001 - truncated streams: salvage what inflates
                    from .text import DecompressionBombError
                    if isinstance(ex, DecompressionBombError):
                        raise
                    raw = _inflate_partial(raw, max(0, self._budget))
                self._spend(len(raw))
                pred = int(self.resolve(p.get("Predictor", 1)) or 1) if isinstance(p, dict) else 1
                if pred >= 10:
                    raw = _png_unpredict(raw, int(self.resolve(p.get("Columns", 1)) or 1),
                                         int(self.resolve(p.get("Colors", 1)) or 1),
                                         int(self.resolve(p.get("BitsPerComponent", 8)) or 8))
            elif f in ("ASCIIHexDecode", "AHx"):
                raw = _ascii_hex(raw)
            elif f in ("ASCII85Decode", "A85"):
                raw = _ascii85(raw)
            elif f in ("LZWDecode", "LZW"):
                early = int(self.resolve(p.get("EarlyChange", 1))) if isinstance(p, dict) else 1
                raw = _lzw(raw, early, max(0, self._budget))
                self._spend(len(raw))
            elif f in ("RunLengthDecode", "RL"):
                raw = _run_length(raw)
            else:                                  # image codecs, Crypt: no text
                return b""
        return raw

    def font(self, v: Any) -> Optional[_Font]:
        key = v.num if isinstance(v, Ref) else id(v)
        if key not in self._fonts:
            d = self.resolve(v)
            self._fonts[key] = _Font(self, d) if isinstance(d, dict) else None
        return self._fonts[key]

    # -- pages
    def pages(self) -> List[Tuple[Any, Dict[str, Any]]]:
        """(contents, resources) per page in page order; [] when there is no page tree."""
        root = None
        for m in re.finditer(rb"/Root\s+(\d+)\s+(\d+)\s+R", self.data):
            root = self.resolve(Ref(int(m.group(1)), int(m.group(2))))
        if root is None:
            for num, (d, _, _) in self.streams.items():
                if d.get("Type") == "XRef" and isinstance(d.get("Root"), Ref):
                    root = self.resolve(d["Root"])
        if not isinstance(root, dict):
            cands = [o for o in self.objs.values() if isinstance(o, dict) and o.get("Type") == "Catalog"]
            root = cands[-1] if cands else None
        if not isinstance(root, dict):
            return []
        out: List[Tuple[Any, Dict[str, Any]]] = []
        seen = set()

        def walk(node: Any, res: Any, depth: int):
            key = node.num if isinstance(node, Ref) else None
            if depth > 64 or (key is not None and key in seen):
                return
            if key is not None:
                seen.add(key)
            n = self.resolve(node)
            if not isinstance(n, dict):
                return
            r = n.get("Resources", res)
            if n.get("Type") == "Pages" or "Kids" in n:
                for kid in self.resolve(n.get("Kids")) or []:
                    walk(kid, r, depth + 1)
            else:
                out.append((n.get("Contents"), self.resolve(r) or {}))

        walk(root.get("Pages"), None, 0)
        return out


def _inflate_partial(raw: bytes, limit: int) -> bytes:
    import zlib
    d = zlib.decompressobj()
    try:
        return d.decompress(raw, limit)
    except zlib.error:
        return b""


# ------------------------------------------------------------------ content streams
class _Text:
    def __init__(self, doc: _Doc):
        self.doc = doc
        self.out: List[str] = []
        self.depth = 0

    def newline(self):
        if self.out and not self.out[-1].endswith("\n"):
            self.out.append("\n")

    def run(self, content: bytes, resources: Dict[str, Any]):
        if self.depth > 8:
            return
        self.depth += 1
        doc = self.doc
        fonts = doc.resolve(resources.get("Font")) if isinstance(resources, dict) else None
        xobjs = doc.resolve(resources.get("XObject")) if isinstance(resources, dict) else None
        font: Optional[_Font] = None
        lx = _Lexer(content)
        stack: List[Any] = []
        last_y: Optional[float] = None
        while True:
            kind, v = lx.token()
            if kind == "eof":
                break
            if kind == "[":
                lx.pos -= 1
                stack.append(lx.parse())
                continue
            if kind == "<<":
                lx.pos -= 2
                stack.append(lx.parse())
                continue
            if kind in ("num", "str", "name"):
                stack.append(v)
                continue
            if kind != "kw":
                continue
            op = v
            if op == "BI":                         # inline image: skip to EI
                j = content.find(b"EI", lx.pos)
                while j >= 0 and not (j + 2 >= len(content) or content[j + 2] in _WS):
                    j = content.find(b"EI", j + 2)
                lx.pos = len(content) if j < 0 else j + 2
            elif op == "Tf" and len(stack) >= 2 and isinstance(stack[-2], str):
                f = fonts.get(stack[-2]) if isinstance(fonts, dict) else None
                font = doc.font(f) if f is not None else None
            elif op == "Tj" and stack and isinstance(stack[-1], bytes):
                self.out.append(self.show(font, stack[-1]))
            elif op in ("'", '"') and stack and isinstance(stack[-1], bytes):
                self.newline()
                self.out.append(self.show(font, stack[-1]))
            elif op == "TJ" and stack and isinstance(stack[-1], list):
                for item in stack[-1]:
                    if isinstance(item, bytes):
                        self.out.append(self.show(font, item))
                    elif isinstance(item, (int, float)) and item < -200:
                        self.out.append(" ")
            elif op in ("Td", "TD") and len(stack) >= 2:
                ty = stack[-1]
                if isinstance(ty, (int, float)) and ty != 0:
                    self.newline()
                elif self.out and not self.out[-1].endswith((" ", "\n")):
                    self.out.append(" ")
            elif op == "Tm" and len(stack) >= 6:
                y = stack[-1]
                if isinstance(y, (int, float)):
                    if last_y is not None and abs(y - last_y) > 0.01:
                        self.newline()
                    last_y = y
            elif op == "T*":
                self.newline()
            elif op == "ET":
                self.newline()
            elif op == "Do" and stack and isinstance(stack[-1], str) and isinstance(xobjs, dict):
                xo = xobjs.get(stack[-1])
                sd = doc.stream_dict(xo)
                if sd is not None and sd.get("Subtype") == "Form":
                    res = doc.resolve(sd.get("Resources")) or resources
                    self.run(doc.stream_data(xo), res)
            stack.clear()
        self.depth -= 1

    @staticmethod
    def show(font: Optional[_Font], raw: bytes) -> str:
        if font is None:
            return raw.decode("latin-1")
        return font.decode(raw)


def pdf_text(data: bytes) -> str:
    doc = _Doc(data)
    t = _Text(doc)
    pages = doc.pages()
    if pages:
        for contents, res in pages:
            c = doc.resolve(contents)
            parts = c if isinstance(c, list) else [contents]
            # a page's content-stream array is one stream split at arbitrary token bounds
            buf = b"\n".join(doc.stream_data(p) for p in parts if p is not None)
            t.run(buf, res if isinstance(res, dict) else {})
            t.newline()
    else:
        # no page tree (fragments, damaged files): every stream that draws text
        for num, (d, _, _) in doc.streams.items():
            if d.get("Type") in ("ObjStm", "XRef") or d.get("Subtype") in ("Image", "Type1C", "CIDFontType0C"):
                continue
            raw = doc.stream_data(("stream", num))
            if b"BT" in raw:
                t.run(raw, {})
                t.newline()
    text = "".join(t.out)
    text = re.sub(r"[ \t]+\n", "\n", text)
    text = re.sub(r"[ \t]{2,}", " ", text)
    return re.sub(r"\n{2,}", "\n", text).strip()
