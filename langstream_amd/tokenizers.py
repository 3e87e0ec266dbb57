"""Tokenizers over the native C++ implementations (``native/tokenizer.cpp``).

* :class:`BPETokenizer` -- byte-level BPE.  Loads an HF ``tokenizer.json`` (BPE model)
  or a tiktoken rank file when one is available; otherwise builds a deterministic,
  self-contained vocabulary by training BPE on a built-in English corpus and padding to
  the model's vocab size with filler words below 256 top special tokens, the Llama-3
  layout, so sampled ids decode to text (this environment has no model
  hub; token ids are exact-size and lossless, merges are not the official ones --
  "parity unpinned" for exact token counts).
* :class:`WordPieceTokenizer` -- BERT WordPiece (``vocab.txt`` or synthetic).
* :func:`cl100k_counter` -- token counter used by ``text-splitter``'s
  ``length_function: cl100k_base`` (reference: TXT/TiktokenLengthFunction.java:21-44).
"""
from __future__ import annotations

import functools
import json
import os
import random
from typing import Iterable, List, Optional, Sequence

from .native import lib

_WORDS = """
the of and to in is you that it he was for on are as with his they at be this have from or one had by word but
not what all were we when your can said there use an each which she do how their if will up other about out many
then them these so some her would make like him into time has look two more write go see number no way could people
my than first water been call who oil its now find long down day did get come made may part over new sound take only
little work know place year live me back give most very after thing our just name good sentence man think say great
where help through much before line right too mean old any same tell boy follow came want show also around form three
small set put end does another well large must big even such because turn here why ask went men read need land
different home us move try kind hand picture again change off play spell air away animal house point page letter
mother answer found study still learn should america world high every near add food between own below country plant
last school father keep tree never start city earth eye light thought head under story saw left few while along might
close something seem next hard open example begin life always those both paper together got group often run important
until children side feet car mile night walk white sea began grow took river four carry state once book hear stop
without second later miss idea enough eat face watch far indian really almost let above girl sometimes mountain cut
young talk soon list song being leave family it's stream pipeline agent topic record gateway model embedding vector
database query document text chunk token streaming kafka pulsar application deploy tenant secret resource compute
completion chat question answer prompt context retrieval search similarity cosine index collection table schema
language python java kubernetes cluster node replica partition offset commit producer consumer reader message event
GPU kernel memory bandwidth latency throughput batch decode prefill attention layer transformer encoder decoder
""".split()


@functools.lru_cache(maxsize=4)
def builtin_corpus(n_sentences: int = 4000, seed: int = 7) -> List[str]:
    rng = random.Random(seed)
    out = []
    punct = [".", ".", ".", "?", "!", ",", ";", ":"]
    for i in range(n_sentences):
        n = rng.randint(4, 18)
        ws = [rng.choice(_WORDS) for _ in range(n)]
        if rng.random() < 0.5:
            ws[0] = ws[0].capitalize()
        s = " ".join(ws) + rng.choice(punct)
        if rng.random() < 0.15:
            s += f" {rng.randint(0, 99999)}"
        if rng.random() < 0.1:
            s += "\n\n"
        out.append(s)
    return out


class BPETokenizer:
    def __init__(self, vocab: dict, merges: Sequence = (), specials: Optional[dict] = None,
                 bos: Optional[str] = None, eos: Sequence[str] = ()):
        self.specials = dict(specials or {})
        self._tok = lib().ByteBPE(list(vocab.items()), list(merges), list(self.specials.items()))
        self.vocab_size = max([len(vocab)] + [i + 1 for i in self.specials.values()])
        self.bos_id = self.specials.get(bos) if bos else None
        self.eos_ids = [self.specials[e] for e in eos if e in self.specials]

    # --- constructors
    @staticmethod
    def synthetic(vocab_size: int = 128256, num_merges: int = 6000, bos: str = "<|begin_of_text|>",
                  eos: Sequence[str] = ("<|end_of_text|>", "<|eot_id|>")) -> "BPETokenizer":
        return _synthetic_bpe(vocab_size, num_merges, bos, tuple(eos))

    @staticmethod
    def from_hf_json(path: str) -> "BPETokenizer":
        with open(path, encoding="utf-8") as f:
            spec = json.load(f)
        model = spec["model"]
        if model.get("type") != "BPE":
            raise ValueError("only BPE tokenizer.json supported here (use WordPieceTokenizer for WordPiece)")
        dec = _unicode_to_bytes()
        to_b = lambda s: bytes(dec.get(ch, ord(ch) & 0xFF) for ch in s)  # noqa: E731
        vocab = {to_b(t): i for t, i in model["vocab"].items()}
        merges = []
        for m in model.get("merges", []):
            a, b = (m.split(" ", 1) if isinstance(m, str) else m)
            merges.append((to_b(a), to_b(b)))
        specials = {t["content"]: t["id"] for t in spec.get("added_tokens", [])}
        return BPETokenizer(vocab, merges, specials)

    @staticmethod
    def from_tiktoken(path: str, specials: Optional[dict] = None) -> "BPETokenizer":
        import base64
        vocab = {}
        with open(path, "rb") as f:
            for line in f:
                if line.strip():
                    tok, rank = line.split()
                    vocab[base64.b64decode(tok)] = int(rank)
        return BPETokenizer(vocab, (), specials)

    # --- api
    def encode(self, text: str, add_bos: bool = False, allow_special: bool = True) -> List[int]:
        ids = self._tok.encode(text, allow_special)
        if add_bos and self.bos_id is not None:
            ids = [self.bos_id] + ids
        return ids

    def encode_batch(self, texts: Sequence[str], threads: int = 4) -> List[List[int]]:
        return self._tok.encode_batch(list(texts), True, threads)

    def count(self, text: str) -> int:
        return self._tok.count(text)

    def decode(self, ids: Iterable[int], skip_special: bool = True) -> str:
        return self._tok.decode_bytes(list(ids), skip_special).decode("utf-8", errors="replace")

    def decode_bytes(self, ids: Iterable[int]) -> bytes:
        return self._tok.decode_bytes(list(ids), True)

    def token_to_id(self, t: str) -> int:
        return self._tok.token_to_id(t)


def _unicode_to_bytes() -> dict:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


@functools.lru_cache(maxsize=8)
def _synthetic_bpe(vocab_size: int, num_merges: int, bos: str, eos: tuple) -> BPETokenizer:
    num_merges = max(0, min(num_merges, vocab_size - 256 - 16))  # leave room for special tokens
    merges = lib().train_bpe(builtin_corpus(), num_merges, 2)
    vocab = {bytes([b]): b for b in range(256)}
    for a, b in merges:
        t = a + b
        if t not in vocab:
            vocab[t] = len(vocab)
    if vocab_size < len(vocab):
        raise ValueError(f"vocab_size {vocab_size} smaller than trained vocab {len(vocab)}")
    # Llama-3 layout: the top 256 ids are special tokens, everything below decodes to text.
    # Ids between the trained vocab and the specials get filler words (never produced by
    # encode, no merges reach them) so randomly sampled ids stream non-empty text the way a
    # real 128K vocabulary does.
    n_special = min(256, max(0, vocab_size - len(vocab)))
    fill_to = vocab_size - n_special
    alpha = b"abcdefghijklmnopqrstuvwxyz"
    i = 0
    while len(vocab) < fill_to:
        n, w = i, b""
        while True:
            w = alpha[n % 26:n % 26 + 1] + w
            n //= 26
            if n == 0:
                break
        i += 1
        t = b" " + w
        if t not in vocab:
            vocab[t] = len(vocab)
    names = [bos, *eos, "<|start_header_id|>", "<|end_header_id|>"]
    specials = {}
    for i in range(n_special):
        name = names[i] if i < len(names) else f"<|reserved_special_token_{i}|>"
        specials[name] = len(vocab) + i
    return BPETokenizer(vocab, merges, specials, bos=bos, eos=eos)


class WordPieceTokenizer:
    def __init__(self, vocab: List[str], lower: bool = True):
        self.vocab = vocab
        self._tok = lib().WordPiece(vocab, lower, lower, "[UNK]", 100)
        self.cls_id = self._tok.token_to_id("[CLS]")
        self.sep_id = self._tok.token_to_id("[SEP]")
        self.pad_id = max(0, self._tok.token_to_id("[PAD]"))
        self.vocab_size = len(vocab)

    @staticmethod
    def from_vocab_file(path: str, lower: bool = True) -> "WordPieceTokenizer":
        with open(path, encoding="utf-8") as f:
            return WordPieceTokenizer([line.rstrip("\n") for line in f], lower)

    @staticmethod
    def synthetic(vocab_size: int = 30522) -> "WordPieceTokenizer":
        return _synthetic_wordpiece(vocab_size)

    def encode(self, text: str, max_len: int = 512, special: bool = True) -> List[int]:
        ids = self._tok.encode(text)
        if special:
            ids = [self.cls_id] + ids[: max_len - 2] + [self.sep_id]
        return ids[:max_len]

    def encode_batch(self, texts: Sequence[str], max_len: int = 512, threads: int = 8) -> List[List[int]]:
        out = self._tok.encode_batch(list(texts), threads)
        return [[self.cls_id] + ids[: max_len - 2] + [self.sep_id] for ids in out]

    def encode_batch_packed(self, texts: Sequence[str], max_len: int = 512, threads: int = 8):
        """Same tokens as ``encode_batch``, packed: (ids int32 [sum lens], lens int32 [n])."""
        return self._tok.encode_batch_packed(list(texts), max_len, self.cls_id, self.sep_id, threads)

    def decode(self, ids: Iterable[int]) -> str:
        return self._tok.decode([i for i in ids if i not in (self.cls_id, self.sep_id, self.pad_id)])


@functools.lru_cache(maxsize=4)
def _synthetic_wordpiece(vocab_size: int) -> WordPieceTokenizer:
    vocab = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    seen = set(vocab)
    chars = [chr(c) for c in range(33, 127)]
    for c in chars:
        for t in (c.lower(), "##" + c.lower()):
            if t not in seen:
                seen.add(t)
                vocab.append(t)
    for w in sorted(set(w.lower() for w in _WORDS)):
        if w not in seen:
            seen.add(w)
            vocab.append(w)
    # frequent sub-word pieces from the BPE trainer, as ## continuations
    for a, b in lib().train_bpe(builtin_corpus(), 3000, 2):
        t = (a + b).decode("utf-8", "ignore").strip().lower()
        for cand in (t, "##" + t):
            if t and cand not in seen and len(vocab) < vocab_size:
                seen.add(cand)
                vocab.append(cand)
    i = 0
    while len(vocab) < vocab_size:
        vocab.append(f"[unused{99 + i}]")
        i += 1
    return WordPieceTokenizer(vocab[:vocab_size])


@functools.lru_cache(maxsize=1)
def cl100k_counter():
    """Token counter for text-splitter ``length_function: cl100k_base``.  Uses a real
    ``cl100k_base.tiktoken`` file if LANGSTREAM_CL100K points to one, else the synthetic
    byte-level BPE (same algorithm, different merges)."""
    path = os.environ.get("LANGSTREAM_CL100K")
    tok = BPETokenizer.from_tiktoken(path) if path and os.path.exists(path) else BPETokenizer.synthetic(100277)
    return tok.count
