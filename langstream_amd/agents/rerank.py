"""re-rank agent: MMR with BM25 relevance and cosine diversity.

Parity: AIA/ai/langstream/ai/agents/rerank/ReRankAgent.java:67-343 -- config field,
output-field, algorithm (MMR|none), max (100), lambda (0.5), k1 (1.5), b (0.75),
query-text, query-embeddings (parsed, unused like the reference), text-field,
embeddings-field; whitespace tokens; BM25 over the REMAINING documents each round;
diversity = mean cosine to already-selected documents; greedy selection of ``max``.

Difference in cost, not result: the pairwise cosine matrix is computed once
(vectorised, [N,d]x[d,N]) instead of re-computing cosine for every (candidate,
selected) pair every round.
"""
from __future__ import annotations

import math
import re
from collections import Counter
from typing import Any, Dict, List

import numpy as np

from ..api.agent import SingleRecordAgentProcessor
from ..runtime.registry import register_agent
from .genai.el import eval_expression
from .genai.mutable import MutableRecord
from ..utils.fastjson import f32_matrix


def _tok(t: str) -> List[str]:
    return [x for x in t.split() if x] if t.strip() else ([""] if t == "" else [])


def bm25_scores(texts: List[str], query: str, k1: float, b: float) -> List[float]:
    n = len(texts)
    if n == 0:
        return []
    docs = [t.split() if t.strip() else [] for t in texts]
    # Java String.split("\\s+") keeps a leading empty token for leading whitespace
    docs = [([""] + d if t[:1].isspace() else d) for t, d in zip(texts, docs)]
    avgdl = sum(len(d) for d in docs) / n
    tfs = [Counter(d) for d in docs]
    q = query.split()
    if query[:1].isspace():
        q = [""] + q
    out = []
    for i in range(n):
        dl = len(docs[i])
        s = 0.0
        for term in q:
            tf = tfs[i].get(term, 0)
            df = sum(1 for c in tfs if term in c)
            idf = math.log((n - df + 0.5) / (df + 0.5) + 1.0)
            denom = tf + k1 * (1 - b + b * (dl / avgdl)) if avgdl else 1.0
            s += idf * (tf * (k1 + 1) / denom) if denom else 0.0
        out.append(s)
    return out


def _java_split(t: str) -> List[str]:
    d = t.split()
    return [""] + d if t[:1].isspace() else (d if d else [""] if t == "" else d)


def mmr(docs: List[Any], texts: List[str], embs: np.ndarray, query: str, max_: int, lam: float, k1: float,
        b: float) -> List[Any]:
    """Vectorised MMR: same scores as :func:`bm25_scores` + mean-cosine diversity, with
    the term-frequency matrix and the pairwise cosine matrix computed once."""
    n = len(docs)
    if n == 0:
        return []
    norms = np.linalg.norm(embs, axis=1)
    safe = np.where(norms == 0, 1.0, norms)
    unit = embs / safe[:, None]
    cos = unit @ unit.T
    cos[norms == 0, :] = 0
    cos[:, norms == 0] = 0
    toks = [t.split() if t.strip() else [] for t in texts]
    toks = [([""] + d if t[:1].isspace() else d) for t, d in zip(texts, toks)]
    q = query.split()
    if query[:1].isspace():
        q = [""] + q
    qc = Counter(q)
    terms = list(qc)
    qw = np.array([qc[t] for t in terms], dtype=np.float64)
    tf = np.array([[c.get(t, 0) for t in terms] for c in map(Counter, toks)], dtype=np.float64).reshape(n, len(terms))
    dl = np.array([len(d) for d in toks], dtype=np.float64)
    remaining = np.ones(n, dtype=bool)
    selected: List[int] = []
    div_sum = np.zeros(n, dtype=np.float64)
    while len(selected) < max_ and len(selected) < n:
        idx = np.flatnonzero(remaining)
        N = len(idx)
        sub = tf[idx]
        dli = dl[idx]
        avgdl = dli.mean()
        df = np.count_nonzero(sub, axis=0)
        idf = np.log((N - df + 0.5) / (df + 0.5) + 1.0) * qw
        norm = (k1 * (1 - b) + (k1 * b / avgdl) * dli) if avgdl else np.full(N, k1)
        denom = sub + norm[:, None]
        with np.errstate(divide="ignore", invalid="ignore"):
            part = np.where(denom > 0, sub * (k1 + 1) / denom, 0.0)
        rel = part @ idf
        div = div_sum[idx] / len(selected) if selected else np.zeros(N)
        score = lam * rel - (1 - lam) * div
        best = int(idx[int(np.argmax(score))])
        selected.append(best)
        remaining[best] = False
        div_sum += cos[:, best]
    return [docs[i] for i in selected]


@register_agent("re-rank")
class ReRankAgent(SingleRecordAgentProcessor):
    def init(self, configuration: Dict[str, Any]) -> None:
        def req(k):
            v = configuration.get(k)
            if v is None or str(v).strip() == "":
                raise ValueError(f"Missing required field '{k}' in re-rank agent")
            return v
        self.field = req("field")
        self.output_field = req("output-field")
        self.algorithm = str(configuration.get("algorithm", "none"))
        if self.algorithm not in ("MMR", "none"):
            raise ValueError(f"unsupported algorithm {self.algorithm}")
        self.query_field = configuration.get("query-text", "")
        self.query_emb_field = configuration.get("query-embeddings", "")
        self.text_field = configuration.get("text-field", "")
        self.emb_field = configuration.get("embeddings-field", "")
        self.max = int(configuration.get("max", 100))
        self.lam = float(configuration.get("lambda", 0.5))
        self.k1 = float(configuration.get("k1", 1.5))
        self.b = float(configuration.get("b", 0.75))

    @staticmethod
    def _getter(expr: str):
        """``record.<name>`` fields read directly; other expressions through the EL."""
        m = re.fullmatch(r"\s*record\.([A-Za-z_][A-Za-z0-9_]*)\s*", expr or "")
        if m:
            name = m.group(1)
            return lambda d: d.get(name) if isinstance(d, dict) else eval_expression(expr, {"record": d})
        return lambda d: eval_expression(expr, {"record": d})

    def process_record(self, record):
        mr = MutableRecord.from_record(record)
        ctx = mr.el_context()
        docs = eval_expression(self.field, ctx) or []
        query = eval_expression(self.query_field, ctx) if self.query_field else None
        if self.algorithm == "none" or not query:
            result = list(docs)
        else:
            texts, embs = [], []
            tget, eget = self._getter(self.text_field), self._getter(self.emb_field)
            for d in docs:
                t = tget(d)
                e = eget(d)
                if e is None:
                    raise ValueError(f"Embeddings are null in record: {d}")
                if t is None:
                    raise ValueError(f"Text is null in record: {d}")
                texts.append(str(t))
                embs.append(e)
            try:   # one native conversion of the whole [docs, dim] list (78 vs 480 us, 20 x 384)
                arr = f32_matrix(embs) if docs else np.zeros((0, 1), np.float32)
            except (TypeError, ValueError):   # ragged / non-numeric entries: per-element float()
                arr = np.asarray([[float(x) for x in e] for e in embs], dtype=np.float32).reshape(len(docs), -1)
            result = mmr(list(docs), texts, arr if docs else np.zeros((0, 1), np.float32), str(query), self.max,
                         self.lam, self.k1, self.b)
        mr.set_result_field(result, self.output_field)
        out = mr.to_record()
        return [out] if out is not None else []
