"""SourceRecordTracker (RT/agent/SourceRecordTracker.java:26-117).

Maps every sink record to its source record, counts the sink writes still pending per
source record, and commits source records STRICTLY in source order: the longest prefix
of tracked source records whose fan-out is complete.
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from typing import List

from ..api.record import Record, SourceRecordAndResult


class SourceRecordTracker:
    def __init__(self, source):
        self.source = source
        self._sink_to_source = {}          # id(sink record) -> source record
        self._remaining = {}               # id(source record) -> remaining sink writes
        self._ordered: "OrderedDict[int, Record]" = OrderedDict()
        self._lock = threading.Lock()

    def track(self, results: List[SourceRecordAndResult]) -> None:
        with self._lock:
            for r in results:
                src = r.source_record
                self._ordered[id(src)] = src
                recs = r.result_records or []
                self._remaining[id(src)] = len(recs)
                for s in recs:
                    self._sink_to_source[id(s)] = src

    def commit(self, sink_records: List[Record]) -> None:
        with self._lock:
            for rec in sink_records:
                src = self._sink_to_source.pop(id(rec), None)
                if src is not None:
                    self._remaining[id(src)] -= 1
            to_commit = []
            for k, src in self._ordered.items():
                rem = self._remaining.get(k)
                if rem is None:
                    raise RuntimeError(f"No sink records for source record {src}. Something went wrong")
                if rem <= 0:
                    to_commit.append(src)
                else:
                    break
            for src in to_commit:
                self._ordered.pop(id(src), None)
                self._remaining.pop(id(src), None)
        if to_commit:
            self.source.commit(to_commit)

    def pending(self) -> int:
        with self._lock:
            return len(self._ordered)
