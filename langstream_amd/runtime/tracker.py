"""SourceRecordTracker (RT/agent/SourceRecordTracker.java:26-117).

Maps every sink record to its source record, counts the sink writes still pending per
source record, and commits source records STRICTLY in source order: the longest prefix
of tracked source records whose fan-out is complete.

``track`` runs on the thread that finishes processing (an embeddings batch callback)
and ``commit`` on the producer's sender thread, once per record each.  Both only append
to a deque (atomic under the GIL) and then *try* to drain: whichever thread gets the
drain lock applies every queued event, the other returns at once instead of blocking
on the lock (two threads ping-ponging one lock per record cost a GIL hand-off each
time).  A drainer re-checks the queues after releasing the lock, so nothing queued
while it held the lock is left behind.
"""
from __future__ import annotations

import threading
from collections import OrderedDict, deque
from typing import List

from ..api.record import Record, SourceRecordAndResult


class SourceRecordTracker:
    def __init__(self, source):
        self.source = source
        self._sink_to_source = {}          # id(sink record) -> source record
        self._remaining = {}               # id(source record) -> remaining sink writes
        self._ordered: "OrderedDict[int, Record]" = OrderedDict()
        self._tracked: deque = deque()     # SourceRecordAndResult not applied yet
        self._done: deque = deque()        # sink records written, not applied yet
        self._lock = threading.Lock()

    def track(self, results: List[SourceRecordAndResult]) -> None:
        self._tracked.extend(results)

    def commit(self, sink_records: List[Record]) -> None:
        self._done.extend(sink_records)
        self._drain()

    def _apply_tracked(self) -> None:
        tracked = self._tracked
        while tracked:
            r = tracked.popleft()
            src = r.source_record
            self._ordered[id(src)] = src
            recs = r.result_records or []
            self._remaining[id(src)] = len(recs)
            for s in recs:
                self._sink_to_source[id(s)] = src

    def _drain(self) -> None:
        while self._done:
            if not self._lock.acquire(blocking=False):
                return      # the holder re-checks the queue after releasing
            try:
                self._apply_tracked()
                done = self._done
                while done:
                    rec = done.popleft()
                    src = self._sink_to_source.pop(id(rec), None)
                    if src is None:
                        # tracked before it was written, but queued after our pass
                        self._apply_tracked()
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
                    # under the lock: commits reach the source in source order
                    self.source.commit(to_commit)
            finally:
                self._lock.release()

    def pending(self) -> int:
        return len(self._ordered) + len(self._tracked)
