"""Record model (parity: API/runner/code/Record.java, SimpleRecord.java:24-111,
Header.java, RecordSink.java:20-40, AgentProcessor.SourceRecordAndResult)."""
from __future__ import annotations

import json
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Iterable, List, Optional, Sequence


@dataclass(frozen=True)
class Header:
    key: str
    value: Any

    def value_as_string(self) -> Optional[str]:
        v = self.value
        if v is None:
            return None
        if isinstance(v, bytes):
            return v.decode("utf-8", errors="replace")
        if isinstance(v, str):
            return v
        if isinstance(v, (dict, list)):
            from ..utils import fastjson
            return fastjson.dumps(v)
        return str(v)


class Record:
    """A streaming record.  Identity semantics (``eq=False``): two records are the same
    only if they are the same object, like the Java runtime's maps keyed by Record."""

    __slots__ = ("_key", "_value", "_origin", "_timestamp", "_headers", "_source_ref")

    def __init__(self, key: Any = None, value: Any = None, origin: Optional[str] = None,
                 timestamp: Optional[int] = None, headers: Optional[Iterable[Header]] = None):
        self._key = key
        self._value = value
        self._origin = origin
        self._timestamp = timestamp
        self._headers = tuple(headers or ())
        self._source_ref = None  # adapter-specific (partition, offset) etc.

    def key(self) -> Any:
        return self._key

    def value(self) -> Any:
        return self._value

    def origin(self) -> Optional[str]:
        return self._origin

    def timestamp(self) -> Optional[int]:
        return self._timestamp

    def headers(self) -> Sequence[Header]:
        return self._headers

    def get_header(self, key: str) -> Optional[Header]:
        for h in self._headers:
            if h.key == key:
                return h
        return None

    def header_value(self, key: str, default=None):
        h = self.get_header(key)
        return default if h is None else h.value

    def __repr__(self) -> str:
        return (f"Record(key={self._key!r}, value={_short(self._value)}, origin={self._origin!r}, "
                f"headers={[(h.key, h.value) for h in self._headers]})")


def _short(v, n=120):
    s = repr(v)
    return s if len(s) <= n else s[:n] + "..."


class SimpleRecord(Record):
    """Builder-style record (``SimpleRecord.builder().from(r).value(x).build()``)."""

    @staticmethod
    def of(key: Any = None, value: Any = None, headers: Optional[Iterable[Header]] = None, origin=None,
           timestamp=None) -> "SimpleRecord":
        return SimpleRecord(key, value, origin, timestamp if timestamp is not None else int(time.time() * 1000),
                            headers)

    @staticmethod
    def copy_from(r: Record, **changes) -> "SimpleRecord":
        """Copy of ``r`` with the given fields replaced (key, value, origin, timestamp, headers)."""
        return SimpleRecord(
            changes.get("key", r.key()),
            changes.get("value", r.value()),
            changes.get("origin", r.origin()),
            changes.get("timestamp", r.timestamp()),
            changes.get("headers", r.headers()),
        )

    @staticmethod
    def with_headers(r: Record, extra: Iterable[Header], replace: bool = True) -> "SimpleRecord":
        extra = list(extra)
        keys = {h.key for h in extra}
        hs = [h for h in r.headers() if not (replace and h.key in keys)] + extra
        return SimpleRecord.copy_from(r, headers=hs)


@dataclass
class SourceRecordAndResult:
    source_record: Record
    result_records: Optional[List[Record]] = None
    error: Optional[BaseException] = None


RecordSink = Callable[[SourceRecordAndResult], None]
