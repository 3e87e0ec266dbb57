"""Helpers for user Python agents."""
from __future__ import annotations

from typing import Any, List, Optional, Tuple

from .api import Record


class SimpleRecord(Record):
    def __init__(self, value=None, key=None, headers: Optional[List[Tuple[str, Any]]] = None, origin: str = None,
                 timestamp: int = None):
        self._value = value
        self._key = key
        self._headers = list(headers or [])
        self._origin = origin
        self._timestamp = timestamp

    def key(self):
        return self._key

    def value(self):
        return self._value

    def headers(self) -> List[Tuple[str, Any]]:
        return self._headers

    def origin(self) -> str:
        return self._origin

    def timestamp(self) -> int:
        return self._timestamp

    def __str__(self):
        return (f"Record(value={self._value}, key={self._key}, origin={self._origin}, "
                f"timestamp={self._timestamp}, headers={self._headers})")

    __repr__ = __str__


class AvroValue:
    def __init__(self, schema: dict, value: Any):
        self.schema = schema
        self.value = value
