"""Error policy (RT/agent/StandardErrorsHandler.java:26-72, ErrorsHandler.java).

A GLOBAL failure counter: while below ``retries`` -> RETRY; afterwards SKIP for
``skip``, FAIL for ``fail`` and ``dead-letter``.  ``fail_processing_on_permanent_errors``
is true only for ``fail`` (dead-letter routes the record to the DLQ and continues).
"""
from __future__ import annotations

import enum
import logging
import threading
from typing import Any, Dict, Optional

log = logging.getLogger(__name__)


class Outcome(enum.Enum):
    SKIP = "SKIP"
    RETRY = "RETRY"
    FAIL = "FAIL"


class StandardErrorsHandler:
    def __init__(self, configuration: Optional[Dict[str, Any]] = None):
        cfg = configuration or {}
        self.retries = int(cfg.get("retries", 0) or 0)
        self.on_failure = str(cfg.get("onFailure", cfg.get("on-failure", "fail")) or "fail")
        self._failures = 0
        self._lock = threading.Lock()

    def handle_errors(self, source_record, error: BaseException) -> Outcome:
        with self._lock:
            self._failures += 1
            n = self._failures
        log.info("Handling error %r for source record, errors count %d (max retries %d)", error, n, self.retries)
        if n >= self.retries:
            return Outcome.SKIP if self.on_failure == "skip" else Outcome.FAIL
        return Outcome.RETRY

    def fail_processing_on_permanent_errors(self) -> bool:
        return self.on_failure not in ("skip", "dead-letter")


class PermanentFailureException(Exception):
    def __init__(self, cause: BaseException):
        super().__init__(str(cause))
        self.__cause__ = cause
